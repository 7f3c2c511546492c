"""Per-kernel parity on the GPU: the fused dequant GEMM (bertx_test_gemm) against a numpy
fp32/f64 reference of the same op, for every weight format and epilogue."""
import ctypes

import numpy as np
import pytest

import oracle_lib

pytestmark = pytest.mark.gpu

FMTS = {0: "f32", 1: "f16", 2: "q4_0", 3: "q4_1", 8: "q8_0"}
BLOCK = {2: 18, 3: 20, 8: 34}


def weight_rows(fmt, W):
    """File-format bytes of W [N][K] and its dequantized f32 values (oracle dequantizer)."""
    N, K = W.shape
    if fmt == 0:
        return W.astype(np.float32).tobytes(), W.astype(np.float32)
    if fmt == 1:
        h = W.astype(np.float16)
        return h.tobytes(), h.astype(np.float32)
    L = oracle_lib.lib()
    rows = []
    deq = np.zeros((N, K), np.float32)
    for n in range(N):
        buf = ctypes.create_string_buffer(K // 32 * BLOCK[fmt])
        x = np.ascontiguousarray(W[n], np.float32)
        L.oracle_quantize_row(fmt, x.ctypes.data, buf, K)
        L.oracle_dequantize_row(fmt, buf, deq[n].ctypes.data, K)
        rows.append(buf.raw)
    return b"".join(rows), deq


def run_gemm(lib, fmt, W, bias, X, epi, res=None, tile_n=0):
    N, K = W.shape
    M = X.shape[0]
    wb, deq = weight_rows(fmt, W)
    xh = np.ascontiguousarray(X.astype(np.float16))
    out = np.zeros((M, N), np.float16)
    resp = None
    if epi == 2:                          # the residual stream is f16
        res = np.ascontiguousarray(res, np.float16)
        resp = res.ctypes.data
    rc = lib.bertx_test_gemm(fmt, N, K, wb, np.ascontiguousarray(bias, np.float32).ctypes.data_as(
        ctypes.POINTER(ctypes.c_float)), M, xh.ctypes.data, epi, resp, out.ctypes.data, tile_n)
    assert rc == 0
    return out.astype(np.float32), deq, xh.astype(np.float32)


@pytest.mark.parametrize("fmt", sorted(FMTS))
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("shape", [(192, 256, 300, 0), (768, 768, 512, 0), (512, 192, 700, 256),
                                   (256, 3072, 256, 128),
                                   # gemm16 (layout 1) configs: 0x1000 | 1 (8 waves 256x256),
                                   # 2 (4 waves 256x128), 3 (4 waves 128x128)
                                   (768, 768, 512, 0x1001), (2304, 768, 768, 0x1002), (448, 192, 700, 0x1003),
                                   (256, 3072, 256, 0x1001),
                                   # 0x1004: the ping-pong kernel (8 waves, 256 x 256, halves alternating)
                                   (768, 768, 512, 0x1004), (512, 3072, 768, 0x1004), (2304, 192, 256, 0x1004)])
def test_gemm_matches_numpy(lib, fmt, epi, shape):
    N, K, M, tile_n = shape
    if tile_n == 256 and epi == 2:   # gemm.hip's 256-wide tile has no residual form
        pytest.skip("the residual epilogue runs 128 wide")
    rng = np.random.default_rng(fmt * 10 + epi)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    W[:, 5] *= 20.0                       # asymmetric outliers catch transposed maps
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    X = rng.standard_normal((M, K)).astype(np.float32)
    X[7] *= 3.0
    res = rng.standard_normal((M, N)).astype(np.float16) if epi == 2 else None
    got, deq, xh = run_gemm(lib, fmt, W, bias, X, epi, res, tile_n)
    # the kernel multiplies f16 operands with f32 accumulation: reference uses f16(weights)
    wref = deq.astype(np.float16).astype(np.float64)
    acc = xh.astype(np.float64) @ wref.T + bias.astype(np.float64)
    if epi == 0:
        ref = acc
        tol = 2e-3 * np.abs(ref).max()
    elif epi == 1:
        x16 = acc.astype(np.float16).astype(np.float64)
        ref = 0.5 * x16 * (1 + np.tanh(0.7978845608028654 * x16 * (1 + 0.044715 * x16 * x16)))
        tol = 3e-3 * np.abs(ref).max()
    else:                                 # f32 sum of the f16 residual, rounded to f16
        ref = res.astype(np.float64) + acc
        tol = 2e-3 * np.abs(ref).max()
    err = np.abs(got - ref).max()
    assert err <= tol, (FMTS[fmt], epi, err, tol)
    # and the dequantized value itself is what the reference uses (f32 math)
    exact = xh.astype(np.float64) @ deq.astype(np.float64).T + bias
    if epi == 0:
        assert np.abs(got - exact).max() <= 5e-3 * np.abs(exact).max()


@pytest.mark.parametrize("N,K,M,epi", [(2304, 768, 8192, 0), (3072, 768, 8192, 1), (768, 3072, 32768, 2)])
def test_gemm_column_split_bitwise(lib, N, K, M, epi):
    """gemm16's column split (gemmz_split_kernel, chosen by the heuristic when a grid of
    256 x 128 tiles is not whole rounds of two per CU: its last columns run as 128 x 128
    tiles in the same launch) gives the bits of the unsplit 256 x 128 grid, and numpy
    within f16 rounding."""
    rng = np.random.default_rng(N + K + epi)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    X = rng.standard_normal((M, K)).astype(np.float32)
    res = rng.standard_normal((M, N)).astype(np.float16) if epi == 2 else None
    split, deq, xh = run_gemm(lib, 2, W, bias, X, epi, res, 0x1005)     # split grid
    whole, _, _ = run_gemm(lib, 2, W, bias, X, epi, res, 0x1002)        # 256 x 128 everywhere
    assert np.array_equal(split, whole)
    acc = xh.astype(np.float64) @ deq.astype(np.float16).astype(np.float64).T + bias
    if epi == 1:
        x16 = acc.astype(np.float16).astype(np.float64)
        ref = 0.5 * x16 * (1 + np.tanh(0.7978845608028654 * x16 * (1 + 0.044715 * x16 * x16)))
    elif epi == 2:
        ref = res.astype(np.float64) + acc
    else:
        ref = acc
    assert np.abs(split - ref).max() <= 3e-3 * np.abs(ref).max()


def ln_ref(y, w, b):
    """ggml_norm (eps 1e-5, mean then centred variance) * w + b (bert.cpp:1048-1056) in f64."""
    y = y.astype(np.float64)
    mean = y.mean(axis=1, keepdims=True)
    sc = 1.0 / np.sqrt(((y - mean) ** 2).mean(axis=1, keepdims=True) + 1e-5)
    return (y - mean) * sc * w + b, mean[:, 0], sc[:, 0]


@pytest.mark.parametrize("fmt", [1, 2, 3, 8])
@pytest.mark.parametrize("N,K,M,rows", [(768, 768, 512, 500), (384, 1536, 256, 256), (1024, 1024, 384, 257),
                                        (768, 3072, 256, 129)])
def test_residual_gemm_panel_layernorm(lib, fmt, N, K, M, rows):
    """Residual projection + the following LN: the panel form fused into the GEMM
    (the workgroup completing a 128-row panel normalises it) equals the separate
    LN kernel bit for bit, and both match numpy (f64) within f16 rounding."""
    rng = np.random.default_rng(fmt + N + rows)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    wb, deq = weight_rows(fmt, W)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    X = rng.standard_normal((M, K)).astype(np.float16)
    res = (rng.standard_normal((M, N)) * 2 + 0.5).astype(np.float16)
    mean = res.astype(np.float64).mean(axis=1)
    stats = np.stack([mean, 1.0 / np.sqrt(res.astype(np.float64).var(axis=1) + 1e-5)], axis=1).astype(np.float32)
    lnw, lnb, nw, nb = (rng.standard_normal(N).astype(np.float32) * s + o
                        for s, o in ((0.1, 1.0), (0.1, 0.0), (0.2, 1.0), (0.1, 0.0)))
    outs = []
    for panel in (1, 0):
        out = np.zeros((M, N), np.float16)
        xh = np.zeros((M, N), np.float16)
        st = stats.copy()
        rc = lib.bertx_test_gemm_ln(fmt, N, K, wb, bias.ctypes.data, M, rows, X.ctypes.data, res.ctypes.data,
                                    st.ctypes.data, lnw.ctypes.data, lnb.ctypes.data, nw.ctypes.data,
                                    nb.ctypes.data, out.ctypes.data, xh.ctypes.data, st.ctypes.data, panel)
        assert rc == 0, (panel, rc)
        outs.append((out, xh, st))
    (o1, x1, s1), (o0, x0, s0) = outs
    assert np.array_equal(o1.view(np.uint16), o0.view(np.uint16))
    assert np.array_equal(x1[:rows].view(np.uint16), x0[:rows].view(np.uint16))
    assert np.array_equal(s1[:rows], s0[:rows])
    assert np.array_equal(s1[rows:], stats[rows:])              # rows past `rows` untouched
    # numpy: out = LN(res) + X W^T + bias; xh = LN'(out)
    r = (res.astype(np.float64) - mean[:, None]) * stats[:, 1:2] * lnw + lnb
    ref = r + X.astype(np.float64) @ deq.astype(np.float16).astype(np.float64).T + bias
    assert np.abs(o1 - ref).max() <= 2e-3 * np.abs(ref).max()
    xref, mref, sref = ln_ref(o1[:rows].astype(np.float64), nw, nb)
    assert np.abs(x1[:rows] - xref).max() <= 4e-3 * np.abs(xref).max()
    assert np.allclose(s1[:rows, 0], mref, rtol=1e-4, atol=1e-4)
    assert np.allclose(s1[:rows, 1], sref, rtol=1e-4)


def attention_ref(qkv, cu, n_head, d):
    """f64 softmax(Q K^T / sqrt(dh)) V per (sentence, head) on the f16 inputs (bert.cpp:1018-1036)."""
    dh = d // n_head
    q, k, v = (qkv[:, i * d:(i + 1) * d].astype(np.float64) for i in range(3))
    out = np.zeros((qkv.shape[0], d))
    for b in range(len(cu) - 1):
        s0, s1 = cu[b], cu[b + 1]
        for h in range(n_head):
            c = slice(h * dh, (h + 1) * dh)
            sc = q[s0:s1, c] @ k[s0:s1, c].T / np.sqrt(dh)
            p = np.exp(sc - sc.max(axis=1, keepdims=True))
            out[s0:s1, c] = (p / p.sum(axis=1, keepdims=True)) @ v[s0:s1, c]
    return out


@pytest.mark.parametrize("variant,dh", [(0, 64), (7, 64), (8, 64), (1, 64), (2, 64), (6, 64), (-1, 64), (0, 32),
                                        (-1, 32)])
def test_attention_matches_numpy(lib, variant, dh):
    """Ragged sentences (1 .. 512 tokens, block edges), one with sharp scores whose row
    maximum moves late (exercises the deferred-max rescale of variant 2)."""
    n_head = 4
    d = n_head * dh
    lens = [1, 5, 63, 64, 65, 200, 512, 130]
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    T = int(cu[-1])
    rng = np.random.default_rng(dh + 3)
    qkv = rng.standard_normal((T, 3 * d)).astype(np.float32)
    s0, s1 = cu[7], cu[8]                 # sentence 7: large Q, and keys that grow along the sentence
    qkv[s0:s1, :d] *= 4.0
    qkv[s0:s1, d:2 * d] *= np.linspace(0.2, 3.0, s1 - s0)[:, None]
    qkv = qkv.astype(np.float16)
    out = np.zeros((T, d), np.float16)
    rc = lib.bertx_test_attention(qkv.ctypes.data, cu.ctypes.data, len(lens), n_head, d, variant, out.ctypes.data)
    assert rc == 0
    ref = attention_ref(qkv, cu, n_head, d)
    got = out.astype(np.float64)
    assert np.isfinite(got).all()
    err = np.abs(got - ref).max()
    # Q pre-scaled in f16, P rounded to f16 for the MFMA, output f16
    assert err < 6e-3 * max(1.0, np.abs(ref).max()), err
