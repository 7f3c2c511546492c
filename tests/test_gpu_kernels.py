"""Per-kernel parity on the GPU: the fused dequant GEMM (bertx_test_gemm / bertx_test_gemm_ln)
against a numpy f64 reference of the same op, for every weight format and epilogue, in the
forward's own LayerNorm-fold forms (kernels.h); the attention kernels against numpy."""
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


def run_gemm(lib, fmt, W, bias, X, epi, res=None, cfg=0):
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
        ctypes.POINTER(ctypes.c_float)), M, xh.ctypes.data, epi, resp, out.ctypes.data, cfg)
    assert rc == 0
    if cfg:                               # the config asked for is the kernel that ran
        assert lib.bertx_test_gemm_ran() == cfg
    return out.astype(np.float32), deq, xh.astype(np.float32)


_GELU_TABLE = None


def era_gelu_table():
    """The era fp16 GELU table over all 65536 f16 inputs, from the oracle (oracle_gelu)."""
    global _GELU_TABLE
    if _GELU_TABLE is None:
        L = oracle_lib.lib()
        xs = np.arange(65536, dtype=np.uint16).view(np.float16).astype(np.float32)
        _GELU_TABLE = np.array([L.oracle_gelu(float(x)) for x in xs], np.float32).astype(np.float16)
    return _GELU_TABLE


def gelu_ref(acc):
    """ggml-era GELU: tanh form on the f16-rounded input (bert.cpp:1063)."""
    x16 = acc.astype(np.float16).astype(np.float64)
    return 0.5 * x16 * (1 + np.tanh(0.7978845608028654 * x16 * (1 + 0.044715 * x16 * x16)))


@pytest.mark.parametrize("fmt", sorted(FMTS))
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("shape", [(192, 256, 300, 0), (768, 768, 512, 0), (512, 192, 700, 3),
                                   (256, 3072, 256, 3),
                                   # tile configs: 2 (4 waves 256x128), 3 (4 waves 128x128),
                                   # 4 (2 waves 64x64)
                                   (768, 768, 512, 2), (2304, 768, 768, 2), (448, 192, 700, 3),
                                   (256, 3072, 256, 2), (2304, 192, 256, 2), (384, 1536, 200, 4),
                                   (96, 768, 32, 4), (1152, 384, 64, 0),
                                   # 11: 256 x 128 with the X pieces in one burst
                                   (768, 768, 512, 11), (1152, 384, 256, 11),
                                   # 16: 64 x 64 on 4 waves, 2 along the tokens, private X rings
                                   (768, 3072, 64, 16), (2304, 768, 130, 16), (96, 768, 32, 16)])
def test_gemm_matches_numpy(lib, fmt, epi, shape):
    N, K, M, cfg = shape
    rng = np.random.default_rng(fmt * 10 + epi)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    W[:, 5] *= 20.0                       # asymmetric outliers catch transposed maps
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    X = rng.standard_normal((M, K)).astype(np.float32)
    X[7] *= 3.0
    res = rng.standard_normal((M, N)).astype(np.float16) if epi == 2 else None
    got, deq, xh = run_gemm(lib, fmt, W, bias, X, epi, res, cfg)
    # the kernel multiplies f16 operands with f32 accumulation: reference uses f16(weights)
    wref = deq.astype(np.float16).astype(np.float64)
    acc = xh.astype(np.float64) @ wref.T + bias.astype(np.float64)
    if epi == 0:
        ref = acc
        tol = 2e-3 * np.abs(ref).max()
    elif epi == 1:
        ref = gelu_ref(acc)
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


@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("N,K,M", [(1152, 384, 96), (384, 1536, 64), (96, 64, 130), (40, 32, 7)])
def test_f32_gemm_matches_numpy(lib, epi, N, K, M):
    """The f32 chain's GEMM (f32.hip, ftype 0 files: f32 x f32 as bert.cpp:995 multiplies
    them) against numpy f64: an f32 FMA chain over K, so the error is a few f32 ulps of
    sum |x w| -- far below any f16 path."""
    rng = np.random.default_rng(N + K + M + epi)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    b = rng.standard_normal(N).astype(np.float32) * 0.1
    X = rng.standard_normal((M, K)).astype(np.float32)
    R = rng.standard_normal((M, N)).astype(np.float32)
    out = np.zeros((M, N), np.float32)
    rc = lib.bertx_test_gemm_f32(N, K, W.ctypes.data, b.ctypes.data, M, X.ctypes.data, epi,
                                 R.ctypes.data if epi == 2 else None, out.ctypes.data)
    assert rc == 0
    acc = X.astype(np.float64) @ W.astype(np.float64).T + b
    mag = np.abs(X).astype(np.float64) @ np.abs(W).astype(np.float64).T + np.abs(b)
    if epi == 1:
        # the era table T(x) = f16(gelu_f32(f16(x))) exactly as the oracle builds it
        # (oracle/ggml_era.c, f32 arithmetic: for x < -3 the f32 1 + tanh cancels, so an
        # f64 formula is several f16 steps away); an f32 sum within a few f32 ulps of an
        # f16 rounding boundary may take the neighbouring input entry, and the GPU's
        # tanhf may round the output one step apart from glibc's
        table = era_gelu_table()
        x16 = acc.astype(np.float16)
        assert np.array_equal(out.astype(np.float16).astype(np.float32), out)   # f16 values, as the table holds
        got = out.astype(np.float16)
        ref = table[x16.view(np.uint16)].astype(np.float64)
        # the f32 sum is within delta = 4e-7 sum|x w| of the f64 one (near-cancelling
        # sums: many f16 steps of a subnormal result), GELU's slope is at most 1.13, and
        # the table rounds to f16 on both sides of that
        # (and both sides round that sum to an f16 input, one input step apart at most)
        delta = 4e-7 * mag
        ulp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
        ulp_in = np.spacing(np.abs(x16)).astype(np.float64)
        bad = np.abs(out - ref) > 1.2 * (delta + ulp_in) + 2 * ulp + 1e-12
        assert not bad.any(), [(acc[i, j], out[i, j], ref[i, j]) for i, j in np.argwhere(bad)[:5]]
        assert np.mean(got != ref.astype(np.float16)) < 1e-2
    else:
        ref = acc + (R if epi == 2 else 0.0)
        assert np.all(np.abs(out - ref) <= 4e-7 * (mag + np.abs(R if epi == 2 else 0.0)) + 1e-30)


@pytest.mark.parametrize("fmt", sorted(FMTS))
@pytest.mark.parametrize("cfg", [2, 3, 4, 11, 16])
def test_gemm_every_k_remainder(lib, cfg, fmt):
    """Every K-loop length from 1 to 7 K-steps (K = 64 .. 448), every epilogue, for each
    shipped tile config -- 2: 256x128 (X ring NS 2, the pieces among the MFMAs), 3: 128x128,
    4: 64x64, 11: 256x128 with the X pieces in one burst in front of the MFMAs, 16: 64x64 on 4
    waves (2 along the tokens) with wave-private X rings (no barrier in the K loop) -- so every
    remainder of the unrolled K loop (triples) and every prologue clamp runs against numpy, and
    the kernel that ran is the one asked for (bertx_test_gemm_ran).  The waits these paths rely
    on are derived, not hand-counted (gemm.hip z_waits)."""
    N = {2: 256, 3: 256, 4: 128, 11: 256, 16: 128}[cfg]
    M = 256
    for ks in range(1, 8):
        K = 64 * ks
        for epi in (0, 1, 2):
            rng = np.random.default_rng(1000 * cfg + 100 * ks + 10 * epi + fmt)
            W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
            W[:, K // 2] *= 20.0
            bias = rng.standard_normal(N).astype(np.float32) * 0.1
            X = rng.standard_normal((M, K)).astype(np.float32)
            res = rng.standard_normal((M, N)).astype(np.float16) if epi == 2 else None
            got, deq, xh = run_gemm(lib, fmt, W, bias, X, epi, res, cfg)
            acc = xh.astype(np.float64) @ deq.astype(np.float16).astype(np.float64).T + bias.astype(np.float64)
            ref = gelu_ref(acc) if epi == 1 else acc + (res.astype(np.float64) if epi == 2 else 0.0)
            tol = (3e-3 if epi == 1 else 2e-3) * np.abs(ref).max()
            err = np.abs(got - ref).max()
            assert err <= tol, (FMTS[fmt], cfg, ks, epi, err, tol)


def ln_ref(y):
    """ggml_norm statistics (eps 1e-5, mean then centred variance; bert.cpp:1048-1056) in f64."""
    y = y.astype(np.float64)
    mean = y.mean(axis=1)
    return mean, 1.0 / np.sqrt(((y - mean[:, None]) ** 2).mean(axis=1) + 1e-5)


def f32p(a):
    return None if a is None else np.ascontiguousarray(a, np.float32).ctypes.data


@pytest.mark.parametrize("fmt", [0, 1, 2, 3, 8])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("N,K,M,cfg", [(2304, 768, 512, 0), (384, 1536, 300, 3), (1024, 1024, 768, 2),
                                       (1536, 384, 96, 4), (3072, 768, 256, 16), (768, 768, 512, 11)])
def test_gemm_input_ln_fold(lib, fmt, epi, N, K, M, cfg):
    """Projection of a LayerNorm'd stream as the forward runs it (kernels.h LN fold):
    the GEMM reads z = f16(y * gamma) and the row statistics of y, and returns
    LN(y) W^T + b (then GELU for epi 1) -- numpy f64 within f16 rounding.  Rows
    carry a large mean and outlier channels (the regime where folding the mean
    out of the product could cancel)."""
    rng = np.random.default_rng(fmt * 7 + epi + N)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    wb, deq = weight_rows(fmt, W)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    y = rng.standard_normal((M, K)) * 2.0 + rng.standard_normal((M, 1)) * 3.0
    y[:, 7] += 80.0
    y[:, 300 % K] -= 150.0
    g = (1.0 + rng.standard_normal(K) * 0.3).astype(np.float32)
    g[7] = 0.3
    be = (rng.standard_normal(K) * 0.1).astype(np.float32)
    mean, r = ln_ref(y)
    stats = np.ascontiguousarray(np.stack([mean, r], axis=1), np.float32)
    z = np.ascontiguousarray((y * g).astype(np.float16))
    out = np.zeros((M, N), np.float16)
    rc = lib.bertx_test_gemm_ln(fmt, N, K, wb, f32p(bias), M, z.ctypes.data, stats.ctypes.data, f32p(g), f32p(be),
                                epi, None, None, None, None, None, out.ctypes.data, None, cfg)
    assert rc == 0
    if cfg:
        assert lib.bertx_test_gemm_ran() == cfg
    x = (y - mean[:, None]) * r[:, None] * g + be
    acc = x @ deq.astype(np.float16).astype(np.float64).T + bias
    if epi == 1:
        ref = gelu_ref(acc)
        tol = 3e-3 * np.abs(ref).max()
    else:
        ref = acc
        tol = 2e-3 * np.abs(ref).max()
    err = np.abs(out.astype(np.float64) - ref).max()
    assert err <= tol, (FMTS[fmt], epi, err, tol)


def ln_row_stats_f32(part, d):
    """ln_row_stats (device_common.h) in numpy float32, op for op (every op IEEE
    round-to-nearest; fmaf(-32, mean, s) and fmaf(q, 1/32, m) are exact scalings
    plus one rounding): part [G][M][2] -> [M][2] (mean, 1/sigma)."""
    f = np.float32
    G, M = part.shape[0], part.shape[1]
    s = np.zeros(M, f)
    for g in range(G):
        s = (s + part[g, :, 0]).astype(f)
    mean = (s / f(d)).astype(f)
    m2 = np.zeros(M, f)
    for g in range(G):
        dm = (part[g, :, 0] - (f(32) * mean).astype(f)).astype(f)
        q = (dm * dm).astype(f)
        m2 = (m2 + ((q / f(32)).astype(f) + part[g, :, 1]).astype(f)).astype(f)
    r = (f(1) / np.sqrt(((m2 / f(d)).astype(f) + f(1e-5)).astype(f)).astype(f)).astype(f)
    return np.stack([mean, r], axis=1).astype(f)


@pytest.mark.parametrize("fmt", [1, 2, 3, 8])
@pytest.mark.parametrize("epi", [0, 1])
@pytest.mark.parametrize("N,K,M,cfg", [(1152, 384, 4096, 0), (1536, 384, 200, 3), (2304, 768, 32, 0),
                                       (3072, 768, 64, 16), (768, 768, 1000, 4), (192, 64, 10, 0),
                                       (2304, 768, 1024, 3), (3072, 768, 1024, 0)])
def test_gemm_statistics_fold(lib, fmt, epi, N, K, M, cfg):
    """The statistics fold of the small-batch forward (LnFold::in_part): the GEMM
    combines the residual GEMM's per-group partials itself.  Its statistics are
    bitwise the statistics kernel's (ln_stats, the launch form) and within rounding
    of ln_row_stats restated in numpy float32, and its output is bitwise the output
    of the same GEMM given those statistics, for every fold config (3: 128-row
    tiles up to d 384, and up to d 768 where they are at most one per CU -- the
    one-workgroup-per-CU form; 4, 16: 64-row tiles up to d 768)."""
    rng = np.random.default_rng(fmt * 5 + epi + N + M)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    wb, deq = weight_rows(fmt, W)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    G = K // 32
    y = (rng.standard_normal((M, K)) * 2.0 + rng.standard_normal((M, 1)) * 3.0).astype(np.float32)
    yg = y.reshape(M, G, 32)
    sg = yg.sum(axis=2, dtype=np.float32)
    q = ((yg - (sg / 32)[:, :, None]) ** 2).sum(axis=2, dtype=np.float32)
    part = np.ascontiguousarray(np.stack([sg.T, q.T], axis=2), np.float32)      # [G][M][2]
    stats = ln_row_stats_f32(part, K)
    g = (1.0 + rng.standard_normal(K) * 0.3).astype(np.float32)
    be = (rng.standard_normal(K) * 0.1).astype(np.float32)
    z = np.ascontiguousarray((y * g).astype(np.float16))
    out = np.zeros((M, N), np.float16)
    st = np.zeros((M, 2), np.float32)
    stk = np.zeros((M, 2), np.float32)
    rc = lib.bertx_test_gemm_fold(fmt, N, K, wb, f32p(bias), M, z.ctypes.data, part.ctypes.data, f32p(g), f32p(be),
                                  epi, out.ctypes.data, st.ctypes.data, stk.ctypes.data, cfg)
    assert rc == 0, rc
    # bitwise the statistics kernel's combine of the same partials (the launch form)
    assert np.array_equal(st.view(np.uint32), stk.view(np.uint32))
    # and the restated arithmetic within the device's f32 division / square root
    assert np.allclose(st, stats, rtol=5e-7, atol=1e-12), np.abs(st - stats).max()
    stats = stk
    ref = np.zeros((M, N), np.float16)
    assert lib.bertx_test_gemm_ln(fmt, N, K, wb, f32p(bias), M, z.ctypes.data, np.ascontiguousarray(stats).ctypes.data,
                                  f32p(g), f32p(be), epi, None, None, None, None, None, ref.ctypes.data, None,
                                  cfg) == 0
    assert np.array_equal(out.view(np.uint16), ref.view(np.uint16))


@pytest.mark.parametrize("fmt", [1, 2, 3, 8])
@pytest.mark.parametrize("N,K,M,cfg", [(768, 768, 512, 0), (384, 1536, 256, 3), (1024, 1024, 384, 2),
                                       (768, 3072, 256, 0), (384, 1536, 130, 4), (768, 3072, 384, 11),
                                       (768, 3072, 64, 16), (384, 1536, 130, 16)])
def test_residual_gemm_ln_statistics(lib, fmt, N, K, M, cfg):
    """Residual projection as the forward runs it: res = f16(y * gamma) with y's
    statistics (the residual is LN(y)), y' = LN(y) + x W^T + b comes back as
    f16(y' * g_next), and y''s (mean, 1/sigma) from the epilogue's 32-feature
    partials + the statistics kernel match numpy's two-pass LN statistics."""
    rng = np.random.default_rng(fmt + N + K)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    wb, deq = weight_rows(fmt, W)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    bias[11] += 60.0                        # an outlier channel of the new stream
    X = rng.standard_normal((M, K)).astype(np.float16)
    y = rng.standard_normal((M, N)) * 2 + 0.5
    g, be, gn = (rng.standard_normal(N).astype(np.float32) * s + o for s, o in ((0.3, 1.0), (0.1, 0.0), (0.3, 1.0)))
    gn[11] = 0.3
    mean, r = ln_ref(y)
    stats = np.ascontiguousarray(np.stack([mean, r], axis=1), np.float32)
    z = np.ascontiguousarray((y * g).astype(np.float16))
    out = np.zeros((M, N), np.float16)
    st = np.zeros((M, 2), np.float32)
    rc = lib.bertx_test_gemm_ln(fmt, N, K, wb, f32p(bias), M, X.ctypes.data, None, None, None, 2, z.ctypes.data,
                                stats.ctypes.data, f32p(g), f32p(be), f32p(gn), out.ctypes.data, st.ctypes.data, cfg)
    assert rc == 0
    if cfg:
        assert lib.bertx_test_gemm_ran() == cfg
    resid = r[:, None] * z.astype(np.float64) - (r * mean)[:, None] * g + be
    y2 = resid + X.astype(np.float64) @ deq.astype(np.float16).astype(np.float64).T + bias
    ref = y2 * gn
    assert np.abs(out - ref).max() <= 2e-3 * np.abs(ref).max()
    m2, r2 = ln_ref(y2)
    assert np.allclose(st[:, 0], m2, rtol=1e-4, atol=1e-5 * np.abs(y2).max())
    assert np.allclose(st[:, 1], r2, rtol=2e-4)
    # plain residual (no LN on it, no statistics): f16(res + x W^T + b)
    out2 = np.zeros((M, N), np.float16)
    rc = lib.bertx_test_gemm_ln(fmt, N, K, wb, f32p(bias), M, X.ctypes.data, None, None, None, 2, z.ctypes.data,
                                None, None, None, None, out2.ctypes.data, None, cfg)
    assert rc == 0
    ref2 = z.astype(np.float64) + X.astype(np.float64) @ deq.astype(np.float16).astype(np.float64).T + bias
    assert np.abs(out2 - ref2).max() <= 2e-3 * np.abs(ref2).max()


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


@pytest.mark.parametrize("variant,dh", [(0, 64), (8, 64), (7, 64), (-1, 64), (0, 32), (-1, 32)])
def test_attention_matches_numpy(lib, variant, dh):
    """Ragged sentences (1 .. 512 tokens, block edges), one with sharp scores whose row
    maximum moves late (exercises the production kernel's offset move + rescale).
    Variants: 0 production, 7 the same kernel on 7 workgroups (many ragged items each),
    -1 the streaming kernel (sentences > 512)."""
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


@pytest.mark.parametrize("seed", [0, 1])
def test_short_attention_bitwise_equal_to_lds3(lib, seed):
    """Batches of at most 64 tokens per sentence (the serving shape) run
    attention_short_kernel: lds3's block-0 arithmetic on one 2-wave workgroup per
    (sentence, head).  Against numpy, and bitwise equal to attention_lds3 forced on
    the same batch (variant 8): a short sentence gets the same bits alone as inside
    a batch with longer sentences (the forward's batch-composition invariance)."""
    n_head, dh = 12, 64
    d = n_head * dh
    lens = [1, 2, 5, 31, 32, 33, 63, 64, 17]
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    T = int(cu[-1])
    rng = np.random.default_rng(seed)
    qkv = (rng.standard_normal((T, 3 * d)) * (1.0 + 3.0 * seed)).astype(np.float16)
    outs = {}
    for variant in (0, 8):
        out = np.zeros((T, d), np.float16)
        rc = lib.bertx_test_attention(qkv.ctypes.data, cu.ctypes.data, len(lens), n_head, d, variant, out.ctypes.data)
        assert rc == 0
        outs[variant] = out
    assert np.array_equal(outs[0].view(np.uint16), outs[8].view(np.uint16))
    ref = attention_ref(qkv, cu, n_head, d)
    got = outs[0].astype(np.float64)
    assert np.isfinite(got).all()
    assert np.abs(got - ref).max() < 6e-3 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_attention_pp_bitwise_equal_to_lds3(lib, seed):
    """attention_pp (the production kernel for 64 < L <= 512: two 8-wave
    workgroups per CU, half an item's queries each, K/V streamed through a
    4-stage ring of 64-key blocks) runs lds3's per-query block sequence on the
    same wave composition: bitwise equal to attention_lds3 (variant 8) on ragged
    lengths around every block, half-item and ring boundary, and within tolerance
    of numpy; seed 2 scales the scores so the offset-moving rescale path runs."""
    n_head, dh = 12, 64
    d = n_head * dh
    lens = [1, 63, 64, 65, 128, 191, 192, 255, 256, 257, 300, 383, 448, 511, 512, 17]
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    T = int(cu[-1])
    rng = np.random.default_rng(seed)
    qkv = (rng.standard_normal((T, 3 * d)) * (1.0 + 3.0 * seed)).astype(np.float16)
    outs = {}
    for variant in (0, 8):
        out = np.zeros((T, d), np.float16)
        rc = lib.bertx_test_attention(qkv.ctypes.data, cu.ctypes.data, len(lens), n_head, d, variant, out.ctypes.data)
        assert rc == 0
        outs[variant] = out
    assert np.array_equal(outs[0].view(np.uint16), outs[8].view(np.uint16))
    got = outs[0].astype(np.float64)
    assert np.isfinite(got).all()
    if seed < 2:   # (seed 2's peaked scores: lds3's own f16 P bounds its error; the bits are the check)
        ref = attention_ref(qkv, cu, n_head, d)
        assert np.abs(got - ref).max() < 6e-3 * max(1.0, np.abs(ref).max())


def test_attention_pp_bitwise_stress(lib):
    """attention_pp's Q rows arrive by asm loads retired by one tied wait, and its
    K/V by a ring of LDS-DMA pieces with counted waits: a missed wait would show as
    a timing-dependent difference.  24 random ragged batches (1-64 sentences of
    1-512 tokens, 12 heads), each bitwise equal to attention_lds3."""
    n_head, dh = 12, 64
    d = n_head * dh
    rng = np.random.default_rng(77)
    for it in range(24):
        n = int(rng.integers(1, 65))
        lens = rng.integers(65, 513, n) if it % 3 else rng.integers(1, 513, n)
        lens[0] = 512 if it % 4 == 0 else lens[0]
        if max(lens) <= 64:
            lens[0] = 65
        cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        T = int(cu[-1])
        qkv = (rng.standard_normal((T, 3 * d)) * 1.5).astype(np.float16)
        outs = []
        for variant in (0, 8):
            out = np.zeros((T, d), np.float16)
            assert lib.bertx_test_attention(qkv.ctypes.data, cu.ctypes.data, n, n_head, d, variant,
                                            out.ctypes.data) == 0
            outs.append(out)
        assert np.array_equal(outs[0].view(np.uint16), outs[1].view(np.uint16)), (it, list(lens[:8]))


@pytest.mark.parametrize("fmt,N,K,M,want", [
    (1, 384, 1536, 256, 4), (1, 1152, 384, 1024, 4), (2, 768, 3072, 1024, 16), (8, 2304, 768, 512, 16),
    (3, 1024, 4096, 1024, 16), (2, 2304, 768, 1024, 3), (1, 1152, 384, 2048, 3), (1, 1536, 384, 4096, 3),
    (2, 3072, 768, 32768, 2), (8, 768, 3072, 32768, 2)])
def test_gemm_tile_heuristic(lib, fmt, N, K, M, want):
    """The tile form the heuristic (gemm.hip pick_cfg, cfg 0) runs on a 256-CU MI355X,
    pinned so a change to it is deliberate: 64 x 64 tiles for small M -- 2 waves for
    f16 weights, 4 waves with wave-private X rings for q4_0 / q4_1 / q8_0
    (profiles/r06_cfg_small_sweep.log, r06_cfg_small_q41.log) -- 128 x 128 once those
    cover half the CUs (r06_cfg34_crossover.log), 256 x 128 at two per CU."""
    # (the choices assume the 256 CUs of one MI355X in SPX mode, as on the test boxes)
    us = ctypes.c_float()
    assert lib.bertx_bench_gemm(fmt, N, K, M, 0 if N > K else 2, 0, 1, ctypes.byref(us)) == 0
    assert lib.bertx_test_gemm_ran() == want


@pytest.mark.parametrize("fmt", [1, 2, 3, 8])
@pytest.mark.parametrize("cfg", [2, 3, 11, 16])
def test_small_tiles_bitwise_equal_to_64x64(lib, fmt, cfg):
    """Tile shape and wave layout change who computes an output, not how: every (token,
    feature) is the same k-ordered MFMA chain and the same epilogue arithmetic, so every
    shipped config gives the 64x64 tile's bits (the forward's batch-composition invariance
    rests on it), including the residual form's LN statistics: the 256- and 128-row tiles,
    the interleaved- and burst-X forms (2, 11) and the wave-private rings on 4 waves (16)."""
    N, K, M = 768, 1536, 256
    rng = np.random.default_rng(fmt + cfg)
    W = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    wb, _ = weight_rows(fmt, W)
    bias = rng.standard_normal(N).astype(np.float32) * 0.1
    X = rng.standard_normal((M, K)).astype(np.float16)
    z = (rng.standard_normal((M, N)) * 2).astype(np.float16)
    stats = np.ascontiguousarray(np.stack([rng.standard_normal(M) * 0.1, 1 + rng.random(M)], axis=1), np.float32)
    g, be, gn = (rng.standard_normal(N).astype(np.float32) * 0.3 + 1 for _ in range(3))
    outs = {}
    for c in (4, cfg):
        out = np.zeros((M, N), np.float16)
        st = np.zeros((M, 2), np.float32)
        assert lib.bertx_test_gemm_ln(fmt, N, K, wb, f32p(bias), M, X.ctypes.data, None, None, None, 2, z.ctypes.data,
                                      stats.ctypes.data, f32p(g), f32p(be), f32p(gn), out.ctypes.data,
                                      st.ctypes.data, c) == 0
        assert lib.bertx_test_gemm_ran() == c
        up = np.zeros((M, N), np.float16)
        assert lib.bertx_test_gemm(fmt, N, K, wb, bias.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), M,
                                   X.ctypes.data, 1, None, up.ctypes.data, c) == 0
        outs[c] = (out, st, up)
    for a, b in zip(outs[4], outs[cfg]):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
