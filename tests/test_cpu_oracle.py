"""CPU tests of the ORACLE (oracle/, test infrastructure) against independent
restatements and the committed golden fixtures -- the oracle must be pinned
before it can judge the HIP path.

Pins (DESIGN.md "Oracle"):
  * fp16 conversion: numpy's IEEE RNE float16 (ggml-era GGML_FP32_TO_FP16 on F16C
    hardware is the same instruction, ggml.c-era vcvtps2ph RNE).
  * GELU / exp tables: the ggml-era definitions (bert.cpp:1063 calls ggml_gelu,
    table-driven in that ggml) recomputed in float64 and rounded to f16.
  * quantizers: numpy restatement of the ggml-era q4_0/q4_1/q8_0 row quantizers
    (models/quantize.cpp:23-142 drives them through ggml_quantize_q4_0/q4_1).
  * tokenizer: tokenizer_cases.json from the reference's OWN tokenizer source
    (bert.cpp:195-417 compiled by oracle/build_ref.sh).
  * forward: tiny models converted by the reference converter
    (models/convert-to-ggml.py) with an independent torch forward (make_golden.py).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

Q4_0, Q4_1, Q8_0 = 2, 3, 8


# ---------------------------------------------------------------- fp16 -------

def test_f32_to_f16_matches_numpy_rne(oracle):
    L = oracle.lib()
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2**32, 60000, dtype=np.uint64).astype(np.uint32)
    vals = bits.view(np.float32)
    edge = np.array([0.0, -0.0, 1.0, 65504.0, 65519.99, 65520.0, 1e-8, 5.96e-8, 2.98e-8, 2.99e-8, 6.1e-5,
                     6.097e-5, -3.5, 1.0009765625, 1.00048828125, 1.00146484375, np.inf, -np.inf], np.float32)
    vals = np.concatenate([vals, edge])
    vals = vals[np.isfinite(vals) | np.isinf(vals)]
    with np.errstate(over="ignore"):
        ref = vals.astype(np.float16).view(np.uint16)
    got = np.array([L.oracle_f32_to_f16(float(v)) for v in vals], np.uint16)
    np.testing.assert_array_equal(got, ref)


def test_f16_to_f32_all_codes(oracle):
    L = oracle.lib()
    codes = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    ref = codes.view(np.float16).astype(np.float32)
    got = np.array([L.oracle_f16_to_f32(int(c)) for c in codes], np.float32)
    fin = np.isfinite(ref)
    np.testing.assert_array_equal(got[fin].view(np.uint32), ref[fin].view(np.uint32))
    assert np.all(np.isnan(got[np.isnan(ref)]))


def _f16_ulp(x):
    x = np.abs(x.astype(np.float16)).astype(np.float32)
    return np.maximum(np.spacing(x.astype(np.float16)).astype(np.float32), 2.0**-24)


def test_gelu_and_exp_tables(oracle):
    """Every finite f16 input: table value within one f16 ulp of the float64
    definition (the table is built in f32 -- tanhf/expf -- then rounded)."""
    L = oracle.lib()
    codes = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    x = codes.view(np.float16).astype(np.float64)
    fin = np.isfinite(x) & (np.abs(x) < 60)
    xs = x[fin][::7]
    g64 = 0.5 * xs * (1.0 + np.tanh(0.79788456080286535587989211986876 * xs * (1.0 + 0.044715 * xs * xs)))
    e64 = np.exp(xs)
    g = np.array([L.oracle_gelu(float(v)) for v in xs])
    e = np.array([L.oracle_exp(float(v)) for v in xs])
    gr = g64.astype(np.float16).astype(np.float64)
    assert np.all(np.abs(g - gr) <= _f16_ulp(gr) + 1e-12)
    ok = e64 < 65504
    er = e64[ok].astype(np.float16).astype(np.float64)
    assert np.all(np.abs(e[ok] - er) <= _f16_ulp(er) + 1e-12)
    assert np.all(np.isinf(e[~ok]))


# ---------------------------------------------------------- quantizers -------

def _np_quantize(kind, x):
    """ggml-era row quantizers restated in numpy float32 (block of 32)."""
    xb = x.reshape(-1, 32).astype(np.float32)
    f16 = lambda v: np.asarray(v, np.float32).astype(np.float16).view(np.uint16)  # noqa: E731
    out = []
    for b in xb:
        if kind == Q4_0:
            j = int(np.argmax(np.abs(b)))          # first index of the largest |x|
            d = np.float32(b[j] / np.float32(-8))
            idd = np.float32(1.0) / d if d != 0 else np.float32(0)
            q = np.trunc(b * idd + np.float32(8.5)).astype(np.int64).clip(max=15)
            qs = (q[:16] | (q[16:] << 4)).astype(np.uint8)
            out.append(f16(d).tobytes() + qs.tobytes())
        elif kind == Q4_1:
            vmin, vmax = b.min(), b.max()
            d = np.float32((vmax - vmin) / np.float32(15))
            idd = np.float32(1.0) / d if d != 0 else np.float32(0)
            q = np.trunc((b - vmin) * idd + np.float32(0.5)).astype(np.int64).clip(max=15)
            qs = (q[:16] | (q[16:] << 4)).astype(np.uint8)
            out.append(f16(d).tobytes() + f16(vmin).tobytes() + qs.tobytes())
        else:
            amax = np.abs(b).max()
            d = np.float32(amax / np.float32(127))
            idd = np.float32(1.0) / d if d != 0 else np.float32(0)
            v = b * idd
            q = (np.sign(v) * np.floor(np.abs(v) + np.float32(0.5))).astype(np.int8)   # roundf
            out.append(f16(d).tobytes() + q.tobytes())
    return b"".join(out)


@pytest.mark.parametrize("kind,bsize", [(Q4_0, 18), (Q4_1, 20), (Q8_0, 34)])
def test_quantize_row_matches_numpy(oracle, kind, bsize):
    L = oracle.lib()
    rng = np.random.default_rng(kind)
    x = (rng.standard_normal(32 * 64) * rng.uniform(0.01, 3.0, 32 * 64)).astype(np.float32)
    x[:32] = 0.0                 # all-zero block: d = 0, id = 0
    x[32:64] = 1.5               # constant block
    x[64 + 5] = -7.0             # negative extreme
    buf = np.zeros(64 * bsize, np.uint8)
    L.oracle_quantize_row(kind, x.ctypes.data, buf.ctypes.data, x.size)
    assert buf.tobytes() == _np_quantize(kind, x)
    # dequantization error within half a step (plus f16 rounding of d / m)
    y = np.zeros_like(x)
    L.oracle_dequantize_row(kind, buf.ctypes.data, y.ctypes.data, x.size)
    xb, yb = x.reshape(-1, 32), y.reshape(-1, 32)
    rng_b = np.abs(xb).max(1) if kind != Q4_1 else (xb.max(1) - xb.min(1))
    steps = {Q4_0: 8.0, Q4_1: 15.0, Q8_0: 127.0}[kind]
    tol = rng_b / steps * (1.0 if kind == Q4_0 else 0.5) + rng_b * 2e-3 + 1e-7
    assert np.all(np.abs(xb - yb) <= tol[:, None])


# ------------------------------------------------------------ tokenizer ------

def test_oracle_tokenizer_matches_reference_goldens(oracle, tok_golden):
    """Oracle tokenizer == token ids of the reference's own tokenizer source."""
    orc = oracle.Oracle(str(GOLDEN + "/tiny32/ggml-model-f32.bin"))
    cases = tok_golden["cases"]
    assert len(cases) >= 100
    bad = []
    for c in cases:
        got = orc.tokenize(bytes.fromhex(c["text_hex"]), c["n_max_tokens"])
        if got != c["ids"]:
            bad.append((c["text_hex"][:40], got[:10], c["ids"][:10]))
    assert not bad, bad[:5]


def expected_id_to_token(vocab):
    """bert_vocab_id_to_token semantics (bert.cpp:121-134 over the maps filled at
    bert.cpp:484-493): first occurrence of a word wins; "##" words always map."""
    seen, out = set(), []
    for w in vocab:
        if w not in seen:
            seen.add(w)
            out.append(w)
        elif w.startswith("##"):
            out.append(w)
        else:
            out.append("[UNK TOKEN from bert_vocab]")
    return out


def test_oracle_vocab_roundtrip(oracle, tok_golden):
    orc = oracle.Oracle(str(GOLDEN + "/tiny32/ggml-model-f32.bin"))
    vocab = tok_golden["vocab"]
    assert orc.n_vocab == len(vocab)
    exp = expected_id_to_token(vocab)
    assert [orc.id_to_token(i).decode("utf-8") for i in range(len(vocab))] == exp
    assert orc.id_to_token(len(vocab) + 5) == b"[UNK TOKEN from bert_vocab]"


# -------------------------------------------------------------- forward ------

@pytest.mark.parametrize("tiny", ["tiny32", "tiny64"])
def test_oracle_forward_matches_torch_golden(oracle, tiny):
    z = np.load(f"{GOLDEN}/{tiny}/forward_f32.npz")
    ids, lens = z["ids"], z["lens"]
    seqs = np.split(ids, np.cumsum(lens)[:-1])
    orc = oracle.Oracle(f"{GOLDEN}/{tiny}/ggml-model-f32.bin")
    emb = orc.forward_batch(seqs, n_threads=4)
    cos = np.sum(emb * z["torch_emb"], axis=1)
    assert cos.min() > 1 - 1e-4, cos.min()
    np.testing.assert_allclose(emb, z["oracle_emb"], atol=2e-6)
    np.testing.assert_allclose(np.linalg.norm(emb, axis=1), 1.0, atol=1e-5)


def test_oracle_batch_vs_single_and_fake(oracle):
    z = np.load(f"{GOLDEN}/tiny32/forward_f32.npz")
    seqs = np.split(z["ids"], np.cumsum(z["lens"])[:-1])[:5]
    orc = oracle.Oracle(f"{GOLDEN}/tiny32/ggml-model-f16.bin")
    batch = orc.forward_batch(seqs)
    single = np.concatenate([orc.forward_batch([s]) for s in seqs])
    fake = orc.forward_fake_batch(seqs)
    assert np.min(np.sum(batch * single, 1)) > 1 - 1e-5
    assert np.min(np.sum(fake * single, 1)) > 1 - 1e-5


def test_oracle_quantized_forward_close(oracle, quant_models):
    z = np.load(f"{GOLDEN}/tiny64/forward_f32.npz")
    seqs = np.split(z["ids"], np.cumsum(z["lens"])[:-1])[:6]
    ref = oracle.Oracle(quant_models[("tiny64", "f32")]).forward_batch(seqs)
    for fmt, lim in (("q8_0", 0.999), ("q4_1", 0.98), ("q4_0", 0.97), ("f16", 0.99999)):
        e = oracle.Oracle(quant_models[("tiny64", fmt)]).forward_batch(seqs)
        assert np.min(np.sum(e * ref, 1)) > lim, fmt


def test_oracle_too_long_refused(oracle):
    orc = oracle.Oracle(f"{GOLDEN}/tiny32/ggml-model-f32.bin")
    assert orc.forward_batch([[101] + [150] * (orc.n_max_tokens + 3) + [102]]) is None


def test_oracle_encode_batch(oracle):
    """bert_encode_batch semantics (bert.cpp:818-880): tokenise, sort by length,
    chunks of n_batch_size; every input written."""
    orc = oracle.Oracle(f"{GOLDEN}/tiny32/ggml-model-f16.bin")
    texts = ["hello world", "the store", "a", "i'm going to the store to buy 3 apples", "", "cloud outside"]
    out, written = orc.encode_batch(texts, 4)
    assert written.all()
    for t, e in zip(texts, out):
        single = orc.forward_batch([orc.tokenize(t)])[0]
        assert float(np.dot(single, e)) > 1 - 1e-5


def test_activation_f32_mode(oracle, quant_models):
    """The diagnostic mode (oracle_forward_batch_ex's act_f32 argument):
    quantized weights times f32 activations instead of the reference's q8
    re-quantized ones.  It changes only the quantized-weight matmuls (f16 / f32 files
    bitwise unchanged), moves a tiny q4_0 model by a little (the q8 rounding), brings
    it closer to the f32-weight forward of the same model, and -- a per-call argument,
    not process state -- leaves every other call in the reference's arithmetic, also
    one running concurrently on another thread."""
    z = np.load(f"{GOLDEN}/tiny64/forward_f32.npz")
    seqs = np.split(z["ids"], np.cumsum(z["lens"])[:-1])[:6]
    ref = oracle.Oracle(quant_models[("tiny64", "f32")]).forward_batch(seqs)
    for fmt in ("f16", "f32"):
        o = oracle.Oracle(quant_models[("tiny64", fmt)])
        assert np.array_equal(o.forward_batch(seqs), o.forward_batch(seqs, activations="f32"))
    o = oracle.Oracle(quant_models[("tiny64", "q8_0")])
    q8 = o.forward_batch(seqs)
    f32 = o.forward_batch(seqs, activations="f32")
    assert not np.array_equal(q8, f32)
    c_q8 = np.sum(q8 * ref, axis=1)
    c_f32 = np.sum(f32 * ref, axis=1)
    assert np.all(np.sum(q8 * f32, axis=1) > 1 - 1e-3)
    assert np.mean(1 - c_f32) <= np.mean(1 - c_q8)
    assert np.array_equal(o.forward_batch(seqs), q8)
    # concurrent callers (ctypes releases the GIL): each keeps its own arithmetic, and
    # the lazily made f32 weight cache is built once under a lock
    import threading
    o2 = oracle.Oracle(quant_models[("tiny64", "q4_0")])
    res = {}

    def run(k, act):
        res[k] = o2.forward_batch(seqs, n_threads=2, activations=act)
    th = [threading.Thread(target=run, args=(k, "f32" if k % 2 else "q8")) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    want_q8, want_f32 = o2.forward_batch(seqs), o2.forward_batch(seqs, activations="f32")
    for k in range(6):
        assert np.array_equal(res[k], want_f32 if k % 2 else want_q8), k


def _model_tensors(oracle, path):
    """(hparams, {name: f32 array}) of a model file in the reference format
    (bert.cpp:434-766); quantized rows dequantized by the oracle's era dequantizer."""
    import struct
    L = oracle.lib()
    f = open(path, "rb").read()
    off = 4
    hp = struct.unpack_from("<7i", f, off)
    off += 28
    for _ in range(hp[0]):
        off += 4 + struct.unpack_from("<i", f, off)[0]
    out = {}
    while off < len(f):
        nd, nl, ft = struct.unpack_from("<3i", f, off)
        off += 12
        ne = struct.unpack_from(f"<{nd}i", f, off)
        off += 4 * nd
        name = f[off:off + nl].decode()
        off += nl
        k, rows = ne[0], int(np.prod(ne[1:])) if nd > 1 else 1
        rb = {0: 4 * k, 1: 2 * k, 2: k // 32 * 18, 3: k // 32 * 20, 8: k // 32 * 34}[ft]
        buf = np.frombuffer(f, np.uint8, rb * rows, off)
        off += rb * rows
        if ft == 0:
            a = buf.view(np.float32).reshape(rows, k)
        elif ft == 1:
            a = buf.view(np.float16).astype(np.float32).reshape(rows, k)
        else:
            a = np.zeros((rows, k), np.float32)
            base = buf.ctypes.data
            for r in range(rows):
                L.oracle_dequantize_row(ft, base + r * rb, a[r].ctypes.data, k)
        out[name] = a if nd > 1 else a.reshape(-1)
    return hp, out


def _torch_forward(hp, tensors, ids_list):
    """An independent float forward: transformers' BertModel with the era constants
    (tanh GELU, LayerNorm eps 1e-5) on the file's (dequantized) weights, masked mean
    pool, L2 normalise (tests/golden/make_golden.py torch_embed)."""
    import torch
    from transformers import BertConfig, BertModel
    cfg = BertConfig(vocab_size=hp[0], hidden_size=hp[2], num_attention_heads=hp[4], intermediate_size=hp[3],
                     num_hidden_layers=hp[5], max_position_embeddings=hp[1], type_vocab_size=2,
                     hidden_act="gelu_pytorch_tanh", layer_norm_eps=1e-5)
    model = BertModel(cfg, add_pooling_layer=False)
    missing, unexpected = model.load_state_dict({k: torch.tensor(np.asarray(v)) for k, v in tensors.items()},
                                                strict=False)
    assert not unexpected and all("position_ids" in k for k in missing), (missing, unexpected)
    model.eval()
    Lm = max(len(x) for x in ids_list)
    ids = torch.full((len(ids_list), Lm), 101, dtype=torch.long)
    mask = torch.zeros((len(ids_list), Lm), dtype=torch.long)
    for i, x in enumerate(ids_list):
        ids[i, : len(x)] = torch.tensor(np.asarray(x, np.int64))
        mask[i, : len(x)] = 1
    with torch.no_grad():
        h = model(input_ids=ids, attention_mask=mask, token_type_ids=torch.zeros_like(ids)).last_hidden_state
        m = mask.unsqueeze(-1).float()
        e = (h * m).sum(1) / m.sum(1)
        e = e / e.norm(dim=-1, keepdim=True)
    return e.numpy().astype(np.float32)


@pytest.mark.parametrize("arch,ftype,profile", [("all-MiniLM-L6-v2", "f32", "sharp"),
                                                 ("bge-base-en-v1.5", "q4_0", "survey")])
def test_oracle_pinned_to_torch_at_survey_dims(oracle, tmp_path, arch, ftype, profile):
    """The oracle's forward against an independent torch/transformers forward at the
    SURVEY architectures (the committed goldens pin it on tiny models only): C1's
    MiniLM-L6 f32 file on sharp weights, and C3's bge-base architecture as a q4_0 file
    -- torch runs the file's dequantized weights (embedding tables included) and the
    oracle runs its f32-activation mode, so both multiply the same weights by f32
    activations and the comparison pins the oracle's q4_0 decoding, layer order, era
    GELU / softmax tables and pooling at full depth.  Ragged lengths (padding and mask)."""
    import bertpy
    hp_arch = bertpy.ARCHS[arch]
    path = str(tmp_path / f"{arch}-{ftype}.bin")
    if ftype == "f32":
        bertpy.write_model(path, hp_arch, bertpy.synthetic_vocab(hp_arch["n_vocab"]),
                           bertpy.synthetic_tensors(hp_arch, 1234, profile), 0)
    else:
        f16 = str(tmp_path / f"{arch}-f16.bin")
        bertpy.write_model(f16, hp_arch, bertpy.synthetic_vocab(hp_arch["n_vocab"]),
                           bertpy.synthetic_tensors(hp_arch, 1234, profile), 1)
        assert oracle.quantize_file(f16, path, 2) == 0
        os.remove(f16)
    hp, tensors = _model_tensors(oracle, path)
    ids = bertpy.synthetic_ids(4, [32, 17, 5, 64], hp[0], seed=7)
    ref = _torch_forward(hp, tensors, ids)
    got = oracle.Oracle(path).forward_batch(ids, activations="f32" if ftype != "f32" else "q8")
    c = np.sum(got * ref, axis=1)
    print(arch, ftype, "oracle vs torch min cosine", c.min())
    assert np.all(c >= 1 - 1e-4), c
