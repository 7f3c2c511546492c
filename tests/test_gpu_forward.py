"""End-to-end parity of the HIP forward (through the C ABI) with the CPU oracle, the
committed torch cross-check goldens, and the reference's batching semantics."""
import os

import numpy as np
import pytest

import bertpy
import oracle_lib
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3   # north_star: float vectors within 1e-3 cosine of the reference path
MIN_SHARE_TOKENS = 8192   # bert_abi.cpp kMinShareTokens (routing: the smallest share of a split call)


@pytest.fixture(scope="module", autouse=True)
def _one_device():
    os.environ.pop("BERT_HOST_ONLY", None)
    os.environ["BERT_DEVICES"] = "0"


def ragged_ids(n_vocab, lens, seed=3):
    rng = np.random.default_rng(seed)
    return [np.concatenate([[101], rng.integers(104, n_vocab, L - 2), [102]]).astype(np.int32) if L >= 2
            else np.array([101], np.int32) for L in lens]


def cosines(a, b):
    return np.sum(a * b, axis=1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))


@pytest.mark.parametrize("tiny", ["tiny32", "tiny64"])
@pytest.mark.parametrize("fmt", ["f32", "f16", "q4_0", "q4_1", "q8_0"])
def test_forward_matches_oracle(quant_models, tiny, fmt):
    path = quant_models[(tiny, fmt)]
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    maxl = m.n_max_tokens
    ids = ragged_ids(o.n_vocab, [2, 3, 17, 64, 100, maxl - 1, maxl, 33])
    got = m.forward_batch(ids)
    ref = o.forward_batch(ids)
    c = cosines(got, ref)
    assert np.all(c >= 1 - COS_TOL), c
    assert np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-5)


F32_COS_TOL = 1e-6   # f32 files: f32 x f32 like the reference (bert.cpp:499-503)


@pytest.mark.parametrize("tiny", ["tiny32", "tiny64"])
def test_f32_file_at_f32_precision(quant_models, tiny):
    """f32 files run the f32 chain (f32.hip: f32 activations x f32 weights, the era's
    fp16-table softmax exp and GELU as the reference applies them): 1 - cos <= 1e-6
    against the oracle's f32 forward on ragged lengths up to n_max_tokens, an
    absolute bound three orders tighter than the f16 paths'."""
    path = quant_models[(tiny, "f32")]
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    ids = ragged_ids(o.n_vocab, [2, 3, 17, 64, 100, m.n_max_tokens - 1, m.n_max_tokens, 33])
    c = cosines(m.forward_batch(ids), o.forward_batch(ids))
    print(tiny, "f32 chain: 1 - min cos vs oracle", float(1.0 - c.min()))
    assert np.all(c >= 1 - F32_COS_TOL), 1.0 - c


@pytest.mark.parametrize("tiny", ["tiny32", "tiny64"])
def test_forward_matches_torch_golden(tiny):
    path = os.path.join(GOLDEN, tiny, "ggml-model-f32.bin")
    g = np.load(os.path.join(GOLDEN, tiny, "forward_f32.npz"))
    lens = g["lens"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    ids = [g["ids"][offs[i]:offs[i + 1]] for i in range(len(lens))]
    got = bertpy.BertModel(path).forward_batch(ids)
    assert np.all(cosines(got, g["torch_emb"]) >= 1 - COS_TOL)
    assert np.all(cosines(got, g["oracle_emb"]) >= 1 - COS_TOL)


def test_batch_composition_invariance(quant_models):
    """A sentence's embedding must not depend on what else is in the batch (bitwise)."""
    m = bertpy.BertModel(quant_models[("tiny64", "q4_0")])
    ids = ragged_ids(690, [5, 300, 512, 40, 2, 129])
    full = m.forward_batch(ids)
    # alone, sentence 5 (129 tokens) takes the one-launch pool over 3 chunks, in
    # the batch (max_len 512) the two-launch pool: same bits
    for i in (0, 2, 4, 5):
        alone = m.forward_batch([ids[i]])
        assert np.array_equal(alone[0], full[i])
    rev = m.forward_batch(ids[::-1])
    assert np.array_equal(rev[::-1], full)


def test_stats_fold_forward_bitwise(quant_models, tmp_path):
    """The small-batch statistics fold (engine.cpp: QKV / FFN-up combine their input's
    LN statistics from the residual GEMM's partials; 2 n_layer - 1 fewer ln_stats
    launches) gives the bits of the launch form end to end.  The switch
    is a process-wide static (BERT_STATS_FOLD), so each form runs in its own
    process on the same ids, for every quantized format and both tile families the
    fold runs on (64-row tiles at a few tokens, 128-row tiles at a few hundred)."""
    import subprocess
    import sys
    ids = ragged_ids(690, [5, 17, 32, 60], seed=4)
    big = ragged_ids(690, [300, 290, 310, 512], seed=5)
    allx = ids + big
    np.savez(tmp_path / "ids.npz", flat=np.concatenate(allx).astype(np.int32), lens=[len(x) for x in allx])
    code = (
        "import sys, numpy as np\n"
        f"sys.path.insert(0, {os.path.join(os.path.dirname(bertpy.__file__), '..')!r})\n"
        "import bertpy\n"
        "m = bertpy.BertModel(sys.argv[1])\n"
        "z = np.load(sys.argv[2])\n"
        "ids = np.split(z['flat'], np.cumsum(z['lens'])[:-1])\n"
        "np.save(sys.argv[3], np.concatenate([m.forward_batch(ids[:4]), m.forward_batch(ids[4:])]))\n")
    for fmt in ("q4_0", "q4_1", "q8_0", "f16"):
        outs = []
        for fold in ("0", "1"):
            out = tmp_path / f"{fmt}_{fold}.npy"
            env = dict(os.environ, BERT_STATS_FOLD=fold, BERT_DEVICES="0")
            r = subprocess.run([sys.executable, "-c", code, quant_models[("tiny64", fmt)], str(tmp_path / "ids.npz"),
                                str(out)], env=env, capture_output=True, timeout=120)
            assert r.returncode == 0, r.stderr.decode()[-2000:]
            outs.append(np.load(out))
        assert np.all(np.isfinite(outs[0]))
        assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32)), fmt


def test_fake_batch_and_forward(quant_models):
    """bert_forward_fake_batch and bert_forward against the oracle's restatements
    (oracle_forward_fake_batch: bert.cpp:1151-1363; bert_forward = a batch of one,
    bert.cpp:817-825), not against the HIP batch path."""
    path = quant_models[("tiny32", "f16")]
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    ids = ragged_ids(690, [4, 50, 128])
    b = m.forward_batch(ids, fake=True)
    assert np.all(cosines(b, o.forward_fake_batch(ids)) >= 1 - COS_TOL)
    one = m.forward(ids[1])
    assert np.all(cosines(one[None], o.forward_batch(ids[1:2])) >= 1 - COS_TOL)


def test_empty_and_degenerate_batches(quant_models):
    """Edge cases of the ABI on a device: an empty batch (forward and encode) is a
    no-op; an empty text encodes as [CLS] [SEP] and a one-token sentence runs, both
    unit-norm and within the cosine bound of the oracle; a sentence at exactly
    n_max_tokens runs beside a one-token one, each bitwise as it is alone."""
    path = quant_models[("tiny64", "q4_0")]
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    assert m.forward_batch([]).shape == (0, m.n_embd)
    assert m.encode([]).shape == (0, m.n_embd)
    e = m.encode(["", "a"], batch_size=2)
    assert np.all(np.isfinite(e)) and np.allclose(np.linalg.norm(e, axis=1), 1.0, atol=1e-5)
    ref, written = o.encode_batch(["", "a"], 2)
    assert written.all()
    assert np.all(cosines(e, ref) >= 1 - COS_TOL)
    ids = ragged_ids(690, [1, m.n_max_tokens], seed=9)
    both = m.forward_batch(ids)
    assert np.all(np.isfinite(both))
    assert np.all(cosines(both, o.forward_batch(ids)) >= 1 - COS_TOL)
    for i in range(2):
        assert np.array_equal(m.forward_batch([ids[i]])[0], both[i])


def test_too_long_is_refused(quant_models):
    m = bertpy.BertModel(quant_models[("tiny32", "f16")])
    ids = ragged_ids(690, [10, 129])          # n_max_tokens = 128
    out = m.forward_batch(ids, fill=5.0)
    assert np.all(out == 5.0)                 # bert.cpp:867-871: nothing written
    fake = m.forward_batch(ids, fake=True, fill=5.0)
    assert not np.all(fake[0] == 5.0) and np.all(fake[1] == 5.0)   # stops at the first long input


def test_encode_batch_matches_oracle(quant_models):
    import json
    path = quant_models[("tiny64", "q8_0")]
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    cases = json.load(open(os.path.join(GOLDEN, "tokenizer_cases.json")))["cases"]
    texts = [bytes.fromhex(c["text_hex"]) for c in cases if c["n_max_tokens"] == 512][:60]
    for bs in (len(texts), 16, 7, 1):
        got = m.encode(texts, batch_size=bs)
        ref, written = o.encode_batch(texts, bs)
        wrote = ~np.all(got == 0.0, axis=1)
        assert np.array_equal(wrote, written), bs
        c = cosines(got[written], ref[written])
        assert np.all(c >= 1 - COS_TOL), (bs, c.min())


def test_c5_multilingual_encode_matches_oracle(tmp_path):
    """SURVEY §8d end-to-end at C5 dims (bge-base-zh q8_0, V 21,128) on multilingual
    text: a BERT-like WordPiece vocab with Latin-1, Greek and CJK entries
    (bertpy.bert_like_vocab), texts of whole words, '##'-split words, accents, digits,
    punctuation, CJK runs and characters outside the vocab, plus all-CJK texts, from
    a few to past 512 tokens.  Through bert_encode_batch (sorted, chunked by
    n_batch_size; a chunk holding an over-long text is refused, as bert.cpp:1408-1443
    does) against the oracle's encode_batch: the same token ids, the same written
    rows, every written row within the north-star cosine."""
    hp = bertpy.ARCHS["bge-base-zh-v1.5"]
    vocab = bertpy.bert_like_vocab(hp["n_vocab"], seed=5)
    path = str(tmp_path / "bge-base-zh-q8_0-multilingual.bin")
    bertpy.synthetic_model(path, "bge-base-zh-v1.5", "q8_0", seed=1234, vocab=vocab)
    texts = []
    for k, nw in enumerate((3, 12, 40, 90, 160, 260)):
        texts += bertpy.bert_like_texts(vocab, 3, nw, seed=20 + k)
    rng = np.random.default_rng(31)
    cjk = [w for w in vocab[104:] if len(w) == 1 and ord(w) >= 0x3400]
    for n in (7, 60, 200, 480, 560):
        texts.append(("".join(cjk[int(i)] + ("\u3002" if j % 17 == 16 else "")
                              for j, i in enumerate(rng.integers(0, len(cjk), n)))).encode("utf-8"))
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    for t in texts:
        ids, n = m.tokenize(t)
        assert ids == o.tokenize(t)[: len(ids)] and n == len(o.tokenize(t)), t[:40]
    lens = [m.tokenize(t)[1] for t in texts]
    assert min(lens) < 16 and max(lens) > 512 and sum(x > 300 for x in lens) >= 3, lens
    for bs in (8, 5, len(texts)):
        got = m.encode(texts, batch_size=bs)
        ref, written = o.encode_batch(texts, bs, n_threads=min(16, os.cpu_count() or 1))
        wrote = ~np.all(got == 0.0, axis=1)
        assert np.array_equal(wrote, written), (bs, wrote, written)
        if bs == len(texts):                                  # one unsorted batch holding a > 512 text: refused
            assert not written.any()
            continue
        assert written.sum() >= len(texts) - bs              # only the chunk with the long text refused
        c = cosines(got[written], ref[written])
        print(f"C5 multilingual encode, batch {bs}: {int(written.sum())} rows, min cos {c.min():.7f}")
        assert np.all(c >= 1 - COS_TOL), (bs, c.min())


def test_bge_base_q4_0_full_size(tmp_path):
    """BASELINE config shape: bge-base q4_0, L = 512, B = 64.  Oracle parity on two
    sentences; size-independent properties on the full batch."""
    path = str(tmp_path / "bge-base-q4_0.bin")
    bertpy.synthetic_model(path, "bge-base-en-v1.5", "q4_0", seed=1234)
    m = bertpy.BertModel(path)
    ids = bertpy.synthetic_ids(64, 512, 30522, seed=7)
    full = m.forward_batch(ids)
    assert np.all(np.isfinite(full))
    assert np.allclose(np.linalg.norm(full, axis=1), 1.0, atol=1e-5)
    # captured on the second run, replayed on the third: the in-launch statistics'
    # flags (cleared by the residual GEMM in front of each projection) hold across
    # replays
    assert np.array_equal(m.forward_batch(ids), full)
    assert np.array_equal(m.forward_batch(ids), full)
    two = m.forward_batch(ids[:2])
    assert np.array_equal(two, full[:2])
    assert np.array_equal(m.forward_batch(ids[62:]), full[62:])
    # every sentence bitwise as in 8-sentence batches (those launch one workgroup
    # per tile and an ln_stats launch in front of each projection; the full batch
    # runs its N = 768 GEMMs persistent, two workgroups per CU walking the tiles,
    # and its projections with in-launch statistics: gemm.hip dispatch_z)
    eights = np.concatenate([m.forward_batch(ids[i:i + 8]) for i in range(0, 64, 8)])
    assert np.array_equal(eights, full)
    ref = oracle_lib.Oracle(path).forward_batch([ids[0], ids[1], ids[63]], n_threads=min(16, os.cpu_count() or 1))
    assert np.all(cosines(full[[0, 1, 63]], ref) >= 1 - COS_TOL)


@pytest.mark.parametrize("arch,ftype", [("all-MiniLM-L6-v2", "f16"), ("bge-base-en-v1.5", "q4_0"),
                                         ("bge-large-en-v1.5", "q4_1")])
def test_graph_replay_bitwise(tmp_path, arch, ftype):
    """A batch runs eagerly on first use, is captured into a HIP graph on its second
    and replayed on its third (engine.cpp forward_ordered): all three give the same
    bits on ragged lengths whose packed rows end mid-tile (tile padding rows carry
    stale values from earlier forwards, which valid rows never read)."""
    hp = bertpy.ARCHS[arch]
    path = str(tmp_path / f"{arch}-{ftype}.bin")
    bertpy.synthetic_model(path, arch, ftype, seed=1234)
    lens = [512, 3, 200, 129, 17, 511, 64, 1, 300]
    ids = bertpy.synthetic_ids(len(lens), lens, hp["n_vocab"], seed=5)
    m = bertpy.BertModel(path)
    a = m.forward_batch(ids)
    b = m.forward_batch(ids)
    c = m.forward_batch(ids)
    assert np.all(np.isfinite(a))
    assert np.array_equal(a, b)
    assert np.array_equal(a, c)


def test_two_replicas_on_one_device_bitwise(quant_models, monkeypatch):
    """In-process sharding (bert_abi.cpp run_forward): BERT_DEVICES=0,0 gives two
    replicas with their own streams; outputs are bitwise those of one replica."""
    path = quant_models[("tiny64", "q4_0")]
    ids = ragged_ids(690, [5, 300, 512, 40, 2, 129, 77, 250, 3])
    one = bertpy.BertModel(path).forward_batch(ids)
    monkeypatch.setenv("BERT_DEVICES", "0,0")
    m2 = bertpy.BertModel(path)
    assert m2.lib.bertx_num_devices(m2.ctx) == 2
    two = m2.forward_batch(ids)
    assert np.array_equal(one, two)


# SURVEY §8 configurations other than the bench's (C3): shapes at full size,
# oracle parity on a few sentences, size-independent properties on the batch.
SURVEY_CONFIGS = {
    "C2-MiniLM-f16-L128-B32": ("all-MiniLM-L6-v2", "f16", [128] * 32, [0, 31]),
    "C4-bge-large-q4_1-L512-B32-shard": ("bge-large-en-v1.5", "q4_1", [512] * 32, [5]),
    "C5-bge-base-zh-q8_0-ragged-B128": ("bge-base-zh-v1.5", "q8_0",
                                        list(np.random.default_rng(11).integers(16, 513, 128)), None),
}


@pytest.mark.parametrize("cfg", list(SURVEY_CONFIGS))
def test_survey_config(tmp_path, cfg):
    arch, ftype, lens, check = SURVEY_CONFIGS[cfg]
    hp = bertpy.ARCHS[arch]
    path = str(tmp_path / f"{arch}-{ftype}.bin")
    bertpy.synthetic_model(path, arch, ftype, seed=1234)
    m = bertpy.BertModel(path)
    ids = bertpy.synthetic_ids(len(lens), lens, hp["n_vocab"], seed=7)
    full = m.forward_batch(ids)
    assert np.all(np.isfinite(full))
    assert np.allclose(np.linalg.norm(full, axis=1), 1.0, atol=1e-5)
    if check is None:                            # ragged: shortest and longest
        check = [int(np.argmin(lens)), int(np.argmax(lens))]
    sub = m.forward_batch([ids[i] for i in check])
    assert np.array_equal(sub, full[check])      # batch-composition invariance
    ref = oracle_lib.Oracle(path).forward_batch([ids[i] for i in check], n_threads=min(16, os.cpu_count() or 1))
    c = cosines(full[check], ref)
    print(cfg, "min cos vs oracle", c.min())
    assert np.all(c >= 1 - COS_TOL), c
    if arch == "bge-large-en-v1.5":
        # the library's in-process split (bert_abi.cpp run_forward) at C4 dims: two
        # replicas (BERT_DEVICES=0,0, own streams and workspaces) give the bits of one
        os.environ["BERT_DEVICES"] = "0,0"
        try:
            m2 = bertpy.BertModel(path)
            assert m2.lib.bertx_num_devices(m2.ctx) == 2
            two = m2.forward_batch(ids)
            split = [p[1] for p in m2.device_last_call()]
            del m2
        finally:
            os.environ["BERT_DEVICES"] = "0"
        assert split == [16, 16], split
        assert np.array_equal(two, full)


def _hip():
    """The HIP runtime libbert.so is linked against (libamdhip64.so.7 of /opt/rocm), by
    soname: the process already holds it, so this is the same runtime instance (torch
    bundles another one, which cannot share streams or pointers with it)."""
    import ctypes
    h = ctypes.CDLL("libamdhip64.so.7")
    vp = ctypes.c_void_p
    h.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    h.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    h.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
    h.hipStreamSynchronize.argtypes = [vp]
    h.hipFree.argtypes = [vp]
    h.hipStreamDestroy.argtypes = [vp]
    return h


def test_device_forward_on_caller_stream_is_ordered_before_host_forward(quant_models):
    """bertx_forward_device enqueues on the caller's stream and returns; a following
    bert_forward_batch (replica stream) must not overwrite the shared workspace
    while that forward is in flight (engine.cpp order_after_last / mark_done)."""
    import ctypes
    hip = _hip()
    path = quant_models[("tiny64", "q4_0")]
    m = bertpy.BertModel(path)
    ids = ragged_ids(690, [512, 300, 512, 129, 512, 77])
    other = ragged_ids(690, [511, 2, 400], seed=9)
    want = m.forward_batch(ids)
    want_other = m.forward_batch(other)
    flat = np.ascontiguousarray(np.concatenate(ids).astype(np.int32))
    cu = np.concatenate([[0], np.cumsum([len(x) for x in ids])]).astype(np.int32)
    T, B = int(cu[-1]), len(ids)
    d_ids, d_cu, d_out, s = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(d_ids), flat.nbytes) == 0
    assert hip.hipMalloc(ctypes.byref(d_cu), cu.nbytes) == 0
    assert hip.hipMalloc(ctypes.byref(d_out), B * m.n_embd * 4) == 0
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    assert hip.hipMemcpy(d_ids, flat.ctypes.data, flat.nbytes, 1) == 0     # H2D
    assert hip.hipMemcpy(d_cu, cu.ctypes.data, cu.nbytes, 1) == 0
    assert m.lib.bertx_reserve(m.ctx, 0, T, B) == 0
    out = np.zeros((B, m.n_embd), np.float32)
    for _ in range(3):                               # eager, then captured, then replayed
        assert m.lib.bertx_forward_device(m.ctx, 0, d_ids, d_cu, B, 512, T, d_out, s) == 0
        got_other = m.forward_batch(other)          # replica stream, issued while s may still run
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipMemcpy(out.ctypes.data, d_out, out.nbytes, 2) == 0   # D2H
        assert np.array_equal(out, want)
        assert np.array_equal(got_other, want_other)
    for p in (d_ids, d_cu, d_out):
        hip.hipFree(p)
    hip.hipStreamDestroy(s)


@pytest.fixture(scope="module")
def c4_model(tmp_path_factory):
    p = str(tmp_path_factory.mktemp("c4") / "bge-large-en-v1.5-q4_1.bin")
    bertpy.synthetic_model(p, "bge-large-en-v1.5", "q4_1", seed=1234)
    return p


def _replicas(path, n, monkeypatch):
    monkeypatch.setenv("BERT_DEVICES", ",".join(["0"] * n))
    m = bertpy.BertModel(path)
    assert m.lib.bertx_num_devices(m.ctx) == n
    return m


def test_c4_256_sentences_over_8_replicas(c4_model, monkeypatch):
    """SURVEY §8 C4 as specified: bge-large q4_1, L 512, 256 sentences through
    bert_forward_batch (reference entry bert.cpp:1374-1444) split by the library over
    8 replicas (BERT_DEVICES=0 x 8: 8 weight replicas, host threads, streams and
    workspaces on the one GPU, the code path an 8-GPU node takes).  32 sentences per
    slot, bitwise equal to one replica, 8 sentences against the oracle."""
    hp = bertpy.ARCHS["bge-large-en-v1.5"]
    ids = bertpy.synthetic_ids(256, 512, hp["n_vocab"], seed=7)
    one = bertpy.BertModel(c4_model).forward_batch(ids)
    assert np.all(np.isfinite(one))
    m8 = _replicas(c4_model, 8, monkeypatch)
    eight = m8.forward_batch(ids)
    per = m8.device_last_call()
    assert [p[1] for p in per] == [32] * 8, per
    assert [p[2] for p in per] == [32 * 512] * 8, per
    assert np.array_equal(eight, one)
    check = [0, 31, 32, 100, 128, 200, 254, 255]
    ref = oracle_lib.Oracle(c4_model).forward_batch([ids[i] for i in check], n_threads=min(16, os.cpu_count() or 1))
    c = cosines(eight[check], ref)
    print("C4 over 8 replicas: min cos vs oracle", c.min())
    assert np.all(c >= 1 - COS_TOL), c


def test_c5_ragged_over_8_replicas(tmp_path, monkeypatch):
    """C5 (bge-base-zh q8_0, ragged 16..512, 128 sentences) over 8 replicas: the
    call's ~33.8k tokens split into tokens // 8,192 = 4 shares (bert_abi.cpp
    kMinShareTokens, set from profiles/r05_share_curve.jsonl: smaller shares are
    launch-bound); the FLOP-cost split (longest-first to the least-loaded replica)
    gives the shares unequal token counts and different sentence lengths; every
    sentence is still bitwise as on one replica."""
    hp = bertpy.ARCHS["bge-base-zh-v1.5"]
    path = str(tmp_path / "bge-base-zh-q8_0.bin")
    bertpy.synthetic_model(path, "bge-base-zh-v1.5", "q8_0", seed=1234)
    lens = [int(x) for x in np.random.default_rng(11).integers(16, 513, 128)]
    ids = bertpy.synthetic_ids(128, lens, hp["n_vocab"], seed=7)
    one = bertpy.BertModel(path).forward_batch(ids)
    m8 = _replicas(path, 8, monkeypatch)
    eight = m8.forward_batch(ids)
    per = m8.device_last_call()
    counts = [p[1] for p in per]
    k = min(8, 128, sum(lens) // MIN_SHARE_TOKENS)
    assert sum(counts) == 128 and sum(c > 0 for c in counts) == k == 4, per
    toks = [p[2] for p in per if p[1] > 0]
    assert sum(toks) == sum(lens) and len(set(toks)) > 1, per   # ragged shards
    assert max(p[0] for p in per) > 0.0
    assert np.array_equal(eight, one)


def test_routing_small_calls_to_distinct_replicas(quant_models, monkeypatch):
    """Serving on several replicas (bert_abi.cpp run_forward routing): a
    call below 2 x 8,192 tokens goes whole to the least-loaded replica (ties rotate),
    so 4 sequential small calls use the 4 replicas once each, and 4 concurrent callers
    (ctypes releases the GIL) land on distinct replicas -- every reply bitwise equal to
    the single-replica result; a call of >= 4 x 8,192 tokens on idle replicas spreads
    over all 4 (bertx_device_calls counts the calls each replica ran)."""
    import threading
    path = quant_models[("tiny64", "q4_0")]
    batches = [ragged_ids(690, [5, 40, 129, 300], seed=s) for s in range(8)]
    monkeypatch.setenv("BERT_DEVICES", "0")
    one = bertpy.BertModel(path)
    want = [one.forward_batch(b) for b in batches]
    del one
    monkeypatch.setenv("BERT_DEVICES", "0,0,0,0")
    m4 = bertpy.BertModel(path)
    assert m4.lib.bertx_num_devices(m4.ctx) == 4

    def calls():
        return [m4.lib.bertx_device_calls(m4.ctx, i) for i in range(4)]

    c0 = calls()
    for b, w in zip(batches[:4], want[:4]):
        assert np.array_equal(m4.forward_batch(b), w)
    c1 = calls()
    assert [b - a for a, b in zip(c0, c1)] == [1, 1, 1, 1], (c0, c1)
    # concurrent: each of 4 threads sends its own small batches
    got = [None] * 8
    errors = []

    def client(k):
        try:
            for j in (k, k + 4):
                got[j] = m4.forward_batch(batches[j])
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    th = [threading.Thread(target=client, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    c2 = calls()
    assert sum(c2) - sum(c1) == 8 and all(b > a for a, b in zip(c1, c2)), (c1, c2)
    # a large call spreads: 64 sentences x 512 tokens = 32,768 tokens = 4 shares
    big = ragged_ids(690, [512] * 64, seed=21)
    monkeypatch.setenv("BERT_DEVICES", "0")
    ref = bertpy.BertModel(path).forward_batch(big)
    out = m4.forward_batch(big)
    c3 = calls()
    assert [b - a for a, b in zip(c2, c3)] == [1, 1, 1, 1], (c2, c3)
    assert [p[1] for p in m4.device_last_call()] == [16] * 4
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("stage", ["replica1", "worker"])
def test_injected_replica_failure_returns_null(quant_models, tmp_path, stage):
    """Round 5's driver run aborted inside bert_load_from_file with 4 replicas
    (DESIGN §11).  The load now runs every HIP call on the loading thread and turns
    every failure into a NULL context: BERT_FAULT_INJECT throws while the second
    replica is being made (`replica1`, after the first one's upload was issued) or
    while the replica workers start (`worker`, a std::system_error as from
    std::thread).  In a child process (an abort shows as its exit status): NULL,
    exit 0, the cause in BERT_LOG, and a normal 4-replica load in the same process
    afterwards works and runs a forward (the failed replicas were released)."""
    import subprocess
    import sys
    code = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np, os, bertpy
L = bertpy.load_lib()
ctx = L.bert_load_from_file(sys.argv[2].encode())
print("FIRST", "NULL" if not ctx else "OK", flush=True)
os.environ.pop("BERT_FAULT_INJECT")   # read per load stage: the next load is clean
m = bertpy.BertModel(sys.argv[2])
print("SECOND", m.lib.bertx_num_devices(m.ctx), flush=True)
e = m.forward_batch([np.arange(5, 40, dtype=np.int32)])
print("FWD", bool(np.isfinite(e).all()), flush=True)
"""
    log = tmp_path / "libbert.log"
    env = dict(os.environ, BERT_DEVICES="0,0,0,0", BERT_FAULT_INJECT=stage, BERT_LOG=str(log))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", code, os.path.join(root, "embeddings.cpp_amd"),
                        quant_models[("tiny64", "q4_0")]], capture_output=True, text=True, env=env, timeout=120)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out
    assert "FIRST NULL" in out, out
    text = log.read_text()
    assert f"BERT_FAULT_INJECT={stage}" in text, text
    assert "SECOND 4" in out and "FWD True" in out, out


@pytest.mark.parametrize("ftype", ["q4_0", "q4_1", "q8_0"])
def test_short_sentences_bitwise_across_tile_forms(tmp_path, ftype):
    """A short sentence alone (64 GEMM rows: the small-batch tile form 16, wave-private
    X rings) has the bits it has inside a large batch (256- and 128-row tiles), for
    every quantized format at MiniLM dims (d 384, 12 heads of 32; the dh-64 short
    attention kernel has its own bitwise test, test_short_attention_bitwise_equal_to_lds3).
    Round 6 also ran an f16 expansion of the QKV / FFN-up weights for the small
    form under this test (bitwise, but slower: profiles/r06_small_f16_expansion_ab.log)."""
    path = str(tmp_path / f"minilm-{ftype}.bin")
    bertpy.synthetic_model(path, "all-MiniLM-L6-v2", ftype, seed=1234)
    m = bertpy.BertModel(path)
    short = ragged_ids(30522, [5, 32, 60], seed=8)
    big = ragged_ids(30522, [512] * 16, seed=9)
    full = m.forward_batch(short + big)
    for i, s in enumerate(short):
        assert np.array_equal(m.forward_batch([s])[0], full[i]), (ftype, len(s))
    assert np.array_equal(m.forward_batch(short), full[:3])


@pytest.mark.parametrize("arch,ftype,n", [("all-MiniLM-L6-v2", "f16", 16), ("bge-base-en-v1.5", "q4_0", 8)])
def test_mid_batch_tile_forms_bitwise(tmp_path, arch, ftype, n):
    """Mid-size batches (1-2k GEMM rows) take 128 x 128 tiles once those cover half the
    CUs (gemm.hip pick_cfg), with the statistics fold in its one-workgroup-per-CU
    24-group form at d 768: every sentence keeps the bits it has alone (64-row tile
    forms) and in a pair, and the batch is within the cosine bound of the oracle."""
    hp = bertpy.ARCHS[arch]
    path = str(tmp_path / f"{arch}-{ftype}.bin")
    bertpy.synthetic_model(path, arch, ftype, seed=1234)
    m = bertpy.BertModel(path)
    ids = ragged_ids(hp["n_vocab"], [128] * n, seed=12)
    full = m.forward_batch(ids)
    assert np.all(np.isfinite(full))
    for i in (0, n // 2, n - 1):
        assert np.array_equal(m.forward_batch([ids[i]])[0], full[i]), (arch, i)
    assert np.array_equal(m.forward_batch(ids[:2]), full[:2])
    ref = oracle_lib.Oracle(path).forward_batch(ids[:2], n_threads=min(16, os.cpu_count() or 1))
    assert np.all(cosines(full[:2], ref) >= 1 - COS_TOL)


def test_load_free_cycles_multi_replica(quant_models, monkeypatch):
    """The load path that aborted on round 5's driver box, exercised repeatedly: ten
    cycles of a 4-replica context on one GPU (load, a small forward on the routed
    replica, free), each bitwise the single-replica result.  Every HIP call of a
    load now runs on the loading thread."""
    path = quant_models[("tiny64", "q8_0")]
    ids = ragged_ids(690, [7, 64, 200], seed=12)
    monkeypatch.setenv("BERT_DEVICES", "0")
    want = bertpy.BertModel(path).forward_batch(ids)
    monkeypatch.setenv("BERT_DEVICES", "0,0,0,0")
    for _ in range(10):
        m = bertpy.BertModel(path)
        assert m.lib.bertx_num_devices(m.ctx) == 4
        assert np.array_equal(m.forward_batch(ids), want)
        del m
