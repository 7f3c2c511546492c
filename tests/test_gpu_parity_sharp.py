"""BASELINE-size parity of the HIP forward with the CPU oracle on "sharp" weights.

The bench's weights (SURVEY §8d, N(0, 0.02)) make attention almost uniform, so a
key permutation or a masking error barely moves the output.  These tests use
bertpy.synthetic_tensors(profile="sharp"): peaked softmax rows in every layer,
LN gains spread 4*(1+N(0,0.3)) and three residual outlier channels at |x| ~ 100
in the f16 pre-LN residual stream (the regime where an f16 residual could fail).

Every SURVEY §8 configuration runs at full shape on the GPU through the C ABI:
C1 MiniLM f32 L32 B1, C2 MiniLM f16 L128 B32, C3 bge-base q4_0 L512 B64, C4
bge-large q4_1 L512 B32 (one GPU's shard of 256 over 8), C5 bge-base-zh q8_0
ragged 16..512 B128.  Every sentence of each batch (C4: 16 of the 32) is
compared with the oracle (oracle/bert_oracle.c, restating bert.cpp:827-1147) at
the north-star tolerance (1e-3 cosine).  The reference's
own q8 activation rounding moves sharp bge-base embeddings by up to 1.5e-4
cosine against the same weights with f32 activations (oracle vs oracle), and
3.4e-4 on a 3-token bge-large sentence, which is why the tolerance is not
tighter (bge-large's Q/K spread is lower: at the bge-base value 24 peaked layers
make the reference disagree with itself at 0.88 cosine).

PARITY_LOG=<file>: each test appends {config, min_cos, n} as one JSON line.
"""
import json
import os

import numpy as np
import pytest

import bertpy
import oracle_lib

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3
N_THR = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module", autouse=True)
def _one_device():
    os.environ.pop("BERT_HOST_ONLY", None)
    os.environ["BERT_DEVICES"] = "0"


@pytest.fixture(scope="module")
def sharp_models(tmp_path_factory):
    d = tmp_path_factory.mktemp("sharp")
    cache = {}

    def get(arch, ftype, profile="sharp"):
        if (arch, ftype, profile) not in cache:
            p = str(d / f"{arch}-{ftype}-{profile}.bin")
            bertpy.synthetic_model(p, arch, ftype, seed=1234, profile=profile)
            cache[(arch, ftype, profile)] = p
        return cache[(arch, ftype, profile)]
    return get


def cosines(a, b):
    return np.sum(a * b, axis=1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))


def record(cfg, c):
    log = os.environ.get("PARITY_LOG")
    print(cfg, "min cos vs oracle %.7f over %d sentences" % (float(np.min(c)), len(c)))
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"config": cfg, "min_cos": float(np.min(c)), "n": int(len(c))}) + "\n")


def pick8(lens):
    """Eight indices: the shortest, the longest, and six spread over the batch."""
    lens = np.asarray(lens)
    idx = [int(np.argmin(lens))]
    if int(np.argmax(lens)) not in idx:
        idx.append(int(np.argmax(lens)))
    for i in np.linspace(0, len(lens) - 1, 8).astype(int):
        if len(idx) < 8 and int(i) not in idx:
            idx.append(int(i))
    i = 0
    while len(idx) < min(8, len(lens)):
        if i not in idx:
            idx.append(i)
        i += 1
    return idx


# config -> (arch, ftype, lengths, sentences compared with the oracle: None = all)
SHARP_CONFIGS = {
    "C2-MiniLM-f16-L128-B32": ("all-MiniLM-L6-v2", "f16", [128] * 32, None),
    "C3-bge-base-q4_0-L512-B64": ("bge-base-en-v1.5", "q4_0", [512] * 64, None),
    "C4-bge-large-q4_1-L512-B32-shard": ("bge-large-en-v1.5", "q4_1", [512] * 32, 16),
    "C5-bge-base-zh-q8_0-ragged-B128": ("bge-base-zh-v1.5", "q8_0",
                                        [int(x) for x in np.random.default_rng(11).integers(16, 513, 128)], None),
}


def oracle_rows(o, ids, idx):
    """Oracle embeddings of ids[i] for i in idx, in groups of similar length (the
    oracle pads a batch to its longest sentence, as bert.cpp:837-843 does)."""
    order = sorted(idx, key=lambda i: len(ids[i]))
    out = {}
    for g in range(0, len(order), 8):
        grp = order[g:g + 8]
        for i, e in zip(grp, o.forward_batch([ids[i] for i in grp], n_threads=N_THR)):
            out[i] = e
    return np.stack([out[i] for i in idx])


@pytest.mark.parametrize("cfg", list(SHARP_CONFIGS))
def test_sharp_config_matches_oracle(sharp_models, cfg):
    arch, ftype, lens, n_cmp = SHARP_CONFIGS[cfg]
    hp = bertpy.ARCHS[arch]
    path = sharp_models(arch, ftype)
    m = bertpy.BertModel(path)
    ids = bertpy.synthetic_ids(len(lens), lens, hp["n_vocab"], seed=7)
    full = m.forward_batch(ids)
    assert np.all(np.isfinite(full))
    assert np.allclose(np.linalg.norm(full, axis=1), 1.0, atol=1e-5)
    check = pick8(lens)
    sub = m.forward_batch([ids[i] for i in check])
    assert np.array_equal(sub, full[check])          # batch-composition invariance
    # oracle parity on every sentence of the batch (C4: the first 16 of its shard)
    cmp_idx = list(range(len(lens) if n_cmp is None else n_cmp))
    for i in check:
        if i not in cmp_idx:
            cmp_idx.append(i)
    c = cosines(full[cmp_idx], oracle_rows(oracle_lib.Oracle(path), ids, cmp_idx))
    record(cfg, c)
    assert np.all(c >= 1 - COS_TOL), c
    # the sentences differ from each other (sharp weights: no collapse to one vector)
    g = full[check] @ full[check].T
    assert np.max(g[~np.eye(len(check), dtype=bool)]) < 0.999


def test_sharp_c1_minilm_f32_single(sharp_models):
    """C1: all-MiniLM-L6-v2 f32, L = 32, B = 1 (bert_forward, a batch of one), plus
    seven more single-sentence calls of lengths 1..32, at 1 - cos <= 1e-6 (f32 chain)."""
    path = sharp_models("all-MiniLM-L6-v2", "f32")
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    lens = [32, 1, 2, 5, 16, 31, 3, 32]
    ids = bertpy.synthetic_ids(len(lens), lens, 30522, seed=7)
    got = np.stack([m.forward(x) for x in ids])
    ref = np.concatenate([o.forward_batch([x], n_threads=N_THR) for x in ids])
    c = cosines(got, ref)
    record("C1-MiniLM-f32-L32-B1", c)
    # f32 files run the f32 chain (f32 x f32 as the reference): an absolute f32-grade bound
    assert np.all(c >= 1 - 1e-6), 1.0 - c
    # and the whole C1 batch of eight through one bert_forward_batch call, bitwise
    assert np.array_equal(m.forward_batch(ids), got)


def test_sharp_fake_batch_matches_oracle(sharp_models):
    """bert_forward_fake_batch (bert.cpp:1151-1363: one graph per sentence, no mask,
    pool 1/N, scale by 1/|e|) against the oracle's restatement of that path
    (oracle_forward_fake_batch), and its write pattern when an input is too long:
    the sentences before the first over-long one are written, the rest are not."""
    path = sharp_models("bge-base-zh-v1.5", "q8_0")
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    lens = [16, 512, 77, 300, 2, 129, 450, 33]
    ids = bertpy.synthetic_ids(len(lens), lens, 21128, seed=9)
    got = m.forward_batch(ids, fake=True)
    ref = o.forward_fake_batch(ids, n_threads=N_THR)
    c = cosines(got, ref)
    record("fake-batch-bge-base-zh-q8_0", c)
    assert np.all(c >= 1 - COS_TOL), c
    one = m.forward(ids[3])                          # bert_forward: a batch of one
    assert cosines(one[None], ref[3:4])[0] >= 1 - COS_TOL
    long_ = ids[:3] + [np.full(513, 1000, np.int32)] + ids[3:5]
    out = m.forward_batch(long_, fake=True, fill=7.0)
    assert not np.any(out[:3] == 7.0)
    assert np.all(out[3:] == 7.0)
    assert o.forward_fake_batch(long_, n_threads=N_THR) is None    # the oracle refuses too
    assert np.array_equal(out[:3], got[:3])



def test_sharp_large_row_mean(sharp_models):
    """The LN fold stores the pre-LN stream as z = f16(y * gamma), whose rounding
    scales with |y| rather than |y - mean|: rows with a large common offset are its
    worst case.  profile "sharp_mean" adds +16 to every channel of the O-proj and
    FFN-down biases (residual rows with mean ~16 against a spread of a few units)
    at C3 dims; 16 sentences against the oracle at the north-star bound, the
    minimum cosine recorded."""
    path = sharp_models("bge-base-en-v1.5", "q4_0", "sharp_mean")
    m = bertpy.BertModel(path)
    lens = [512, 3, 200, 511, 17, 64, 129, 300, 512, 40, 2, 450, 128, 256, 77, 500]
    ids = bertpy.synthetic_ids(len(lens), lens, 30522, seed=13)
    got = m.forward_batch(ids)
    c = cosines(got, oracle_rows(oracle_lib.Oracle(path), ids, list(range(len(lens)))))
    record("C3-dims-q4_0-large-row-mean", c)
    assert np.all(c >= 1 - COS_TOL), c


@pytest.mark.parametrize("qk", [0.03, 0.05])
def test_q8_activation_envelope_c4(tmp_path, qk):
    """Which arithmetic the HIP path tracks.  C4 dims
    (bge-large q4_1, 24 layers, sharp weights) with the Q/K spread raised to `qk`:
    peaked attention over 24 layers amplifies any activation rounding.  Three forwards
    of the same sentences: HIP (f16 activations), the oracle in the reference's
    arithmetic (q8_0 / q8_1 re-quantized activations, bert.cpp:995) and the oracle
    with f32 activations (oracle_forward_batch_ex's act_f32, the diagnostic mode).
      qk 0.03: HIP within 1e-4 cosine of the f32-activation forward, while the
               reference's own q8 rounding already moves it by up to 5.7e-3
               (profiles/r05_q8_envelope.jsonl);
      qk 0.05: the model is chaotic -- the reference arithmetic sits at 0.85 cosine
               from its own f32-activation forward -- so a per-sentence ordering
               would be coincidental; asserted on the aggregate: HIP's
               mean 1 - cos to the f32-activation forward is within 1.25x of the
               reference arithmetic's (recorded per sentence, not gated).
    The north-star bound (1e-3 against the reference) is met where the reference
    agrees with itself to 1e-3 (qk 0.02 for bge-large: test_sharp_config_matches_oracle)."""
    path = str(tmp_path / f"bge-large-q4_1-qk{qk}.bin")
    bertpy.synthetic_model(path, "bge-large-en-v1.5", "q4_1", seed=1234, profile="sharp", qk_std=qk)
    lens = [3, 64, 300, 512]
    ids = bertpy.synthetic_ids(len(lens), lens, 30522, seed=7)
    hip = bertpy.BertModel(path).forward_batch(ids)
    o = oracle_lib.Oracle(path)
    q8 = np.concatenate([o.forward_batch([x], n_threads=N_THR) for x in ids])
    f32 = np.concatenate([o.forward_batch([x], n_threads=N_THR, activations="f32") for x in ids])
    c_hf, c_qf, c_hq = cosines(hip, f32), cosines(q8, f32), cosines(hip, q8)
    record(f"C4-dims-envelope-qk{qk}-hip_vs_f32", c_hf)
    record(f"C4-dims-envelope-qk{qk}-q8_vs_f32", c_qf)
    record(f"C4-dims-envelope-qk{qk}-hip_vs_q8", c_hq)
    if qk <= 0.03:
        assert np.all(c_hf >= 1 - 1e-4), c_hf
        assert np.all(c_hf >= c_qf), (c_hf, c_qf)
    else:
        assert np.mean(1 - c_hf) <= 1.25 * np.mean(1 - c_qf), (c_hf, c_qf)


TORCH_CONFIGS = {
    "C2-MiniLM-f16": ("all-MiniLM-L6-v2", "f16", [128, 128, 3, 77]),
    "C3-bge-base-q4_0": ("bge-base-en-v1.5", "q4_0", [512, 3, 77, 300, 512, 129]),
    "C4-bge-large-q4_1": ("bge-large-en-v1.5", "q4_1", [512, 3, 200]),
    "C5-bge-base-zh-q8_0": ("bge-base-zh-v1.5", "q8_0", [16, 511, 250, 90]),
}


@pytest.mark.parametrize("cfg", list(TORCH_CONFIGS))
def test_hip_vs_torch_f32_activations(tmp_path, cfg):
    """An independent cross-check of the HIP path that does not go through the oracle:
    each SURVEY architecture and weight format on sharp weights against
    transformers' BertModel on the file's dequantized weights with f32 activations
    (tests/test_cpu_oracle.py _torch_forward: era constants, masked mean pool, L2
    norm), ragged lengths up to 512.  The HIP path (f16 activations) tracks that
    f32-activation forward to 1e-4 in cosine."""
    import torch
    from test_cpu_oracle import _model_tensors, _torch_forward
    torch.set_num_threads(N_THR)
    arch, ftype, lens = TORCH_CONFIGS[cfg]
    hp_arch = bertpy.ARCHS[arch]
    path = str(tmp_path / f"{arch}-{ftype}-sharp.bin")
    bertpy.synthetic_model(path, arch, ftype, seed=1234, profile="sharp")
    ids = bertpy.synthetic_ids(len(lens), lens, hp_arch["n_vocab"], seed=17)
    hip = bertpy.BertModel(path).forward_batch(ids)
    hp, tensors = _model_tensors(oracle_lib, path)
    ref = _torch_forward(hp, tensors, ids)
    c = cosines(hip, ref)
    record(f"{cfg}-hip_vs_torch_f32", c)
    assert np.all(c >= 1 - 1e-4), c
