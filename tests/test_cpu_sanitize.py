"""ASan + UBSan runs of the host C++ (tokenizer, model-file loader, quantizer, converter)
and of the C oracle, as standalone programs built by tests/sanitize/Makefile (SURVEY §5:
sanitizers on host code only; GPU sanitizers are unavailable on this pool).  Each run
must exit 0 with no sanitizer report and give the same results as the production build."""
import fcntl
import os
import random
import struct
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from test_cpu_abi import _parse_model_file, _write_hf_dir

SAN = os.path.join(ROOT, "tests", "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def harness():
    # one build at a time: pytest-xdist workers each run this fixture, and a worker
    # must not exec a harness another worker's make is still linking
    with open(os.path.join(SAN, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", SAN, "-j2"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return os.path.join(SAN, "_build")


def run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, env=ENV, timeout=600)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    return r.stdout


def write_blobs(path, blobs, with_nmax=None):
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(blobs)))
        for i, b in enumerate(blobs):
            if with_nmax is not None:
                f.write(struct.pack("<i", with_nmax[i]))
            f.write(struct.pack("<I", len(b)))
            f.write(b)


def read_ids(path, n_max):
    out, data, o = [], open(path, "rb").read(), 0
    for nm in n_max:
        (n,) = struct.unpack_from("<i", data, o)
        o += 4
        w = min(n, nm)
        out.append((n, list(struct.unpack_from("<%di" % w, data, o)) if w > 0 else []))
        o += 4 * max(w, 0)
    assert o == len(data)
    return out


def random_texts(n, seed):
    """ASCII, punctuation, accents, CJK, emoji and invalid UTF-8 bytes."""
    rnd = random.Random(seed)
    pieces = [b"hello", b"World", b" ", b"  ", b"\t", b"\n", b"!", b"?", b"x!x", b"caf\xc3\xa9", b"\xc3\x80",
              b"\xe4\xb8\xad\xe6\x96\x87", b"\xe3\x80\x82", b"\xef\xbc\x8c", b"\xf0\x9f\x98\x80", b"\xff", b"\xc3",
              b"##", b"w12", b"w3", b"[UNK]", b"a" * 700]
    return [b"".join(rnd.choice(pieces) for _ in range(rnd.randint(0, 40))) for _ in range(n)]


def test_tokenizer_under_sanitizers(harness, tmp_path, tok_golden, lib, monkeypatch):
    vocab = [v.encode("utf-8") for v in tok_golden["vocab"]]
    cases = tok_golden["cases"]
    texts = [bytes.fromhex(c["text_hex"]) for c in cases]
    n_max = [c["n_max_tokens"] for c in cases]
    extra = random_texts(200, 3)
    texts += extra
    n_max += [random.Random(i).choice([1, 2, 8, 64, 512]) for i in range(len(extra))]
    write_blobs(tmp_path / "vocab.bin", vocab)
    write_blobs(tmp_path / "texts.bin", texts, n_max)
    run(os.path.join(harness, "host_harness"), "tok", tmp_path / "vocab.bin", tmp_path / "texts.bin",
        tmp_path / "ids.bin")
    got = read_ids(tmp_path / "ids.bin", n_max)
    for c, (n, ids) in zip(cases, got):
        assert n == len(c["ids"]) and ids == c["ids"][: c["n_max_tokens"]]
    # the random texts: same ids as the production library's tokenizer
    import bertpy
    monkeypatch.setenv("BERT_HOST_ONLY", "1")
    m = bertpy.BertModel(os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin"))
    write_blobs(tmp_path / "vocab2.bin", [m.id_to_token(i) for i in range(m.hparams()[0])])
    write_blobs(tmp_path / "texts2.bin", extra, n_max[len(cases):])
    run(os.path.join(harness, "host_harness"), "tok", tmp_path / "vocab2.bin", tmp_path / "texts2.bin",
        tmp_path / "ids2.bin")
    for t, nm, (n, ids) in zip(extra, n_max[len(cases):], read_ids(tmp_path / "ids2.bin", n_max[len(cases):])):
        ref, rn = m.tokenize(t, nm)
        assert (n, ids) == (rn, ref[:nm])


@pytest.mark.parametrize("tiny", ["tiny32", "tiny64"])
def test_loader_quantizer_under_sanitizers(harness, tmp_path, lib, tiny):
    exe = os.path.join(harness, "host_harness")
    src = os.path.join(GOLDEN, tiny, "ggml-model-f16.bin")
    for ft in ("f32", "f16"):
        run(exe, "load", os.path.join(GOLDEN, tiny, f"ggml-model-{ft}.bin"))
    for it in (2, 3, 8):
        out = tmp_path / f"q{it}.bin"
        run(exe, "quant", src, out, it)
        ref = tmp_path / f"ref{it}.bin"
        assert lib.bertx_quantize_file(src.encode(), str(ref).encode(), it) == 0
        assert open(out, "rb").read() == open(ref, "rb").read()
        hp = run(exe, "load", out).split()
        assert int(hp[6]) == it
    # a truncated file is refused cleanly (no out-of-bounds read)
    data = open(src, "rb").read()
    (tmp_path / "trunc.bin").write_bytes(data[: len(data) // 2])
    r = subprocess.run([exe, "load", str(tmp_path / "trunc.bin")], capture_output=True, text=True, env=ENV)
    assert r.returncode == 5 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_converter_under_sanitizers(harness, tmp_path):
    ref32 = os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin")
    hp, vocab, tens = _parse_model_file(ref32)
    d = str(tmp_path / "hf")
    _write_hf_dir(d, hp, vocab, tens, prefix="bert.", shards=2)
    for ft, fn in ((0, "ggml-model-f32.bin"), (1, "ggml-model-f16.bin")):
        out = tmp_path / fn
        run(os.path.join(harness, "host_harness"), "convert", d, out, ft)
        assert open(out, "rb").read() == open(os.path.join(GOLDEN, "tiny32", fn), "rb").read()


def test_oracle_under_sanitizers(harness, tmp_path, oracle):
    path = os.path.join(GOLDEN, "tiny64", "ggml-model-f32.bin")
    o = oracle.Oracle(path)
    rng = np.random.default_rng(4)
    lens = [1, 2, 17, 64, o.n_max_tokens]
    ids = [np.concatenate([[101], rng.integers(104, o.n_vocab, max(L - 2, 0)), [102]])[:L].astype(np.int32)
           for L in lens]
    with open(tmp_path / "ids.bin", "wb") as f:
        f.write(struct.pack("<I", len(ids)))
        for x in ids:
            f.write(struct.pack("<I", len(x)))
            f.write(x.tobytes())
    run(os.path.join(harness, "oracle_harness"), "fwd", path, tmp_path / "ids.bin", tmp_path / "out.bin")
    got = np.fromfile(tmp_path / "out.bin", np.float32).reshape(len(ids), -1)
    ref = o.forward_batch(ids)
    assert np.allclose(got, ref, rtol=0, atol=1e-6)
