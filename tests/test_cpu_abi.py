"""CPU tests of the product library's boundary (no GPU compute):

  * libbert.so loads and exports every function include/*.h declares;
  * without a HIP device bert_load_from_file fails loudly (no CPU compute path);
  * the host side behind the ABI -- model-file loader, tokenizer, quantizer --
    in a tokenizer-only context (BERT_HOST_ONLY=1), checked bit-exact against
    the reference's golden token ids and the oracle's quantizer bytes.
"""
import ctypes
import glob
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from test_cpu_oracle import expected_id_to_token

HAS_GPU_NODE = os.path.exists("/dev/kfd")


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\b((?:bert|bertx|ggml)_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert {"bert_load_from_file", "bert_encode_batch", "bert_forward_batch", "bert_tokenize",
            "bertx_forward_device", "ggml_time_us"} <= names
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "build", "libbert.so")],
                        capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    assert names <= exported, names - exported
    # nothing but the ABI leaks out (hidden visibility for everything else)
    assert {n for n in exported if not n.startswith(("bert", "ggml_"))} <= {"_init", "_fini"}


@pytest.mark.parametrize("checker", ["check_drain.py", "check_asm_loads.py"])
def test_code_object_checks(lib, checker):
    """The shipped gfx950 code objects, disassembled: every GEMM / attention kernel
    drains its hand-counted asm LDS reads before the epilogue (check_drain, round 3's
    fault class), and attention_pp touches no Q register while its asm Q loads are
    in flight (check_asm_loads)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", checker),
                        os.path.join(ROOT, "build", "libbert.so")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_asm_load_checker_catches_the_hazard():
    """check_asm_loads' rule on hand-written sequences: the hipcc copy that round 6
    met (a v_mov of a pending Q register in front of the tied wait) and an address
    taken from a pending destination are caught; the shipped shape passes."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import check_asm_loads as c
    loads = ["global_load_dwordx4 v[14:17], v[2:3], off", "v_lshl_add_u64 v[4:5], v[2:3], 0, 32",
             "global_load_dwordx4 v[10:13], v[4:5], off", "global_load_dwordx4 v[6:9], v[4:5], off",
             "global_load_dwordx4 v[2:5], v[2:3], off"]
    wait = ["s_waitcnt vmcnt(4)"]
    assert c.check(loads + ["v_mov_b32_e32 v20, s1"] + wait) is None
    assert c.check(loads + ["v_mov_b64_e32 v[32:33], v[14:15]"] + wait) is not None
    bad_addr = ["global_load_dwordx4 v[14:17], v[2:3], off", "global_load_dwordx4 v[10:13], v[14:15], off",
                "global_load_dwordx4 v[6:9], v[4:5], off", "global_load_dwordx4 v[2:5], v[4:5], off"]
    assert c.check(bad_addr + wait) is not None


def test_version_and_time(lib):
    v = lib.bertx_version().decode()
    assert "gfx950" in v
    t0 = lib.ggml_time_us()
    t1 = lib.ggml_time_us()
    assert t1 >= t0 >= 0


@pytest.mark.skipif(HAS_GPU_NODE, reason="checks the no-device failure path")
def test_load_without_device_fails_loudly(lib, monkeypatch):
    monkeypatch.delenv("BERT_HOST_ONLY", raising=False)
    ctx = lib.bert_load_from_file(os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin").encode())
    assert not ctx


@pytest.fixture
def host_model(lib, monkeypatch):
    import bertpy
    monkeypatch.setenv("BERT_HOST_ONLY", "1")
    m = bertpy.BertModel(os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin"), lib=lib)
    yield m
    del m


def test_host_context_metadata(host_model, tok_golden):
    assert host_model.n_embd == 64 and host_model.n_max_tokens == 128
    n_vocab, n_max, d, f, h, nl, ftype = host_model.hparams()
    assert (n_vocab, n_max, d, f, h, nl, ftype) == (len(tok_golden["vocab"]), 128, 64, 128, 2, 2, 0)
    assert host_model.lib.bertx_num_devices(host_model.ctx) == 0
    exp = expected_id_to_token(tok_golden["vocab"])
    assert [host_model.id_to_token(i).decode() for i in range(len(exp))] == exp


def test_host_tokenizer_matches_reference_goldens(host_model, tok_golden):
    """Token ids bit-exact.  The reference's n_max_tokens is checked only between
    words (bert.cpp:386), so its count can exceed it (it then writes past the
    caller's buffer); the product reports the same count but never writes past
    n_max_tokens, so the written prefix is compared."""
    bad, over = [], 0
    for c in tok_golden["cases"]:
        ids, n = host_model.tokenize(bytes.fromhex(c["text_hex"]), c["n_max_tokens"])
        g = c["ids"]
        over += n > c["n_max_tokens"]
        if n != len(g) or ids != g[: c["n_max_tokens"]]:
            bad.append((bytes.fromhex(c["text_hex"])[:30], n, len(g), ids[:8], g[:8]))
    assert not bad, bad[:5]
    assert over > 0     # the goldens do exercise the overflow quirk


def test_host_tokenizer_matches_oracle_on_random_text(host_model, oracle):
    """Random UTF-8 mixes (ASCII, punctuation, accents, CJK, invalid bytes)."""
    orc = oracle.Oracle(os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin"))
    rng = np.random.default_rng(3)
    alphabet = list("abcdefghijklmnopqrstuvwxyz     ,.!?'-0123456789") + ["é", "Ü", "ß", "中", "日", "本", "\t",
                                                                          "\n", "ﬁ", "Æ", "##"]
    for i in range(300):
        n = int(rng.integers(0, 80))
        s = "".join(alphabet[j] for j in rng.integers(0, len(alphabet), n)).encode()
        if i % 10 == 0:
            s += bytes([0xff, 0xc3])           # invalid / truncated UTF-8 tail
        for n_max in (128, 7):
            ids, n = host_model.tokenize(s, n_max)
            ref = orc.tokenize(s, n_max)
            assert n == len(ref) and ids == ref[:n_max], (s, n_max)


def test_host_forward_refused(host_model):
    """A tokenizer-only context has no compute path: forward leaves outputs alone."""
    out = host_model.forward_batch([[101, 150, 102]], fill=7.0)
    assert np.all(out == 7.0)


@pytest.mark.parametrize("bad", ["missing", "empty", "magic", "truncated"])
def test_bad_model_files(lib, tmp_path, monkeypatch, bad):
    monkeypatch.setenv("BERT_HOST_ONLY", "1")
    src = open(os.path.join(GOLDEN, "tiny32", "ggml-model-f16.bin"), "rb").read()
    p = tmp_path / "m.bin"
    if bad == "empty":
        p.write_bytes(b"")
    elif bad == "magic":
        p.write_bytes(b"\0\0\0\0" + src[4:])
    elif bad == "truncated":
        p.write_bytes(src[: len(src) // 2])
    assert not lib.bert_load_from_file(str(p).encode())


@pytest.mark.parametrize("itype", [2, 3, 8])
@pytest.mark.parametrize("tiny,src", [("tiny32", "f32"), ("tiny64", "f16")])
def test_quantizer_bytes_match_oracle(lib, oracle, tmp_path, tiny, src, itype):
    """bertx_quantize_file (and the quantize CLI) == the oracle quantizer, byte for byte."""
    fin = os.path.join(GOLDEN, tiny, f"ggml-model-{src}.bin")
    a, b, c = str(tmp_path / "prod.bin"), str(tmp_path / "orc.bin"), str(tmp_path / "cli.bin")
    assert lib.bertx_quantize_file(fin.encode(), a.encode(), itype) == 0
    assert oracle.quantize_file(fin, b, itype) == 0
    assert open(a, "rb").read() == open(b, "rb").read()
    cli = os.path.join(ROOT, "build", "bin", "quantize")
    if os.path.exists(cli):
        r = subprocess.run([cli, fin, c, str(itype)], capture_output=True)
        assert r.returncode == 0
        assert open(c, "rb").read() == open(b, "rb").read()


def test_quantizer_rejects_bad_type(lib, tmp_path):
    fin = os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin")
    assert lib.bertx_quantize_file(fin.encode(), str(tmp_path / "x.bin").encode(), 5) != 0
    assert lib.bertx_quantize_file(b"/nonexistent/model.bin", str(tmp_path / "y.bin").encode(), 2) != 0
    cli = os.path.join(ROOT, "build", "bin", "quantize")
    if os.path.exists(cli):
        assert subprocess.run([cli], capture_output=True).returncode != 0


def test_quantized_file_loads_in_host_context(lib, tmp_path, monkeypatch):
    import bertpy
    monkeypatch.setenv("BERT_HOST_ONLY", "1")
    q = str(tmp_path / "q.bin")
    assert lib.bertx_quantize_file(os.path.join(GOLDEN, "tiny64", "ggml-model-f16.bin").encode(), q.encode(), 2) == 0
    m = bertpy.BertModel(q, lib=lib)
    assert m.hparams()[6] == 2 and m.n_embd == 64


def test_synthetic_model_writer_roundtrip(lib, oracle, tmp_path, monkeypatch):
    """bertpy's reference-format writer (bench / tests) produces files both the
    product loader and the oracle accept with the same header."""
    import bertpy
    monkeypatch.setenv("BERT_HOST_ONLY", "1")
    hp = dict(n_vocab=300, n_max_tokens=64, n_embd=64, n_intermediate=128, n_head=2, n_layer=1)
    p = str(tmp_path / "syn.bin")
    bertpy.write_model(p, hp, bertpy.synthetic_vocab(300), bertpy.synthetic_tensors(hp), 1)
    m = bertpy.BertModel(p, lib=lib)
    o = oracle.Oracle(p)
    assert m.hparams()[:6] == [o.n_vocab, o.n_max_tokens, o.n_embd, o.n_intermediate, o.n_head, o.n_layer]
    assert m.hparams()[:6] == [300, 64, 64, 128, 2, 1]
    assert ctypes.sizeof(ctypes.c_int32) == 4


# ---- native converter vs the reference converter's committed output ----

def _parse_model_file(path):
    """-> (hparams[7], vocab list of bytes, [(name, np.ndarray f32 in torch shape)])."""
    import struct
    b = open(path, "rb").read()
    hp = struct.unpack("8i", b[:32])[1:]
    o, vocab = 32, []
    for _ in range(hp[0]):
        n = struct.unpack("i", b[o:o + 4])[0]
        vocab.append(b[o + 4:o + 4 + n])
        o += 4 + n
    tens = []
    while o < len(b):
        nd, nl, ft = struct.unpack("3i", b[o:o + 12])
        o += 12
        ne = struct.unpack("%di" % nd, b[o:o + 4 * nd])
        o += 4 * nd
        name = b[o:o + nl].decode()
        o += nl
        cnt = int(np.prod(ne)) if nd else 1
        dt = np.float32 if ft == 0 else np.float16
        a = np.frombuffer(b, dt, cnt, o).astype(np.float32).reshape(tuple(reversed(ne)))
        o += cnt * np.dtype(dt).itemsize
        tens.append((name, a))
    return hp, vocab, tens


def _write_hf_dir(d, hp, vocab, tens, prefix="", extra=True, shards=1):
    import json as _json
    from safetensors.numpy import save_file
    os.makedirs(d, exist_ok=True)
    cfg = dict(vocab_size=hp[0], max_position_embeddings=hp[1], hidden_size=hp[2], intermediate_size=hp[3],
               num_attention_heads=hp[4], num_hidden_layers=hp[5], model_type="bert", layer_norm_eps=1e-12)
    with open(os.path.join(d, "config.json"), "w") as f:
        _json.dump(cfg, f)
    with open(os.path.join(d, "vocab.txt"), "wb") as f:
        f.write(b"".join(v + b"\n" for v in vocab))
    t = {prefix + n: np.ascontiguousarray(a) for n, a in tens}
    if extra:   # what BertModel checkpoints also hold; the reference skips them (convert-to-ggml.py:86-87)
        t[prefix + "pooler.dense.weight"] = np.zeros((hp[2], hp[2]), np.float32)
        t[prefix + "pooler.dense.bias"] = np.zeros((hp[2],), np.float32)
        t[prefix + "embeddings.position_ids"] = np.arange(hp[1], dtype=np.float32)[None]
    names = sorted(t)
    if shards == 1:
        save_file(t, os.path.join(d, "model.safetensors"))
    else:
        wm = {}
        for s in range(shards):
            part = {n: t[n] for n in names[s::shards]}
            fn = "model-%05d-of-%05d.safetensors" % (s + 1, shards)
            save_file(part, os.path.join(d, fn))
            wm.update({n: fn for n in part})
        with open(os.path.join(d, "model.safetensors.index.json"), "w") as f:
            _json.dump({"metadata": {}, "weight_map": wm}, f)


@pytest.mark.parametrize("tiny", ["tiny32", "tiny64"])
@pytest.mark.parametrize("layout", [dict(), dict(prefix="bert.", shards=3)])
def test_converter_bytes_match_reference_script(lib, tmp_path, tiny, layout):
    """build/bin/convert (converter.cpp) on an HF directory holding the weights
    of the committed fixtures == the bytes models/convert-to-ggml.py wrote for
    them (tests/golden/<tiny>/ggml-model-{f32,f16}.bin, make_golden.py)."""
    ref32 = os.path.join(GOLDEN, tiny, "ggml-model-f32.bin")
    hp, vocab, tens = _parse_model_file(ref32)
    d = str(tmp_path / "hf")
    _write_hf_dir(d, hp, vocab, tens, **layout)
    for ft, fn in ((0, "ggml-model-f32.bin"), (1, "ggml-model-f16.bin")):
        out = str(tmp_path / fn)
        assert lib.bertx_convert_hf(d.encode(), out.encode(), ft) == 0
        assert open(out, "rb").read() == open(os.path.join(GOLDEN, tiny, fn), "rb").read(), fn


def test_converter_cli_and_errors(lib, tmp_path):
    hp, vocab, tens = _parse_model_file(os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin"))
    d = str(tmp_path / "hf")
    _write_hf_dir(d, hp, vocab, tens)
    exe = os.path.join(ROOT, "build", "bin", "convert")
    r = subprocess.run([exe, d, "1"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert open(os.path.join(d, "ggml-model-f16.bin"), "rb").read() == \
        open(os.path.join(GOLDEN, "tiny32", "ggml-model-f16.bin"), "rb").read()
    assert subprocess.run([exe, d, "2"], capture_output=True).returncode != 0      # Invalid ftype
    assert subprocess.run([exe], capture_output=True).returncode != 0               # usage
    # missing tensor / short vocab / no checkpoint: refused, nothing claimed
    bad = str(tmp_path / "bad")
    _write_hf_dir(bad, hp, vocab, [t for t in tens if "layer.1.output.dense.bias" not in t[0]])
    assert lib.bertx_convert_hf(bad.encode(), str(tmp_path / "x.bin").encode(), 0) != 0
    _write_hf_dir(bad, hp, vocab[:-5], tens)
    assert lib.bertx_convert_hf(bad.encode(), str(tmp_path / "x.bin").encode(), 0) != 0
    os.remove(os.path.join(bad, "model.safetensors"))
    assert lib.bertx_convert_hf(bad.encode(), str(tmp_path / "x.bin").encode(), 0) != 0


_LOAD_PROBE = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
L.bert_load_from_file.restype = ctypes.c_void_p
L.bert_load_from_file.argtypes = [ctypes.c_char_p]
ctx = L.bert_load_from_file(sys.argv[2].encode())
print("CTX", "NULL" if not ctx else "OK", flush=True)
"""


def _load_in_child(tmp_path, model, env_extra):
    """bert_load_from_file in a fresh process, so an abort shows as its exit status
    instead of killing the test run; returns (returncode, stdout, BERT_LOG text)."""
    log = tmp_path / "libbert.log"
    env = dict(os.environ)
    env.pop("BERT_HOST_ONLY", None)
    env.update(env_extra)
    env["BERT_LOG"] = str(log)
    p = subprocess.run([os.sys.executable, "-c", _LOAD_PROBE, os.path.join(ROOT, "build", "libbert.so"), model],
                       capture_output=True, text=True, env=env, timeout=120)
    return p.returncode, p.stdout + p.stderr, log.read_text() if log.exists() else ""


@pytest.mark.parametrize("stage", ["load", "image"])
def test_injected_load_failure_returns_null(lib, tmp_path, stage):
    """Every failure of the load path is a NULL context plus a message, never an
    abort (reference loader: bert.cpp:423-443, 684-750 print and return nullptr).
    BERT_FAULT_INJECT makes a load stage throw: `load` at the entry, `image` inside the
    host repack (a bad_alloc, as a host out-of-memory would).  The process must exit
    normally with a NULL context, and the BERT_LOG sink must hold the cause."""
    rc, out, log = _load_in_child(tmp_path, os.path.join(GOLDEN, "tiny32", "ggml-model-f16.bin"),
                                  {"BERT_FAULT_INJECT": stage})
    assert rc == 0, (rc, out)
    assert "CTX NULL" in out, out
    want = "load failed: BERT_FAULT_INJECT=load" if stage == "load" else "out of host memory building the device image"
    assert want in log, log
    assert want in out   # ... and the same line on stderr


@pytest.mark.skipif(HAS_GPU_NODE, reason="checks the no-device failure path")
def test_bert_log_sink_records_errors(lib, tmp_path):
    """BERT_LOG=<file> receives every libbert error line (and the load path's
    stage lines) with the pid, unbuffered: here the no-device refusal."""
    rc, out, log = _load_in_child(tmp_path, os.path.join(GOLDEN, "tiny32", "ggml-model-f32.bin"), {})
    assert rc == 0 and "CTX NULL" in out, (rc, out)
    assert "no HIP (gfx950) device available" in log, log
    assert "bytes (pageable), 0 replica(s)" in log and log.startswith("[")


def test_bert_log_fd_form_checks_identity(lib, tmp_path):
    """BERT_LOG=fd:<n>:<dev>:<ino> (tests/conftest.py hands pytest's stderr over this
    way) writes to descriptor n only while it is that file: a child process in which
    n is another file writes nothing there."""
    target = tmp_path / "target.log"
    other = tmp_path / "other.log"
    code = r"""
import ctypes, os, sys
fd = os.open(sys.argv[2], os.O_WRONLY | os.O_CREAT | os.O_APPEND)
os.environ["BERT_LOG"] = sys.argv[3].replace("N", str(fd))
L = ctypes.CDLL(sys.argv[1])
L.bert_load_from_file.restype = ctypes.c_void_p
L.bert_load_from_file(b"/nonexistent/model.bin")
"""
    st = os.stat(target.parent)   # a different file's identity: must not be written
    so = os.path.join(ROOT, "build", "libbert.so")
    env = dict(os.environ)
    env.pop("BERT_LOG", None)
    subprocess.run([os.sys.executable, "-c", code, so, str(other), f"fd:N:{st.st_dev}:{st.st_ino}"],
                   env=env, check=True, capture_output=True, timeout=120)
    assert other.read_text() == ""
    # the matching identity: written
    target.write_text("")
    st = os.stat(target)
    subprocess.run([os.sys.executable, "-c", code, so, str(target), f"fd:N:{st.st_dev}:{st.st_ino}"],
                   env=env, check=True, capture_output=True, timeout=120)
    assert "bert_load_from_file" in target.read_text()
