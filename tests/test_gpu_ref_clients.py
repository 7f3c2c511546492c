"""Drop-in check on the GPU: the reference's OWN example programs (server.cpp,
main.cpp, test_batch_encode.cpp), compiled unmodified against include/bert.h and
linked to build/libbert.so by scripts/build_ref_clients.sh, plus a ctypes client
declared exactly as examples/sample_dylib.py:19-34 declares it.  Outputs are
compared with the CPU oracle.  The binaries are built in the build container
(the reference is not on the GPU box); tests skip when they are absent."""
import ctypes
import os
import re
import socket
import struct
import subprocess
import time

import numpy as np
import pytest

import oracle_lib
from conftest import ROOT

pytestmark = pytest.mark.gpu

CLIENTS = os.path.join(ROOT, "build", "ref_clients")
COS_TOL = 1e-3


def _need(name):
    p = os.path.join(CLIENTS, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (scripts/build_ref_clients.sh)")
    return p


def _env():
    env = dict(os.environ)
    env.pop("BERT_HOST_ONLY", None)
    env["BERT_DEVICES"] = "0"
    return env


def _oracle_embed(path, text):
    o = oracle_lib.Oracle(path)
    ids = o.tokenize(text)
    return ids, o.forward_batch([ids])[0]


def _cos(a, b):
    return float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b)))


def test_reference_main(quant_models):
    exe = _need("main")
    path = quant_models[("tiny64", "q4_0")]
    prompt = "i'm going to the store to buy 3 apples and a banana!"
    r = subprocess.run([exe, "-m", path, "-p", prompt], capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lists = re.findall(r"^\[(.*)\]$", r.stdout, flags=re.M)
    toks = [int(x) for x in lists[0].split(",") if x.strip()]
    emb = np.array([float(x) for x in lists[1].split(",") if x.strip()], np.float32)
    ids, ref = _oracle_embed(path, prompt)
    assert toks == ids
    assert _cos(emb, ref) >= 1 - COS_TOL        # printed with 4 decimals


def test_reference_test_batch_encode(quant_models):
    exe = _need("test_batch_encode")
    path = quant_models[("tiny64", "f16")]
    r = subprocess.run([exe, "-m", path], capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [np.array([float(x) for x in m.split(",") if x.strip()], np.float32)
            for m in re.findall(r"^\[(.*)\]$", r.stdout, flags=re.M)]
    texts = ["你好世界", "こんにちは、世界！", "hello world"]      # test_batch_encode.cpp:39-43
    o = oracle_lib.Oracle(path)
    ref, written = o.encode_batch(texts, len(texts))
    assert written.all() and len(rows) == 3
    for got, want in zip(rows, ref):
        np.testing.assert_allclose(got, want[:10], atol=3e-3)


def test_reference_server_protocol(quant_models):
    """server.cpp:107-116: int32 n_embd on connect, then one text per recv ->
    n_embd raw float32."""
    exe = _need("server")
    path = quant_models[("tiny64", "q8_0")]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    proc = subprocess.Popen([exe, "-m", path, "--port", str(port)], stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL, env=_env())
    try:
        sock = None
        for _ in range(300):
            try:
                sock = socket.create_connection(("127.0.0.1", port), timeout=30)
                break
            except OSError:
                if proc.poll() is not None:
                    pytest.fail(f"server exited with {proc.returncode}")
                time.sleep(0.1)
        assert sock is not None
        with sock:
            n_embd = struct.unpack("i", sock.recv(4))[0]
            assert n_embd == 64
            for text in ["hello world", "what is the monthly premium for a cloud store?", "x"]:
                sock.sendall(text.encode())
                buf = b""
                while len(buf) < 4 * n_embd:
                    chunk = sock.recv(4 * n_embd - len(buf))
                    assert chunk
                    buf += chunk
                got = np.frombuffer(buf, np.float32)
                _, ref = _oracle_embed(path, text)
                assert _cos(got, ref) >= 1 - COS_TOL, text
    finally:
        proc.kill()
        proc.wait(timeout=30)


def test_sample_dylib_style_ctypes_client(quant_models):
    """The four declarations of examples/sample_dylib.py:19-34, nothing else, and
    its call pattern (n_threads 6, batch 16, numpy rows as destinations)."""
    path = quant_models[("tiny32", "q4_1")]
    lib = ctypes.cdll.LoadLibrary(os.path.join(ROOT, "build", "libbert.so"))
    lib.bert_load_from_file.restype = ctypes.c_void_p
    lib.bert_load_from_file.argtypes = [ctypes.c_char_p]
    lib.bert_n_embd.restype = ctypes.c_int32
    lib.bert_n_embd.argtypes = [ctypes.c_void_p]
    lib.bert_free.argtypes = [ctypes.c_void_p]
    lib.bert_encode_batch.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.POINTER(ctypes.c_float))]
    os.environ.pop("BERT_HOST_ONLY", None)
    ctx = lib.bert_load_from_file(path.encode("utf-8"))
    assert ctx
    n_embd = lib.bert_n_embd(ctx)
    sentences = ["hello world", "the store", "how do i get a replacement card?", "", "apple banana " * 20]
    n = len(sentences)
    emb = np.zeros((n, n_embd), dtype=np.float32)
    ptrs = (ctypes.POINTER(ctypes.c_float) * n)(*[e.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) for e in emb])
    texts = (ctypes.c_char_p * n)(*[s.encode("utf-8") for s in sentences])
    lib.bert_encode_batch(ctx, 6, 16, n, texts, ptrs)
    lib.bert_free(ctx)
    for s, e in zip(sentences, emb):
        _, ref = _oracle_embed(path, s)
        assert _cos(e, ref) >= 1 - COS_TOL, s
