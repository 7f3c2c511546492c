"""The tokenizer at BERT's vocabulary size (30,522 WordPiece entries, bertpy.bert_like_vocab):
libbert's trie tokenizer (csrc/tokenizer.cpp) against the reference's own tokenizer
source (bert.cpp:195-417 compiled by oracle/build_ref.sh into oracle/_ref/libreftok.so)
and against the C oracle's restatement, id for id, on texts with glued word pieces,
accents, capitals, unknown letter runs, CJK, 4-byte characters and irregular
whitespace; and bertx_tokenize_batch (the stage bert_encode_batch runs, on the
library's persistent thread pool) equal to one bert_tokenize call per text at every
thread count.  CPU only (BERT_HOST_ONLY context)."""
import ctypes
import os

import numpy as np
import pytest

import bertpy
import oracle_lib
from conftest import ROOT

REFTOK = os.path.join(ROOT, "oracle", "_ref", "libreftok.so")


@pytest.fixture(scope="module")
def bert_vocab_model(tmp_path_factory):
    """A model file whose vocab is the synthetic 30,522-entry one (tiny dims: only the
    tokenizer is exercised)."""
    vocab = bertpy.bert_like_vocab(30522, seed=0)
    hp = dict(n_vocab=len(vocab), n_max_tokens=512, n_embd=64, n_intermediate=128, n_head=1, n_layer=1)
    path = str(tmp_path_factory.mktemp("bv") / "bertvocab-f32.bin")
    bertpy.write_model(path, hp, vocab, bertpy.synthetic_tensors(hp, seed=1), 0)
    return path, vocab


@pytest.fixture(scope="module")
def host_ctx(bert_vocab_model, lib):
    os.environ["BERT_HOST_ONLY"] = "1"
    try:
        m = bertpy.BertModel(bert_vocab_model[0], lib=lib)
    finally:
        os.environ.pop("BERT_HOST_ONLY", None)
    return m


def texts():
    vocab = bertpy.bert_like_vocab(30522, seed=0)
    t = bertpy.bert_like_texts(vocab, 240, 60, seed=3)
    t += bertpy.bert_like_texts(vocab, 8, 700, seed=4)          # past n_max_tokens (the overflow quirk)
    t += [b"", b" ", b"\xe4\xb8\xad", "Ünïcödé ÀÉÎÕÜ ç".encode(), b"a" * 700, b"x!x" * 50]
    return t


def test_matches_reference_tokenizer_source(bert_vocab_model, host_ctx):
    if not os.path.exists(REFTOK):
        pytest.skip("oracle/_ref/libreftok.so not built (needs /root/reference; built by __graft_entry__.build)")
    _, vocab = bert_vocab_model
    R = ctypes.CDLL(REFTOK)
    R.reftok_new.restype = ctypes.c_void_p
    R.reftok_add.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int]
    R.reftok_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    R.reftok_free.argtypes = [ctypes.c_void_p]
    rc = R.reftok_new()
    for i, v in enumerate(vocab):
        b = v.encode()
        R.reftok_add(rc, b, len(b), i)
    buf = (ctypes.c_int32 * 4096)()
    try:
        for t in texts():
            n = ctypes.c_int32()
            R.reftok_tokenize(rc, t, buf, ctypes.byref(n), 512)
            ref = list(buf[:min(n.value, 512)])
            got, n_got = host_ctx.tokenize(t, 512)
            assert n_got == n.value and got == ref, t[:80]
    finally:
        R.reftok_free(rc)


def test_matches_oracle_and_batch_stage(bert_vocab_model, host_ctx):
    path, _ = bert_vocab_model
    o = oracle_lib.Oracle(path)
    tx = texts()
    single = [host_ctx.tokenize(t, 512) for t in tx]
    for t, (ids, n) in zip(tx, single):
        full = o.tokenize(t, 512)              # the oracle returns every counted id
        assert len(full) == n and full[:512] == ids, t[:80]
    lib = host_ctx.lib
    arr = (ctypes.c_char_p * len(tx))(*tx)
    for thr in (1, 3, 8, 16):
        ids = np.zeros((len(tx), 512), np.int32)
        lens = np.zeros(len(tx), np.int32)
        assert lib.bertx_tokenize_batch(host_ctx.ctx, thr, len(tx), arr, 512, ids.ctypes.data, lens.ctypes.data) == 0
        for i, (ref, n) in enumerate(single):
            assert lens[i] == n and list(ids[i, :min(n, 512)]) == ref, (thr, i)


def test_batch_stage_in_a_forked_child(host_ctx):
    """The tokenizer pool (csrc/task_pool.cpp) after fork: the child has none of the
    parent's pool threads; pthread_atfork gives it a fresh pool, so a multi-threaded
    batch in the child finishes with the parent's ids instead of waiting forever on
    workers that do not exist."""
    lib = host_ctx.lib
    tx = texts()[:64]
    arr = (ctypes.c_char_p * len(tx))(*tx)
    want = np.zeros((len(tx), 512), np.int32)
    wl = np.zeros(len(tx), np.int32)
    assert lib.bertx_tokenize_batch(host_ctx.ctx, 8, len(tx), arr, 512, want.ctypes.data, wl.ctypes.data) == 0
    pid = os.fork()
    if pid == 0:                                   # child: exit code 0 only on equal ids
        rc = 1
        try:
            ids = np.zeros_like(want)
            lens = np.zeros_like(wl)
            ok = lib.bertx_tokenize_batch(host_ctx.ctx, 8, len(tx), arr, 512, ids.ctypes.data, lens.ctypes.data) == 0
            rc = 0 if ok and np.array_equal(ids, want) and np.array_equal(lens, wl) else 1
        finally:
            os._exit(rc)
    deadline = 60.0
    import time
    t0 = time.time()
    while True:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        if time.time() - t0 > deadline:
            os.kill(pid, 9)
            os.waitpid(pid, 0)
            pytest.fail("the forked child's tokenizer batch hung")
        time.sleep(0.05)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0
    # and the parent's pool still works
    ids = np.zeros_like(want)
    assert lib.bertx_tokenize_batch(host_ctx.ctx, 8, len(tx), arr, 512, ids.ctypes.data, wl.ctypes.data) == 0
    assert np.array_equal(ids, want)
