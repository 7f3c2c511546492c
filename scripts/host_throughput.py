#!/usr/bin/env python3
"""Host-side throughput of the two SURVEY §8(f) rows around the GPU forward.

  tok     (f2, CPU only) WordPiece tokenization of ~500-token texts over a
          30,522-entry BERT-size vocab: the reference's own tokenizer source
          (bert.cpp:195-417 compiled into oracle/_ref/libreftok.so by
          oracle/build_ref.sh -- std::map substring probes, one thread, as
          bert_encode_batch runs it, bert.cpp:1402-1406) against the library's own
          batch stage bertx_tokenize_batch (csrc/tokenizer.cpp trie on the persistent
          pool, csrc/task_pool.cpp) at 1 / 8 / 16 threads.  Token ids of both are
          compared on every text the reference tokenizes.
  server  (f3, GPU) requests/s of the TCP protocol (examples/server.cpp: int32 n_embd
          on connect, one text per recv, n_embd float32 back) with 1 / 8 / 64
          concurrent clients: build/bin/server (micro-batching) against the
          reference's own examples/server.cpp linked to libbert.so
          (build/ref_clients/server: one client at a time, one text per forward).

Prints one JSON object per measurement.  Server model: the bench's synthetic
bge-base-en-v1.5 q4_0 (words w<i> are single tokens, so a text of k words is
exactly k + 2 tokens).
"""
import argparse
import ctypes
import json
import os
import socket
import struct
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


def make_texts(vocab, n, n_words, seed=0):
    """Words of 1-3 word pieces (first piece a whole-word token, later pieces '##'
    continuations with the '##' dropped), so greedy longest-prefix matching splits
    them again; some punctuation and accented letters."""
    rng = np.random.default_rng(seed)
    whole = [v for v in vocab if v.isalpha() and not v.startswith("[")]
    subs = [v[2:] for v in vocab if v.startswith("##") and v[2:].isalpha()]
    extras = [",", ".", "!", "café", "naïve", "(", ")"]
    out = []
    for _ in range(n):
        words = []
        for _ in range(n_words):
            r = rng.random()
            if r < 0.06:
                words.append(extras[int(rng.integers(len(extras)))])
                continue
            w = whole[int(rng.integers(len(whole)))]
            for _ in range(int(rng.integers(0, 3))):
                w += subs[int(rng.integers(len(subs)))]
            words.append(w.upper() if rng.random() < 0.05 else w)
        out.append(" ".join(words).encode())
    return out


def cmd_tok(a):
    """Tokenizer throughput at BERT's vocabulary size: 30,522 WordPiece entries
    (bertpy.bert_like_vocab) and ~500-token texts (bertpy.bert_like_texts); the
    reference's tokenizer source on one thread (as bert_encode_batch runs it,
    bert.cpp:1402-1406) against the library's own batch stage, bertx_tokenize_batch
    -- the function bert_encode_batch calls -- on 1 / 8 / 16 threads of its
    persistent pool, one call over all texts, timed around that call."""
    vocab = bertpy.bert_like_vocab(30522, seed=0)
    n_max = 512
    hp = dict(n_vocab=len(vocab), n_max_tokens=n_max, n_embd=64, n_intermediate=128, n_head=1, n_layer=1)
    path = os.path.join("/tmp", "host_tok_bertvocab.bin")
    bertpy.write_model(path, hp, vocab, bertpy.synthetic_tensors(hp, seed=1), 0)
    os.environ["BERT_HOST_ONLY"] = "1"
    lib = bertpy.load_lib()
    m = bertpy.BertModel(path, lib=lib)
    probe = bertpy.bert_like_texts(vocab, 8, 200, seed=1)
    per_word = np.mean([m.tokenize(t, 100000)[1] for t in probe]) / 200
    texts = bertpy.bert_like_texts(vocab, a.texts, int(500 / per_word), seed=2)
    arr = (ctypes.c_char_p * len(texts))(*texts)
    ids = np.zeros((len(texts), n_max), np.int32)
    lens = np.zeros(len(texts), np.int32)
    assert lib.bertx_tokenize_batch(m.ctx, 1, len(texts), arr, n_max, ids.ctypes.data, lens.ctypes.data) == 0
    emit(kind="texts", n=len(texts), vocab=len(vocab), mean_tokens=float(np.mean(lens)), min_tokens=int(lens.min()),
         max_tokens=int(lens.max()), mean_bytes=float(np.mean([len(t) for t in texts])))
    res = {}
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libreftok.so")
    if os.path.exists(ref_path):
        R = ctypes.CDLL(ref_path)
        R.reftok_new.restype = ctypes.c_void_p
        R.reftok_add.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int]
        R.reftok_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int32]
        rc = R.reftok_new()
        for i, v in enumerate(vocab):
            b = v.encode()
            R.reftok_add(rc, b, len(b), i)
        rbuf = (ctypes.c_int32 * (4 * n_max))()
        nref = min(len(texts), a.ref_texts)
        t0 = time.perf_counter()
        for i, t in enumerate(texts[:nref]):
            rn = ctypes.c_int32()
            R.reftok_tokenize(rc, t, rbuf, ctypes.byref(rn), n_max)
            # ids equal on every text timed (the written prefix)
            assert rn.value == lens[i] and list(rbuf[:min(rn.value, n_max)]) == list(ids[i, :min(lens[i], n_max)])
        el = time.perf_counter() - t0
        res["reference"] = nref / el
        emit(kind="tokenizer", impl="reference bert.cpp:195-417 (std::map), 30,522-entry vocab", threads=1,
             texts=nref, texts_per_s=round(nref / el, 1), us_per_text=round(el / nref * 1e6, 2))
    for thr in a.threads:
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            assert lib.bertx_tokenize_batch(m.ctx, thr, len(texts), arr, n_max, ids.ctypes.data,
                                            lens.ctypes.data) == 0
            best = max(best, len(texts) / (time.perf_counter() - t0))
        res[thr] = best
        emit(kind="tokenizer", impl="libbert bertx_tokenize_batch (trie, persistent pool)", threads=thr,
             texts=len(texts), texts_per_s=round(best, 1), us_per_text_per_thread=round(thr / best * 1e6, 2),
             vs_reference_1thread=round(best / res["reference"], 2) if "reference" in res else None,
             cpus_visible=len(os.sched_getaffinity(0)))


def recv_exact(sock, n):
    b = b""
    while len(b) < n:
        c = sock.recv(n - len(b))
        if not c:
            raise RuntimeError("closed")
        b += c
    return b


def _client_proc(port, n_threads, per_client, text, q):
    """One load-generator process: n_threads clients, each sending per_client texts
    and reading the n_embd-float replies; reports (latencies, errors, cpu seconds)."""
    errors, lat = [], []

    def client():
        try:
            with socket.create_connection(("127.0.0.1", port), timeout=300) as s:
                nd = struct.unpack("i", recv_exact(s, 4))[0]
                for _ in range(per_client):
                    t0 = time.perf_counter()
                    s.sendall(text)
                    recv_exact(s, 4 * nd)
                    lat.append(time.perf_counter() - t0)
        except Exception as e:  # noqa: BLE001 -- reported
            errors.append(repr(e))

    c0 = os.times()
    ths = [threading.Thread(target=client) for _ in range(n_threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(600)
    c1 = os.times()
    q.put((lat, errors, (c1.user - c0.user) + (c1.system - c0.system)))


def run_server_load(exe_args, port, n_clients, per_client, text, env):
    """Clients spread over up to 16 load-generator processes (a single Python process
    is GIL-bound long before the server is); returns (requests/s, median latency,
    the generator's CPU use as a fraction of its processes' wall time)."""
    import multiprocessing as mp
    proc = subprocess.Popen(exe_args, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
    try:
        for _ in range(1200):
            try:
                socket.create_connection(("127.0.0.1", port), timeout=5).close()
                break
            except OSError:
                if proc.poll() is not None:
                    raise RuntimeError(f"server exited {proc.returncode}")
                time.sleep(0.1)
        n_proc = min(16, n_clients)
        per_proc = [n_clients // n_proc + (1 if i < n_clients % n_proc else 0) for i in range(n_proc)]
        ctx = mp.get_context("fork")
        q = ctx.Queue()
        ps = [ctx.Process(target=_client_proc, args=(port, k, per_client, text, q)) for k in per_proc]
        t0 = time.perf_counter()
        for p_ in ps:
            p_.start()
        res = [q.get(timeout=900) for _ in ps]
        el = time.perf_counter() - t0
        for p_ in ps:
            p_.join(60)
        errors = [e for r in res for e in r[1]]
        if errors:
            raise RuntimeError(errors[:3])
        lat = [x for r in res for x in r[0]]
        cpu = sum(r[2] for r in res) / (el * n_proc)
        return n_clients * per_client / el, float(np.median(lat)), cpu
    finally:
        proc.kill()
        proc.wait(timeout=30)


def cmd_server(a):
    model_dir = os.environ.get("EMB_MODEL_DIR", "/tmp/emb_models")
    os.makedirs(model_dir, exist_ok=True)
    path = os.path.join(model_dir, "bge-base-en-v1.5-q4_0-seed1234.bin")
    if not os.path.exists(path):
        bertpy.synthetic_model(path + ".part", "bge-base-en-v1.5", "q4_0", seed=1234)
        os.replace(path + ".part", path)
    text = " ".join(f"w{1000 + 37 * i}" for i in range(a.words)).encode()   # a.words + 2 tokens
    env = dict(os.environ, BERT_DEVICES="0")
    env.pop("BERT_HOST_ONLY", None)
    ours = os.path.join(ROOT, "build", "bin", "server")
    ref = os.path.join(ROOT, "build", "ref_clients", "server")
    for n_cli in a.clients:
        per = max(a.min_requests // n_cli, 2)
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        rps, med, cpu = run_server_load([ours, "-m", path, "--port", str(port), "--max-batch", "64", "--wait-us",
                                         str(a.wait_us)], port, n_cli, per, text, env)
        emit(kind="server", impl="build/bin/server (micro-batching)", clients=n_cli, tokens_per_text=a.words + 2,
             requests=n_cli * per, requests_per_s=round(rps, 1), median_latency_ms=round(med * 1e3, 3),
             client_cpu_frac=round(cpu, 3), client_bound=bool(cpu > 0.9))
        if os.path.exists(ref) and n_cli == 1:
            # the reference server takes one client at a time (backlog 1, serial accept
            # loop, examples/server.cpp:92-118): concurrent clients queue behind each
            # other (and behind SYN retransmits), so its N-client rate is at most this one
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            rps, med, cpu = run_server_load([ref, "-m", path, "--port", str(port)], port, n_cli, per, text, env)
            emit(kind="server", impl="reference examples/server.cpp on libbert (batch 1 per recv)", clients=n_cli,
                 tokens_per_text=a.words + 2, requests=n_cli * per, requests_per_s=round(rps, 1),
                 median_latency_ms=round(med * 1e3, 3), client_cpu_frac=round(cpu, 3))


def main():
    p = argparse.ArgumentParser()
    sub = p.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("tok")
    t.add_argument("--texts", type=int, default=2000)
    t.add_argument("--threads", type=int, nargs="+", default=[1, 8, 16])
    t.add_argument("--ref-texts", type=int, default=400, help="texts timed through the reference tokenizer")
    s = sub.add_parser("server")
    s.add_argument("--clients", type=int, nargs="+", default=[1, 8, 32, 64])
    s.add_argument("--words", type=int, default=126)
    s.add_argument("--min-requests", type=int, default=5000)
    s.add_argument("--wait-us", type=int, default=2000)
    a = p.parse_args()
    cmd_tok(a) if a.cmd == "tok" else cmd_server(a)


if __name__ == "__main__":
    main()
