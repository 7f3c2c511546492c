"""The micro-batching server (build/bin/server, tools/server_main.cpp):
the reference server's wire protocol (examples/server.cpp:26-116: int32 n_embd on
connect, one text per recv, n_embd raw float32 back) with concurrent clients whose
texts share GPU batches.  Every reply equals the library's own embedding of that
text alone bit for bit (per-sentence results do not depend on the batch), matches
the oracle, and a text past n_max_tokens gets zeros as in the reference."""
import os
import socket
import struct
import subprocess
import threading
import time

import numpy as np
import pytest

import bertpy
import oracle_lib
from conftest import ROOT

pytestmark = pytest.mark.gpu

EXE = os.path.join(ROOT, "build", "bin", "server")
COS_TOL = 1e-3


def _recv_exact(sock, n):
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        assert chunk, "server closed the connection"
        buf += chunk
    return buf


@pytest.mark.parametrize("devices", ["0", "0,0,0,0"])
def test_microbatch_server_concurrent_clients(quant_models, devices, monkeypatch):
    """One replica (one batcher), and four replicas on the one GPU (BERT_DEVICES=0,0,0,0:
    four batchers, each micro-batch routed whole to the least-loaded replica)."""
    if not os.path.exists(EXE):
        pytest.skip(f"{EXE} not built")
    path = quant_models[("tiny64", "q4_0")]
    env = dict(os.environ)
    env.pop("BERT_HOST_ONLY", None)
    env["BERT_DEVICES"] = devices
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    rng = np.random.default_rng(3)
    words = ["hello", "world", "store", "apple", "banana", "card", "premium", "cloud", "the", "a", "x!x"]
    n_cli, per = 8, 6
    texts = [[" ".join(rng.choice(words, int(rng.integers(1, 40)))) for _ in range(per)] for _ in range(n_cli)]
    texts[0][0] = "apple " * 600                  # past n_max_tokens: refused -> zeros
    results = [[None] * per for _ in range(n_cli)]
    errors = []

    def client(k):
        try:
            with socket.create_connection(("127.0.0.1", port), timeout=60) as sock:
                n = struct.unpack("i", _recv_exact(sock, 4))[0]
                for j, t in enumerate(texts[k]):
                    sock.sendall(t.encode())
                    results[k][j] = np.frombuffer(_recv_exact(sock, 4 * n), np.float32)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    proc = subprocess.Popen([EXE, "-m", path, "--port", str(port), "--max-batch", "16", "--wait-us", "3000"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
    try:
        for _ in range(600):
            try:
                socket.create_connection(("127.0.0.1", port), timeout=5).close()
                break
            except OSError:
                if proc.poll() is not None:
                    pytest.fail(f"server exited with {proc.returncode}")
                time.sleep(0.1)
        threads = [threading.Thread(target=client, args=(k,)) for k in range(n_cli)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(120)
        assert not errors, errors
    finally:
        proc.kill()
        proc.wait(timeout=30)

    monkeypatch.setenv("BERT_DEVICES", "0")
    m = bertpy.BertModel(path)
    o = oracle_lib.Oracle(path)
    for k in range(n_cli):
        for j, t in enumerate(texts[k]):
            got = results[k][j]
            assert got is not None and got.shape == (m.n_embd,)
            if (k, j) == (0, 0):
                assert np.all(got == 0.0)
                continue
            alone = m.encode(t)
            assert np.array_equal(got, alone), t
            ref = o.forward_batch([o.tokenize(t)])[0]
            assert float(np.dot(got, ref)) >= 1 - COS_TOL, t
