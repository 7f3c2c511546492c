#!/usr/bin/env python3
"""Forwards for a kernel trace (rocprofv3 --kernel-trace --stats): by default
bge-base q4_0, B 1, L 32 through bertx_forward_device, graph-replayed, the bench's
synthetic model; args: L reps [B arch ftype] (C2: 128 200 32 all-MiniLM-L6-v2 f16).
Prints the replay latency."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import bertpy  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
arch = sys.argv[4] if len(sys.argv) > 4 else "bge-base-en-v1.5"
ftype = sys.argv[5] if len(sys.argv) > 5 else "q4_0"
lib = bertpy.load_lib()
path = bench.ensure_model(bertpy, os.environ.get("EMB_MODEL_DIR", "/tmp/emb_models"), arch, ftype, 1234)
hp = bertpy.ARCHS[arch]
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
f = bench.DeviceForward(lib, bertpy, torch, path, bertpy.synthetic_ids(B, L, hp["n_vocab"], seed=7), dev, stream)
for _ in range(5):
    f.step()
f.sync()
t0 = time.perf_counter()
for _ in range(reps):
    f.step()
f.sync()
print(f"B{B} L{L} {arch} {ftype}: {(time.perf_counter() - t0) / reps * 1e6:.1f} us per forward (graph replay)", flush=True)
