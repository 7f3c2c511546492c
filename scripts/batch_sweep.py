#!/usr/bin/env python3
"""Forward throughput over batch sizes (bertx_forward_device, graph-replayed like
bench.py's headline): sentences/s of MiniLM f16 at L 128 and bge-base q4_0 at L 512
and L 128, for the batch sizes between the small-batch and C2 / C3 regimes, where the
GEMM tile heuristic changes form.  BERT_LIB picks the build (A/B runs); one JSON
line per (model, B, L)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import bertpy  # noqa: E402

# SWEEP_CASES: "arch:ftype:L:B,B,...;..." (default: the round-6 mid-batch sweep)
SPEC = os.environ.get("SWEEP_CASES", "all-MiniLM-L6-v2:f16:128:8,12,16,20,24,28,32;"
                      "bge-base-en-v1.5:q4_0:512:1,2,3,4,6,8;bge-base-en-v1.5:q4_0:128:8,16,24,32")
CASES = [(a, f, int(L), [int(x) for x in bs.split(",")]) for a, f, L, bs in (c.split(":") for c in SPEC.split(";") if c)]
model_dir = os.environ.get("SWEEP_MODEL_DIR", "/tmp/bench_models")
steps = int(os.environ.get("SWEEP_STEPS", "50"))
lib = bertpy.load_lib()
dev = torch.device("cuda:0")
stream = torch.cuda.Stream(dev)
tag = os.environ.get("BERT_LIB", "build/libbert.so")
for arch, ftype, L, bs in CASES:
    path = bench.ensure_model(bertpy, model_dir, arch, ftype, 0)
    hp = bertpy.ARCHS[arch]
    for B in bs:
        f = bench.DeviceForward(lib, bertpy, torch, path, bertpy.synthetic_ids(B, L, hp["n_vocab"], seed=7), dev,
                                stream)
        for _ in range(3):
            f.step()
        f.sync()
        f.check()
        el = bench.timed_steps(f.step, steps, f.sync)
        print(json.dumps({"lib": tag, "model": f"{arch} {ftype}", "B": B, "L": L, "tokens": B * L,
                          "sentences_per_s": round(B * steps / el, 1), "us_per_batch": round(el / steps * 1e6, 1)}),
              flush=True)
        del f
