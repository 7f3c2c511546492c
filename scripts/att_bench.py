#!/usr/bin/env python3
"""Attention micro-benchmark: the production kernels (0: attention_pp for 64 < L <=
512, dh 64), attention_lds3 (8) and its 7-workgroup form (7); VARIANTS picks them."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
variants = [int(v) for v in os.environ.get("VARIANTS", "0,8").split(",")]
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for n_seqs, ln, nh, dh in [(64, 512, 12, 64), (32, 128, 12, 32)]:
        for v in variants:
            us = ctypes.c_float()
            rc = L.bertx_bench_attention(n_seqs, ln, nh, dh, v, 20, ctypes.byref(us))
            fl = 4.0 * n_seqs * ln * ln * nh * dh
            print(f"r{rnd} B={n_seqs} L={ln} H={nh} dh={dh} var={v}: {us.value:8.1f} us {fl/us.value/1e6:7.1f} TF/s rc={rc}",
                  flush=True)
