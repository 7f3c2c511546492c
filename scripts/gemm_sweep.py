#!/usr/bin/env python3
"""GEMM micro-benchmark sweep (device-timed, random operands): production
configurations of the bge-base forward and ablation builds.  Prints one line per
case: name, avg us, TFLOP/s."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
cases = [("qkv", 2, 2304, 768, 0), ("attn_out", 2, 768, 768, 2), ("ffn_up", 2, 3072, 768, 1),
         ("ffn_down", 2, 768, 3072, 2), ("ffn_up_f16", 1, 3072, 768, 1), ("ffn_up_q8", 8, 3072, 768, 1)]
for name, fmt, N, K, epi in cases:
    us = ctypes.c_float()
    rc = L.bertx_bench_gemm(fmt, N, K, M, epi, 0, -1, 20, ctypes.byref(us))
    print(f"{name:12s} fmt={fmt} N={N} K={K} epi={epi}: {us.value:8.1f} us  {2*M*N*K/us.value/1e6:7.1f} TF/s rc={rc}",
          flush=True)
for bn in (256, 128):
    for abl in [int(a) for a in os.environ.get("SWEEP_ABL", "0,1,4,8,15").split(",")]:
        us = ctypes.c_float()
        rc = L.bertx_bench_gemm(1, 3072, 768, M, 0, bn, abl, 20, ctypes.byref(us))
        print(f"ablate bn={bn} abl={abl:2d}: {us.value:8.1f} us  {2*M*3072*768/us.value/1e6:7.1f} TF/s rc={rc}",
              flush=True)
