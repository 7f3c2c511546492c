#!/usr/bin/env python3
"""Diagnostics: per-wave s_memtime phase cycles of the q4_0 gemmqw kernel at the
bge-base production shapes, optionally with ablations (libbert prints one line
per case to stderr).  DIAGS=0,1,2,... (see gemm_q.hip DIAG bits)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
cases = [("qkv", 2304, 768, 0, 256), ("attn_out", 768, 768, 2, 128), ("ffn_up", 3072, 768, 1, 256),
         ("ffn_down", 768, 3072, 2, 128)]
only = os.environ.get("CASES")
diags = [int(x) for x in os.environ.get("DIAGS", "0").split(",")]
for name, N, K, epi, tile in cases:
    if only and name not in only.split(","):
        continue
    for dg in diags:
        us = ctypes.c_float()
        rc = L.bertx_bench_gemm(2, N, K, M, epi, tile, -3 - dg, 10, ctypes.byref(us))
        print(f"{name:10s} diag={dg:2d} {us.value:8.1f} us {2*M*N*K/us.value/1e6:7.1f} TF/s rc={rc}", flush=True)
