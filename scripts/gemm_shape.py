#!/usr/bin/env python3
"""GEMM micro-benchmark of arbitrary shapes (bertx_bench_gemm: random operands, the
forward's LN-fold forms): args: fmt N K M epi cfg[,cfg...] [iters]."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

fmt, N, K, M, epi = (int(a) for a in sys.argv[1:6])
cfgs = [int(c) for c in sys.argv[6].split(",")]
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 50
L = bertpy.load_lib()
for cfg in cfgs:
    us = ctypes.c_float()
    rc = L.bertx_bench_gemm(fmt, N, K, M, epi, cfg, iters, ctypes.byref(us))
    print(f"fmt={fmt} N={N} K={K} M={M} epi={epi} cfg={cfg} ran={L.bertx_test_gemm_ran()}: {us.value:8.2f} us rc={rc}", flush=True)
