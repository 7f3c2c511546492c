#!/usr/bin/env python3
"""Epilogue cost on a projection shape (bge-base q4_0, M 32768; default FFN-up):
bias only / era GELU, each with the input LN fold (production) and plain."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (3072, 768)
for rep in range(3):
    for epi in (0, 1):
        for name, flag in (("ln-fold", 0), ("plain", 0x100)):
            us = ctypes.c_float()
            rc = L.bertx_bench_gemm(2, N, K, 32768, epi, flag, 20, ctypes.byref(us))
            print(f"N={N} K={K} epi={epi} {name:8s}: {us.value:.1f} us rc={rc}", flush=True)
