#!/usr/bin/env python3
"""Diagnostics: s_memtime phase cycles of the q4_0 gemmqv kernel (two workgroups
per CU) at the bge-base shapes (tile code 4 = BM 256, 5 = BM 128)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = 32768
for name, N, K, epi, tile in [("qkv", 2304, 768, 0, 4), ("attn_out", 768, 768, 2, 5), ("ffn_up", 3072, 768, 1, 4),
                              ("ffn_up_bm128", 3072, 768, 1, 5), ("ffn_down", 768, 3072, 2, 5)]:
    us = ctypes.c_float()
    rc = L.bertx_bench_gemm(2, N, K, M, epi, tile, -3, 10, ctypes.byref(us))
    print(f"{name:12s} rc={rc}", flush=True)
