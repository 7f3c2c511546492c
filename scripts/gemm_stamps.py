#!/usr/bin/env python3
"""Diagnostics: per-wave s_memtime phase cycles of the q4_0 gemmqw kernel at the
bge-base production shapes (libbert prints one line per case to stderr)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
for name, N, K, epi, tile in [("qkv", 2304, 768, 0, 256), ("attn_out", 768, 768, 2, 128),
                              ("ffn_up", 3072, 768, 1, 256), ("ffn_down", 768, 3072, 2, 128),
                              ("ffn_up_noepi_gelu", 3072, 768, 0, 256)]:
    us = ctypes.c_float()
    rc = L.bertx_bench_gemm(2, N, K, M, epi, tile, -3, 10, ctypes.byref(us))
    print(f"{name:10s} {us.value:8.1f} us {2*M*N*K/us.value/1e6:7.1f} TF/s rc={rc}", flush=True)
