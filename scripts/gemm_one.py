#!/usr/bin/env python3
"""One GEMM form, one tile config, N launches (for rocprofv3 PMC passes):
args: name tile_n [iters].  Random operands (bertx_bench_gemm)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

cases = {"qkv": (2, 2304, 768, 0), "attn_out": (2, 768, 768, 2), "ffn_up": (2, 3072, 768, 1),
         "ffn_down": (2, 768, 3072, 2)}
fmt, N, K, epi = cases[sys.argv[1]]
tile = int(sys.argv[2], 0)
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
us = ctypes.c_float()
L = bertpy.load_lib()
rc = L.bertx_bench_gemm(fmt, N, K, int(os.environ.get("SWEEP_M", "32768")), epi, tile, -1, iters, ctypes.byref(us))
print(sys.argv[1], hex(tile), us.value, "us", rc)
