#!/usr/bin/env python3
"""Per-phase s_memtime stamps of the gemm16 kernels (bertx_bench_gemm ablate -3,
tile_n 0x1000 | cfg) at the C3 shapes, q4_0: prologue / per-K-step / epilogue
cycles per wave, realtime span and CU busy fraction (printed by the library to stderr)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
cases = [("qkv", 2304, 768, 0), ("attn_out", 768, 768, 2), ("ffn_up", 3072, 768, 1), ("ffn_down", 768, 3072, 2)]
for cfg in [int(c) for c in os.environ.get("CFGS", "1,2,3").split(",")]:
    for name, N, K, epi in cases:
        us = ctypes.c_float()
        sys.stderr.flush()
        print(f"== cfg {cfg} {name}", flush=True)
        rc = L.bertx_bench_gemm(2, N, K, M, epi, 0x1000 | cfg, -3, 10, ctypes.byref(us))
        sys.stderr.flush()
