#!/usr/bin/env python3
"""A/B of gemmqw diagnostic builds (q4_0, one 8-wave workgroup per CU): per-wave
phase stamps (stderr) and the device time of the same build without stamps.
env: DIAGS (comma list, default 0,256), SWEEP_ROUNDS (2), SWEEP_M (32768)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
diags = [int(x) for x in os.environ.get("DIAGS", "0,256").split(",")]
cases = [("qkv", 2304, 768, 0), ("ffn_up", 3072, 768, 1), ("attn_out", 768, 768, 2), ("ffn_down", 768, 3072, 2)]
for rnd in range(int(os.environ.get("SWEEP_ROUNDS", "2"))):
    for name, N, K, epi in cases:
        for d in diags:
            us = ctypes.c_float()
            rc = L.bertx_bench_gemm(2, N, K, M, epi, 0, -3 - d, 20, ctypes.byref(us))
            print(f"r{rnd} diag={d:4d} {name:10s} {us.value:8.1f} us {2*M*N*K/us.value/1e6:7.1f} TF/s rc={rc}",
                  flush=True)
