#!/usr/bin/env python3
"""A/B of the GEMM kernels (VARIANTS="name:tile_n,...") in one process (device-timed, random operands):
gemm.hip production (32x32x16, layout 0) vs gemm16.hip (16x16x32, layout 1)
configs (tile_n 0x1000 | c) 1 (8 waves 256x256), 2 (4 waves 256x128), 3 (4 waves 128x128).
env: SWEEP_M (32768), SWEEP_ROUNDS (2), SWEEP_CASES (comma list of names)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
cases = [("qkv", 2, 2304, 768, 0), ("attn_out", 2, 768, 768, 2), ("ffn_up", 2, 3072, 768, 1),
         ("ffn_down", 2, 768, 3072, 2), ("ffn_up_q8", 8, 3072, 768, 1), ("ffn_up_q41", 3, 3072, 768, 1),
         ("ffn_up_f16", 1, 3072, 768, 1), ("qkv_f16", 1, 2304, 768, 0), ("attn_out_f16", 1, 768, 768, 2),
         ("ffn_down_f16", 1, 768, 3072, 2)]
want = os.environ.get("SWEEP_CASES")
if want:
    cases = [c for c in cases if c[0] in want.split(",")]
variants = [(n, int(t, 0)) for n, t in (v.split(":") for v in os.environ.get(
    "VARIANTS", "old:0,z0:0x1000,z1:0x1001,z3:0x1003").split(","))]
for rnd in range(int(os.environ.get("SWEEP_ROUNDS", "2"))):
    for name, fmt, N, K, epi in cases:
        for vname, tile in variants:
            us = ctypes.c_float()
            rc = L.bertx_bench_gemm(fmt, N, K, M, epi, tile, -1, 20, ctypes.byref(us))
            print(f"r{rnd} {vname:4s} {name:12s} fmt={fmt} N={N} K={K} epi={epi}: {us.value:8.1f} us  "
                  f"{2*M*N*K/us.value/1e6:7.1f} TF/s rc={rc}", flush=True)
