#!/usr/bin/env python3
"""GEMM micro-benchmark sweep (device-timed, random operands): production
configurations of the bge-base forward, production vs gemmqw.  Prints one line per
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
         ("ffn_down", 2, 768, 3072, 2), ("ffn_up_q8", 8, 3072, 768, 1), ("ffn_up_q41", 3, 3072, 768, 1),
         ("ffn_up_f16", 1, 3072, 768, 1), ("qkv_f16", 1, 2304, 768, 0), ("ffn_down_f16", 1, 768, 3072, 2)]
variants = [("prod", -1), ("qw", -2)]
for rnd in range(int(os.environ.get("SWEEP_ROUNDS", "2"))):
    for name, fmt, N, K, epi in cases:
        for vname, abl in variants:
            us = ctypes.c_float()
            rc = L.bertx_bench_gemm(fmt, N, K, M, epi, 0, abl, 20, ctypes.byref(us))
            print(f"r{rnd} {vname} {name:12s} fmt={fmt} N={N} K={K} epi={epi}: {us.value:8.1f} us  "
                  f"{2*M*N*K/us.value/1e6:7.1f} TF/s rc={rc}", flush=True)
