#!/usr/bin/env python3
"""GEMM micro-benchmark (bertx_bench_gemm: random operands, the forward's own
LN-fold / residual-statistics forms): args: form|all [cfg] [iters], forms at C3
(bge-base q4_0, M = SWEEP_M tokens, default 32768).  Also the target of the
rocprofv3 PMC passes (scripts/gpu_gemm_pmc.sh)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

cases = {"qkv": (2, 2304, 768, 0), "attn_out": (2, 768, 768, 2), "ffn_up": (2, 3072, 768, 1),
         "ffn_down": (2, 768, 3072, 2)}
names = list(cases) if sys.argv[1] == "all" else [sys.argv[1]]
cfg = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
M = int(os.environ.get("SWEEP_M", "32768"))
fmt_env = os.environ.get("SWEEP_FMT")
L = bertpy.load_lib()
for name in names:
    fmt, N, K, epi = cases[name]
    if fmt_env:
        fmt = int(fmt_env)
    us = ctypes.c_float()
    rc = L.bertx_bench_gemm(fmt, N, K, M, epi, cfg, iters, ctypes.byref(us))
    tf = 2.0 * M * N * K / (us.value * 1e-6) / 1e12 if us.value > 0 else 0.0
    print(f"{name:9s} fmt={fmt} N={N} K={K} M={M} cfg={cfg}: {us.value:8.1f} us {tf:7.1f} TF/s rc={rc}", flush=True)
