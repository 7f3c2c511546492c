#!/usr/bin/env python3
"""Per-tile overhead probe: GEMM micro-bench time against K at fixed M, N (tile
count fixed), so time = overhead + K-loop slope * K; per epilogue form."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
M = int(os.environ.get("SWEEP_M", "32768"))
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for N, epi in [(3072, 1), (3072, 0), (3072, 2), (768, 2)]:
    for rep in range(2):
        for K in (384, 768, 1536, 3072):
            us = ctypes.c_float()
            rc = L.bertx_bench_gemm(2, N, K, M, epi, cfg, 20, ctypes.byref(us))
            print(f"N={N} epi={epi} K={K:5d} cfg={cfg}: {us.value:8.1f} us {2.0 * M * N * K / us.value / 1e6:7.1f} TF/s rc={rc}",
                  flush=True)
