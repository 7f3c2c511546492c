#!/usr/bin/env python3
"""Wave-quantization probe: GEMM micro-bench time against M (tile count) for the
N = 768 residual forms (O-proj K 768, FFN-down K 3072) and QKV, tile configs
2 (256 x 128) and 3 (128 x 128)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
for (name, N, K, epi) in [("attn_out", 768, 768, 2), ("ffn_down", 768, 3072, 2), ("qkv", 2304, 768, 0)]:
    for cfg in (2, 3):
        for M in (16384, 21504, 24576, 32768, 43008, 49152):
            us = ctypes.c_float()
            rc = L.bertx_bench_gemm(2, N, K, M, epi, cfg, 20, ctypes.byref(us))
            bm = 256 if cfg == 2 else 128
            tiles = (M // bm) * ((N + 127) // 128)
            print(f"{name:9s} cfg={cfg} M={M:6d} tiles={tiles:5d} {us.value:8.1f} us  {us.value / M * 32768:8.1f} us/32k-rows "
                  f"{2.0 * M * N * K / us.value / 1e6:7.1f} TF/s rc={rc}", flush=True)
