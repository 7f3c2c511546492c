#!/usr/bin/env python3
"""Calibration only (not the product): torch.matmul (hipBLASLt) f16 time at the
bge-base production GEMM shapes on random data, for comparison with the
hand-written kernels (scripts/gemm_sweep.py)."""
import torch

M = 32768
for name, N, K in [("qkv", 2304, 768), ("attn_out", 768, 768), ("ffn_up", 3072, 768), ("ffn_down", 768, 3072)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    w = torch.randn(N, K, device="cuda", dtype=torch.float16) * 0.02
    for _ in range(5):
        y = a @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"hipblaslt {name:9s} N={N} K={K}: {us:8.1f} us {2*M*N*K/us/1e6:7.1f} TF/s", flush=True)
