#!/usr/bin/env python3
"""Per-phase cycle budget of attention_lds3 from the ATT_STAMPS diagnostic build
(build/stamps/libbert.so): per wave and item, blocks 0 / 1-3 / B1 wait / 4-7 /
S wait / stores, at the C3 shape (B 64, L 512, 12 heads, dh 64)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib(os.environ.get("STAMPS_LIB") or os.path.join(ROOT, "build", "stamps", "libbert.so"))
us = ctypes.c_float()
assert L.bertx_bench_attention(64, 512, 12, 64, int(os.environ.get("ATT_VARIANT", "0")), 20, ctypes.byref(us)) == 0
n = 1 << 17
buf = (ctypes.c_ulonglong * n)()
L.bertx_att_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.bertx_att_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16, 4, 8).astype(np.int64)
print(f"attention C3 shape: {us.value:.1f} us per launch (20 launches; stamps of the last)")
names = ["block 0", "blocks 1-3", "B1 wait", "blocks 4-7", "S wait (+Q load)", "stores"]
for it in range(3):
    x = a[:, :, it, :]
    print(f" item {it}:")
    for k, nm in enumerate(names):
        v = (x[:, :, k + 1] - x[:, :, k]).ravel()
        print(f"   {nm:17s} median {np.median(v):7.0f}  p10 {np.percentile(v, 10):7.0f}  p90 {np.percentile(v, 90):7.0f} cycles")
    tot = (x[:, :, 6] - x[:, :, 0]).ravel()
    print(f"   item total        median {np.median(tot):7.0f}")
span = (a[:, :, 2, 6].max(axis=1) - a[:, :, 0, 0].min(axis=1))
print(f" workgroup span (3 items) median {np.median(span):.0f} cycles; implied clock {np.median(span) / (us.value * 1e3):.2f} GHz")
# in-kernel wait of the first item's prologue: from the earliest item-0 start on a CU
# per wave index: arrival at B1 and at S relative to the workgroup's item start
print(" per wave (item 1): B1 arrival / S arrival after the item's first start, median over workgroups")
x = a[:, :, 1, :]
t0 = x[:, :, 0].min(axis=1, keepdims=True)
b1 = np.median(x[:, :, 2] - t0, axis=0)
sa = np.median(x[:, :, 4] - t0, axis=0)
hw = x[:, :, 7]
simd = (hw >> 4) & 3
for w in range(16):
    print(f"   wave {w:2d} simd {np.bincount(simd[:, w], minlength=4).argmax()}: B1 {b1[w]:7.0f}  S {sa[w]:7.0f}")
