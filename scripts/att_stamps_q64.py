#!/usr/bin/env python3
"""Per-phase cycle budget of attention_q64 (variant 8) from the ATT_STAMPS diagnostic
build (build/stamps/libbert.so), at the C3 shape (B 64, L 512, 12 heads, dh 64): per
wave and item, unit 0 (+ A(1) + C(0)), units 1-6, the B1a wait (region B landed),
units 7-8, the B1b wait (region A free), units 9-15, the S wait (+ next Q), stores."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib(os.path.join(ROOT, "build", "stamps", "libbert.so"))
us = ctypes.c_float()
assert L.bertx_bench_attention(64, 512, 12, 64, 8, 20, ctypes.byref(us)) == 0
n = 1 << 17
buf = (ctypes.c_ulonglong * n)()
L.bertx_att_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.bertx_att_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 16, 4, 8).astype(np.int64)[:, :8]
print(f"attention_q64 C3 shape: {us.value:.1f} us per launch (20 launches; stamps of the last)")
names = ["unit 0", "units 1-6", "B1a wait", "units 7-8", "B1b wait + issue", "units 9-15", "S wait (+Q)", "stores"]
# slots: 0 start, 1 after unit 0, 2 B1a arrive, 3 after B1a, 4 B1b arrive, 5 loop end, 6 after S, 7 after stores
edges = [(0, 1), (1, 2), (2, 3), (3, 4), None, (4, 5), (5, 6), (6, 7)]
for it in range(3):
    x = a[:, :, it, :]
    print(f" item {it}:")
    for nm, e in zip(names, edges):
        if e is None:
            continue
        v = (x[:, :, e[1]] - x[:, :, e[0]]).ravel()
        print(f"   {nm:17s} median {np.median(v):7.0f}  p10 {np.percentile(v, 10):7.0f}  p90 {np.percentile(v, 90):7.0f} cycles")
    tot = (x[:, :, 7] - x[:, :, 0]).ravel()
    print(f"   item total        median {np.median(tot):7.0f}")
