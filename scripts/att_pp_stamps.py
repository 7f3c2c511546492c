#!/usr/bin/env python3
"""Per-phase cycle budget of attention_pp from the ATT_STAMPS diagnostic build
(build/stamps/libbert.so) at the C3 shape (B 64, L 512, 12 heads, dh 64): per
unit and wave the prologue (Q + blocks 0-2 landed, first barrier), block 0, the
summed wait + barrier + issue of blocks 1-7, their summed compute, the stores;
then per CU how the two co-resident workgroups overlap."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib(os.environ.get("STAMPS_LIB") or os.path.join(ROOT, "build", "stamps", "libbert.so"))
us = ctypes.c_float()
assert L.bertx_bench_attention(64, 512, 12, 64, 0, 20, ctypes.byref(us)) == 0
n = 1 << 17
buf = (ctypes.c_ulonglong * n)()
L.bertx_att_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.bertx_att_stamps(buf, n) == 0
units = 64 * 12 * 2
a = np.frombuffer(buf, dtype=np.uint64)[: units * 64].reshape(units, 8, 8).astype(np.int64)
print(f"attention_pp, C3 shape: {us.value:.1f} us per launch (20 launches; stamps of the last)")
rows = [("prologue (Q, blocks 0-2, barrier)", a[:, :, 1] - a[:, :, 0]),
        ("block 0", a[:, :, 2] - a[:, :, 1]),
        ("blocks 1-7: wait + barrier + issue", a[:, :, 3]),
        ("blocks 1-7: compute", a[:, :, 4]),
        ("after the loop (drain)", a[:, :, 5] - a[:, :, 2] - a[:, :, 3] - a[:, :, 4]),
        ("stores", a[:, :, 6] - a[:, :, 5]),
        ("unit total", a[:, :, 6] - a[:, :, 0])]
for name, v in rows:
    v = v.ravel()
    print(f"  {name:36s} median {np.median(v):7.0f}  p10 {np.percentile(v, 10):7.0f}  p90 {np.percentile(v, 90):7.0f} cycles")
# per CU: workgroup lifetimes (wave 0's start .. latest store end) and overlap
hw = a[:, 0, 7]
cu = (hw >> 8) & 0xF            # CU_ID
sh = (hw >> 12) & 0x1           # SH_ID
se = (hw >> 13) & 0x7           # SE_ID
xcc = None
t0 = a[:, :, 0].min(axis=1)
t1 = a[:, :, 6].max(axis=1)
key = se * 32 + sh * 16 + cu
span = t1.max() - t0.min()
busy = {}
for k, s0, s1 in zip(key, t0, t1):
    busy.setdefault(int(k), []).append((int(s0), int(s1)))
life = np.median(t1 - t0)
print(f"  unit lifetime median {life:.0f} cycles; kernel span {span} cycles -> implied clock "
      f"{span / (us.value * 1e3):.2f} GHz (clocks differ per XCD: indicative)")
