#!/usr/bin/env python3
"""Per-phase cycle budget of one GEMM launch from the GEMM_STAMPS diagnostic
build (BERT_LIB=build/stamps/libbert.so): prologue / K loop / epilogue per
wave-tile, and per CU how the tiles follow each other.  args: N K epi cfg."""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib(os.environ.get("STAMPS_LIB", os.path.join(ROOT, "build", "stamps", "libbert.so")))
N, K, epi, cfg = (int(x) for x in sys.argv[1:5])
M = int(os.environ.get("SWEEP_M", "32768"))
us = ctypes.c_float()
rc = L.bertx_bench_gemm(int(os.environ.get("SWEEP_FMT", "2")), N, K, M, epi, cfg, 1, ctypes.byref(us))
n = 1 << 18
buf = (ctypes.c_ulonglong * n)()
L.bertx_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert L.bertx_gemm_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
nw = 4 if cfg in (2, 3, 5, 0, 7, 11, 13, 15, 16, 19) else 2
bm = {2: 256, 3: 128, 4: 64, 5: 128, 7: 64, 14: 64, 15: 64, 16: 64, 17: 64, 19: 64, 20: 64, 6: 64, 8: 64}.get(cfg, 256)
bn = 256 if cfg == 5 else 32 * nw // (2 if cfg in (7, 8, 15, 16, 19) else 1)
tiles = (M // bm) * ((N + bn - 1) // bn)
a = a[:tiles * nw]
print(f"N={N} K={K} epi={epi} cfg={cfg} M={M}: {us.value:.1f} us, {tiles} tiles", flush=True)
pro, kl, ep = a[:, 1] - a[:, 0], a[:, 2] - a[:, 1], a[:, 3] - a[:, 2]
for nm, v in (("prologue", pro), ("K loop", kl), ("epilogue", ep), ("wave-tile", a[:, 3] - a[:, 0])):
    print(f"  {nm:9s} cycles: median {np.median(v):8.0f}  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}")
ksteps = K // 64
# K-loop split (slots 6, 7; NS >= 3 forms): load wait in front of the MFMAs, wait + barrier behind them
print(f"  K loop per K-step: front wait {np.median(a[:, 6]) / ksteps:.0f}, back wait + barrier {np.median(a[:, 7]) / ksteps:.0f}, "
      f"rest (MFMA section) {np.median(kl - a[:, 6] - a[:, 7]) / ksteps:.0f} cycles")
print(f"  K loop per K-step: {np.median(kl) / ksteps:.0f} cycles (MFMA floor per wave {64 * 16 * (bm // 256 if bm >= 256 else 1) * (2 if cfg == 5 else 1) * (bm // 128 if bm == 128 else 1) if False else 0})")
# per CU: blocks (wave 0 rows) in start order
cu = defaultdict(list)
for i in range(0, len(a), nw):
    blk = a[i:i + nw]
    key = (int(blk[0, 5]) & 0xF, (int(blk[0, 4]) >> 8) & 0xFF)
    cu[key].append((blk[:, 0].min(), blk[:, 3].max(), blk[:, 1].max(), blk[:, 2].min()))
spans, busy2, gaps, conc = [], [], [], []
for key, bl in cu.items():
    bl.sort()
    s0 = min(b[0] for b in bl)
    s1 = max(b[1] for b in bl)
    spans.append(s1 - s0)
    # time with 2 / 1 / 0 blocks resident
    ev = sorted([(b[0], 1) for b in bl] + [(b[1], -1) for b in bl])
    cur, last, hist = 0, ev[0][0], defaultdict(int)
    for t, d in ev:
        hist[cur] += t - last
        cur += d
        last = t
    tot = sum(hist.values())
    conc.append([hist[k] / tot for k in (0, 1, 2)])
print(f"  CUs {len(cu)}, blocks per CU median {np.median([len(v) for v in cu.values()]):.0f}, CU span median {np.median(spans):.0f} cycles")
c = np.array(conc).mean(axis=0)
print(f"  fraction of CU span with 0/1/2 blocks resident: {c[0]:.3f} {c[1]:.3f} {c[2]:.3f}")
print(f"  implied clock: {np.median(spans) / (us.value * 1e3):.2f} GHz (CU span / event time)")
