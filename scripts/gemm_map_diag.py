#!/usr/bin/env python3
"""Index-map diagnostic for a GEMM config: W = identity (N = K), so out[m][n]
must equal X[m][n].  Two runs with X[m][k] = k and X[m][k] = m report which
(k, m) each output element actually came from.  usage: gemm_map_diag.py TILE_N [K] [M]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

L = bertpy.load_lib()
tile = int(sys.argv[1], 0)
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
M = int(sys.argv[3]) if len(sys.argv) > 3 else 256
N = K
W = np.eye(N, K, dtype=np.float16)
bias = np.zeros(N, np.float32)
for name, X in (("k", np.tile(np.arange(K, dtype=np.float16), (M, 1))),
                ("m", np.tile(np.arange(M, dtype=np.float16)[:, None], (1, K)))):
    out = np.zeros((M, N), np.float16)
    rc = L.bertx_test_gemm(1, N, K, W.tobytes(), bias.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), M,
                           np.ascontiguousarray(X).ctypes.data, 0, None, out.ctypes.data, tile)
    exp = X.astype(np.float32)
    got = out.astype(np.float32)
    bad = np.argwhere(got != exp)
    print(f"tile {tile:#x} X={name}: rc={rc} mismatches {len(bad)} of {M*N}")
    for m, n in bad[:24]:
        print(f"   out[{m}][{n}] = {got[m, n]:.0f}  expected {exp[m, n]:.0f}")
