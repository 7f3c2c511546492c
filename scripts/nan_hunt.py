#!/usr/bin/env python3
"""Diagnostics: run the full-size bge-base q4_0 forward several times with
BERT_CHECK_FINITE=1 (libbert reports the first kernel producing non-finite
values) and report which runs went non-finite."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
os.environ["BERT_CHECK_FINITE"] = os.environ.get("BERT_CHECK_FINITE", "1")
os.environ["BERT_DEVICES"] = "0"
import bertpy  # noqa: E402

arch, ftype = sys.argv[1] if len(sys.argv) > 1 else "bge-base-en-v1.5", sys.argv[2] if len(sys.argv) > 2 else "q4_0"
path = f"/tmp/nan_{arch}_{ftype}.bin"
if not os.path.exists(path):
    bertpy.synthetic_model(path, arch, ftype, seed=1234)
m = bertpy.BertModel(path)
ids = bertpy.synthetic_ids(64, 512, bertpy.ARCHS[arch]["n_vocab"], seed=7)
ref = None
for it in range(int(os.environ.get("RUNS", "6"))):
    e = m.forward_batch(ids if it % 2 == 0 else ids[:33])
    fin = np.isfinite(e).all(axis=1)
    msg = f"run {it}: finite rows {fin.sum()}/{len(fin)}"
    if it % 2 == 0:
        if ref is None and fin.all():
            ref = e
        elif ref is not None:
            msg += f" bitwise-equal-to-first {np.array_equal(e, ref)}"
    print(msg, flush=True)
