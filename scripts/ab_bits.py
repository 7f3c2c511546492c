#!/usr/bin/env python3
"""Forward outputs of one build (BERT_LIB) saved for a bitwise A/B against another:
args: out.npy arch ftype [n_sentences length]; synthetic weights (seed 1234) and
ragged ids (seed 5), so two builds given the same args see the same inputs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402

out, arch, ftype = sys.argv[1:4]
n = int(sys.argv[4]) if len(sys.argv) > 4 else 24
path = f"/tmp/ab_bits_{arch}_{ftype}.bin"
if not os.path.exists(path):
    bertpy.synthetic_model(path + ".part", arch, ftype, seed=1234)
    os.replace(path + ".part", path)
hp = bertpy.ARCHS[arch]
rng = np.random.default_rng(5)
lens = [int(x) for x in rng.integers(1, 513, n)]
m = bertpy.BertModel(path)
ids = bertpy.synthetic_ids(n, lens, hp["n_vocab"], seed=5)
e = np.concatenate([m.forward_batch(ids), m.forward_batch(ids[:1]), m.forward_batch(ids[:4])])
np.save(out, e)
print(out, e.shape, bool(np.isfinite(e).all()))
