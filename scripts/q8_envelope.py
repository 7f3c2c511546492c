#!/usr/bin/env python3
"""How far the reference's own q8 activation rounding moves an embedding, and which
arithmetic the HIP path tracks.

The reference multiplies q4/q8 weights by activations re-quantized per 32-block to
q8_0 / q8_1 (bert.cpp:995 through ggml).  The HIP path multiplies
the same weights by f16 activations.  At C4 dims (bge-large-en-v1.5, q4_1, 24
layers, "sharp" weights) with the Q/K spread swept over 0.02 / 0.03 / 0.05, this
records per sentence the cosines

    hip_vs_q8   HIP (libbert)            vs oracle, reference arithmetic (q8 activations)
    hip_vs_f32  HIP                      vs oracle with f32 activations (diagnostic switch)
    q8_vs_f32   oracle (q8 activations)  vs oracle (f32 activations)

one JSON line per (qk_std, statistic) into --out.  Runs on the GPU box (libbert
needs a gfx950 device); the oracle is the checker, timed nowhere.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bertpy      # noqa: E402
import oracle_lib  # noqa: E402


def cos(a, b):
    return np.sum(a * b, axis=1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="bge-large-en-v1.5")
    ap.add_argument("--ftype", default="q4_1")
    ap.add_argument("--qk", default="0.02,0.03,0.05")
    ap.add_argument("--lens", default="3,17,64,128,200,300,450,512")
    ap.add_argument("--threads", type=int, default=min(16, len(os.sched_getaffinity(0))))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "q8_envelope.jsonl"))
    ap.add_argument("--model-dir", default="/tmp/q8_envelope")
    a = ap.parse_args()
    os.makedirs(a.model_dir, exist_ok=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    os.environ.setdefault("BERT_DEVICES", "0")
    hp = bertpy.ARCHS[a.arch]
    lens = [int(x) for x in a.lens.split(",")]
    ids = bertpy.synthetic_ids(len(lens), lens, hp["n_vocab"], seed=7)
    with open(a.out, "a") as f:
        for qk in [float(x) for x in a.qk.split(",")]:
            t0 = time.perf_counter()
            path = os.path.join(a.model_dir, f"{a.arch}-{a.ftype}-sharp-qk{qk}.bin")
            if not os.path.exists(path):
                bertpy.synthetic_model(path, a.arch, a.ftype, seed=1234, profile="sharp", qk_std=qk)
            m = bertpy.BertModel(path)
            hip = m.forward_batch(ids)
            del m
            o = oracle_lib.Oracle(path)
            q8 = np.concatenate([o.forward_batch([x], n_threads=a.threads) for x in ids])
            f32 = np.concatenate([o.forward_batch([x], n_threads=a.threads, activations="f32") for x in ids])
            del o
            rows = {"hip_vs_q8": cos(hip, q8), "hip_vs_f32": cos(hip, f32), "q8_vs_f32": cos(q8, f32)}
            for k, c in rows.items():
                rec = {"arch": a.arch, "ftype": a.ftype, "qk_std": qk, "stat": k, "min_cos": float(np.min(c)),
                       "per_sentence": {str(L): round(float(v), 7) for L, v in zip(lens, c)}}
                f.write(json.dumps(rec) + "\n")
                print(json.dumps(rec), flush=True)
            print(f"qk {qk}: {time.perf_counter() - t0:.1f} s", flush=True)
            os.remove(path)


if __name__ == "__main__":
    main()
