#!/usr/bin/env python3
"""Per-share forward latency against tokens on one replica (set
the routing threshold kMinShareTokens, bert_abi.cpp, from a measurement).

A call of T tokens split over k idle replicas finishes in about lat(T / k) and
occupies k replicas for that long.  Splitting buys latency only where lat() is still
proportional to the tokens: below the knee a forward is launch- and latency-bound,
lat(T / k) ~ lat(T), and the split only costs the other replicas a whole forward.
This times bert_forward_batch (host ids in, host rows out: the path a routed share
runs) of n sentences x L tokens on one replica, for T = n L from 128 to 65,536, and
prints one JSON line per T plus the knee: the smallest T whose per-token cost is
within --eff of the large-T asymptote (the median of the three largest T).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
import bertpy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="bge-base-en-v1.5")
    ap.add_argument("--ftype", default="q4_0")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--eff", type=float, default=1.25)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "share_curve.jsonl"))
    a = ap.parse_args()
    os.environ["BERT_DEVICES"] = "0"
    hp = bertpy.ARCHS[a.arch]
    path = f"/tmp/share_curve_{a.arch}_{a.ftype}.bin"
    if not os.path.exists(path):
        bertpy.synthetic_model(path, a.arch, a.ftype, seed=1234)
    m = bertpy.BertModel(path)
    rows = []
    T = a.seq
    while T <= 65536:
        n = max(1, T // a.seq)
        ids = bertpy.synthetic_ids(n, min(a.seq, T), hp["n_vocab"], seed=7)
        for _ in range(3):
            m.forward_batch(ids)
        reps = max(5, min(200, int(2e5 // T)))
        t0 = time.perf_counter()
        for _ in range(reps):
            m.forward_batch(ids)
        lat = (time.perf_counter() - t0) / reps
        rows.append({"tokens": n * min(a.seq, T), "sentences": n, "seq": min(a.seq, T), "lat_ms": round(lat * 1e3, 4),
                     "us_per_token": round(lat * 1e6 / (n * min(a.seq, T)), 4)})
        print(json.dumps(rows[-1]), flush=True)
        T *= 2
    asym = float(np.median([r["us_per_token"] for r in rows[-3:]]))
    knee = next(r["tokens"] for r in rows if r["us_per_token"] <= a.eff * asym)
    summ = {"arch": a.arch, "ftype": a.ftype, "seq": a.seq, "asymptote_us_per_token": asym, "eff": a.eff,
            "knee_tokens": knee, "curve": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "a") as f:
        f.write(json.dumps(summ) + "\n")
    print(json.dumps({"knee_tokens": knee, "asymptote_us_per_token": asym}), flush=True)


if __name__ == "__main__":
    main()
