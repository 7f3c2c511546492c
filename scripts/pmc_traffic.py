#!/usr/bin/env python3
"""HBM-side bytes per launch, per kernel class, from two rocprofv3 PMC passes
of bench.py (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]":
  * the counters are in KiB;
  * FETCH_SIZE reports half the bytes of wide coalesced (16 B/lane) reads on
    gfx950 -> doubled (all hot-path loads here are 16 B/lane);
  * WRITE_SIZE is exact for 16-B-per-lane stores.
Counts are fabric-side requests: Infinity-Cache hits are included, so the
figure is an upper bound on DRAM bytes.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR [out.json]
Kernel -> bench class: by kernel name; the two EPI_BIAS_RES_F32 GEMMs of a
layer (attention output, FFN down) share a name and alternate in dispatch order.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = [r for r in csv.DictReader(open(f[0])) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def classify(rows):
    """-> list of (class, value KiB) in dispatch order."""
    out, res_i = [], 0
    for r in rows:
        k = r["Kernel_Name"]
        m = re.search(r"gemm[qvwz]*_kernelILi(\d+)ELi(\d+)E", k)
        if m:
            epi = int(m.group(2))
            if epi == 0:
                c = "gemm_qkv"
            elif epi == 1:
                c = "gemm_ffn_up"
            else:
                c = "gemm_attn_out" if res_i % 2 == 0 else "gemm_ffn_down"
                res_i += 1
        elif "attention" in k:
            c = "attention"
        elif "ln_stats" in k:
            c = "ln_stats"
        elif "embed_ln_kernel" in k:
            c = "embed_ln"
        elif "pool_partial" in k:
            c = "pool_partial"
        elif "pool_final" in k:
            c = "pool_final"
        else:
            continue
        out.append((c, float(r["Counter_Value"])))
    return out


def main():
    fetch = classify(load(sys.argv[1], "FETCH_SIZE"))
    write = classify(load(sys.argv[2], "WRITE_SIZE"))
    agg = collections.defaultdict(lambda: [0.0, 0, 0.0, 0])
    for c, v in fetch:
        agg[c][0] += v * 1024 * 2
        agg[c][1] += 1
    for c, v in write:
        agg[c][2] += v * 1024
        agg[c][3] += 1
    res = {}
    for c, (fb, fn, wb, wn) in sorted(agg.items()):
        if fn and wn:
            res[c] = round(fb / fn + wb / wn)     # bytes per launch
    if "pool_partial" in res and "pool_final" in res:       # the bench's pool_l2 class = both stages
        res["pool_l2"] = res.pop("pool_partial") + res.pop("pool_final")
    res["_note"] = ("HBM-side bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B), rocprofv3 PMC passes "
                    "of bench.py; Infinity-Cache hits included (upper bound on DRAM bytes)")
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                              "pmc_traffic.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
