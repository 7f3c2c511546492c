#!/usr/bin/env python3
"""Per-kernel-class PMC summary of scripts/pmc.sh runs (one counter group per
rocprofv3 pass over the same bench.py invocation): counters summed over every
launch of the class, then the derived ratios DESIGN.md §3 quotes.
usage: pmc_classes.py TITLE DIR [DIR ...]   (e.g. gpurun_out/r04pmc_pmc*)

  mfma_busy   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
  parked      SQ_WAIT_ANY / SQ_WAVE_CYCLES        (s_waitcnt / barrier)
  issue_stall SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  active      SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu_per_mfma, lds_bank_conflict (per LDS-array cycle),
  lds_active  SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 * 256 CUs), tcc_hit."""
import collections
import csv
import glob
import json
import os
import re
import sys


def kclass(name):
    m = re.search(r"gemmz_kernelILi(\d+)ELi(\d+)E", name)
    if m:
        return {"0": "gemm_qkv", "1": "gemm_ffn_up", "2": "gemm_res (O-proj + FFN-down)"}[m.group(2)]
    for key, cls in (("attention", "attention"), ("embed_ln", "embed_ln"), ("ln_stats", "ln_stats"), ("pool", "pool")):
        if key in name:
            return cls
    return None


title, dirs = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            c = kclass(r["Kernel_Name"])
            if c:
                agg[c][r["Counter_Name"]] += float(r["Counter_Value"])


def ratio(a, b):
    return a / b if b else float("nan")


print(f"# {title}")
print("# Sums over every launch of the class (one counter group per rocprofv3 pass; scripts/pmc.sh). "
      "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs); wave-cycle shares from "
      "SQ_WAIT_ANY (parked: s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall), SQ_ACTIVE_INST_ANY; "
      "lds_active = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 * 256 CUs).")
for c in ("gemm_qkv", "attention", "gemm_res (O-proj + FFN-down)", "gemm_ffn_up", "embed_ln", "ln_stats", "pool"):
    if c not in agg:
        continue
    v = agg[c]
    g = v.get("GRBM_GUI_ACTIVE", 0.0) / 8
    wc = v.get("SQ_WAVE_CYCLES", 0.0)
    parts = [
        ("mfma_busy", ratio(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), g * 1024), 3),
        ("parked", ratio(v.get("SQ_WAIT_ANY", 0.0), wc), 2),
        ("issue_stall", ratio(v.get("SQ_WAIT_INST_ANY", 0.0), wc), 2),
        ("active", ratio(v.get("SQ_ACTIVE_INST_ANY", 0.0), wc), 2),
        ("valu_per_mfma", ratio(v.get("SQ_INSTS_VALU", 0.0), v.get("SQ_INSTS_MFMA", 0.0)), 1),
        ("lds_bank_conflict", ratio(v.get("SQ_LDS_BANK_CONFLICT", 0.0), v.get("SQ_LDS_IDX_ACTIVE", 0.0)), 3),
        ("lds_active", ratio(v.get("SQ_LDS_IDX_ACTIVE", 0.0), g * 256), 3),
        ("tcc_hit", ratio(v.get("TCC_HIT_sum", 0.0), v.get("TCC_HIT_sum", 0.0) + v.get("TCC_MISS_sum", 0.0)), 2),
    ]
    print(f"{c}: " + "  ".join(f"{k} {x:.{n}f}" for k, x, n in parts))
    print("   raw: " + json.dumps(dict(sorted(v.items()))))
