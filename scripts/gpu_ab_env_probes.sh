#!/bin/bash
# A/B of one environment knob on the full bench line (C3 + the probes: B 1, C2, C1,
# C4 shard, C5), alternating the values twice on one box.  VAR = the variable,
# VALS = its values.  Output: gpurun_out/<TAG>/ab.log, one line per run.
set -o pipefail
OUT=gpurun_out/${TAG:-abp}
mkdir -p $OUT
for r in 1 2; do
  for v in $VALS; do
    lg=$OUT/run_${v//\//_}_${r}.log
    env $VAR=$v timeout -k 10 400 python -u bench.py --no-pmc --no-encode --no-cpu-baseline ${BENCH_ARGS:-} > $lg 2>&1 || { tail -20 $lg; exit 1; }
    python3 - "$lg" "$VAR=$v" <<'PY' | tee -a $OUT/ab.log
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["probes"]
k = lambda q: {n: round(v, 1) for n, v in p[q].get("kernel_avg_us", {}).items() if n in ("embed_ln", "attention", "pool_l2")}
print(sys.argv[2], "C3", d["value"], "B1", p["q4_0_hbm"]["latency_us"], k("q4_0_hbm"), "C2", p["f16_mfma"]["sentences_per_s"],
      k("f16_mfma"), "C1", p["c1_f32"].get("latency_us"), "C4", p["c4_shard"]["sentences_per_s"], "C5", p["c5_ragged"]["sentences_per_s"])
PY
  done
done
