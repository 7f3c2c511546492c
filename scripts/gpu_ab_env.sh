#!/bin/bash
# A/B of one environment knob on the C3 bench, alternating variants twice on one box.
# VAR = the variable, VALS = its values; BENCH_ARGS = extra bench.py flags.
# Output: gpurun_out/<TAG>/ab.log (one line per run: value, per-kernel averages,
# and per-class PMC bytes when the run kept its PMC passes).
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for r in 1 2; do
  for v in $VALS; do
    lg=$OUT/run_${v//\//_}_${r}.log
    env $VAR=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-probes --no-library ${BENCH_ARGS:-} > $lg 2>&1 || { tail -20 $lg; exit 1; }
    python3 - "$lg" "$VAR=$v" <<'PY' | tee -a $OUT/ab.log
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {n: round(v["avg_us"], 1) for n, v in d["kernels"].items()}
h = d.get("hbm", {}).get("per_class", {})
b = {n: round(v["bytes_per_launch"] / 1e6, 1) for n, v in h.items() if n.startswith("gemm")}
print(sys.argv[2], d["value"], k, "MB/launch", b)
PY
  done
done
