#!/bin/bash
# A/B of a small-batch change against OFF_ENV (the environment that turns it
# off; first used for the LN-statistics fold, BERT_STATS_FOLD_ROWS=0): the GPU
# suite once, then alternating bench runs whose probes (C2 f16 L128 B32, B 1
# L 32 q4_0) are the small-batch workloads.  Every GPU step has its own limit.
set -o pipefail
TAG=${TAG:-pfold}
OFF_ENV=${OFF_ENV:-BERT_STATS_FOLD_ROWS=0}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  step 300 python bench.py --no-cpu-baseline --no-library > $OUT/bench_on$i.log 2>&1 || { tail -20 $OUT/bench_on$i.log; exit 1; }
  env $OFF_ENV timeout -k 10 300 python bench.py --no-cpu-baseline --no-library > $OUT/bench_off$i.log 2>&1 || { tail -20 $OUT/bench_off$i.log; exit 1; }
done
python3 - $OUT <<'P'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    p = d["probes"]
    print(os.path.basename(f), "C3 %.1f sent/s" % d["value"], "| C2 %.0f sent/s %.3f ms" % (p["f16_mfma"]["sentences_per_s"], p["f16_mfma"]["ms_per_batch"]),
          "| B1 L32 %.1f us" % p["q4_0_hbm"]["latency_us"])
P
echo ab-ok
