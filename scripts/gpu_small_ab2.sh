#!/bin/bash
# A/B of a small-batch change selected by an environment (ON_ENV; round 5:
# BERT_GEMM_SMALL=17: the 16-feature-wave tiles) against the default heuristic:
# the GEMM kernel tests, the forward tests with ON_ENV, then alternating bench
# runs whose probes (C2 f16 L128 B32, B 1 L 32 q4_0) are the small-batch
# workloads.  Every GPU step has its own limit; the first failure ends it.
set -o pipefail
TAG=${TAG:-smallab}
ON_ENV=${ON_ENV:?set ON_ENV to the environment that turns the change on}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $OUT/t_kernels.log 2>&1 || { tail -30 $OUT/t_kernels.log; exit 1; }
  tail -1 $OUT/t_kernels.log
  env $ON_ENV timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${ON_TESTS:-tests/test_gpu_forward.py} > $OUT/t_forward_on.log 2>&1 || { tail -30 $OUT/t_forward_on.log; exit 1; }
  tail -1 $OUT/t_forward_on.log
fi
B="--no-cpu-baseline --no-library --no-pmc --no-encode --steps 20"
for i in $(seq 1 ${ROUNDS:-2}); do
  step 300 python bench.py $B > $OUT/bench_off$i.log 2>&1 || { tail -20 $OUT/bench_off$i.log; exit 1; }
  env $ON_ENV timeout -k 10 300 python bench.py $B > $OUT/bench_on$i.log 2>&1 || { tail -20 $OUT/bench_on$i.log; exit 1; }
done
python3 - $OUT <<'P'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.log")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    p = d["probes"]
    print(os.path.basename(f), "C3 %.1f sent/s" % d["value"], "| C2 %.0f sent/s %.3f ms" % (p["f16_mfma"]["sentences_per_s"], p["f16_mfma"]["ms_per_batch"]),
          "| B1 L32 %.1f us" % p["q4_0_hbm"]["latency_us"])
    for k in ("f16_mfma", "q4_0_hbm"):
        print("    ", k, " ".join("%s=%.2f" % kv for kv in p[k]["kernel_avg_us"].items()))
P
echo ab-ok
