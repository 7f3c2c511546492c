#!/bin/bash
# Small-batch GEMM micro-benchmark: the four bge-base forms at M = 64 / 128 / 4096
# rows in f16 (fmt 1) vs q4_0 (fmt 2) weights, the production tile heuristic,
# alternating twice; each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-smallfmt}
mkdir -p $OUT
for r in 1 2; do
  for m in 64 128 4096; do
    for f in 2 1; do
      SWEEP_M=$m SWEEP_FMT=$f timeout -k 10 120 python3 scripts/gemm_one.py all 0 50 >> $OUT/gemm.log 2>&1 || exit $?
    done
  done
done
cat $OUT/gemm.log
