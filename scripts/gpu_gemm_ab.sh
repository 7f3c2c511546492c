#!/bin/bash
# GEMM micro-benchmark of the four C3 forms: LN-fold (production) vs plain, and
# each tile config; every step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-gab}
mkdir -p $OUT
for r in 1 2; do
  for cfg in 0 0x100 3 0x103; do
    timeout -k 10 120 python3 scripts/gemm_one.py all $cfg 20 >> $OUT/gemm.log 2>&1 || exit $?
  done
done
cat $OUT/gemm.log
