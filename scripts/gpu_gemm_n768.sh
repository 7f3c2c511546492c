#!/bin/bash
# GEMM micro-benchmark of the N = d forms at C3 (O-proj, FFN-down; random operands,
# the forward's residual LN-fold form): tile configs 2 (production), 11, 3, 12,
# alternating twice; each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-n768}
mkdir -p $OUT
for r in 1 2; do
  for cfg in 2 3 12 11; do
    for f in attn_out ffn_down; do
      timeout -k 10 120 python3 scripts/gemm_one.py $f $cfg 20 >> $OUT/gemm.log 2>&1 || exit $?
    done
  done
done
cat $OUT/gemm.log
