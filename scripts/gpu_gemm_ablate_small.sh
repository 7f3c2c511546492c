#!/bin/bash
# GEMM K-loop cost ablations at small batches (diagnostic builds as
# gpu_gemm_ablate.sh): the four bge-base forms at M = 64 and 4096 rows.
set -o pipefail
OUT=gpurun_out/${TAG:-ablsmall}
mkdir -p $OUT
for r in 1 2; do
  for m in 64 4096; do
    for b in build build/abl1 build/abl2 build/abl3; do
      echo "## $b M=$m" >> $OUT/gemm.log
      SWEEP_M=$m BERT_LIB=$b/libbert.so timeout -k 10 120 python3 scripts/gemm_one.py all 0 50 >> $OUT/gemm.log 2>&1 || exit $?
    done
  done
done
cat $OUT/gemm.log
