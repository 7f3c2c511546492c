#!/bin/bash
# GEMM K-loop cost ablations (diagnostic builds, wrong results by design): the C3 forms
# on random operands with the production library, without X LDS-DMA pieces (abl1),
# without dequantization (abl2), without both (abl3); alternating twice.
set -o pipefail
OUT=gpurun_out/${TAG:-abl}
mkdir -p $OUT
for r in 1 2; do
  for b in build build/abl1 build/abl2 build/abl3; do
    echo "## $b" >> $OUT/gemm.log
    BERT_LIB=$b/libbert.so timeout -k 10 120 python3 scripts/gemm_one.py all 0 20 >> $OUT/gemm.log 2>&1 || exit $?
  done
done
cat $OUT/gemm.log
