#!/bin/bash
# Residual-epilogue load latency ablation (diagnostic build abl4: every residual
# row read from the tile's first 32 rows, wrong results): the two residual GEMM
# forms at C3 on random operands, production vs abl4, alternating twice.
set -o pipefail
OUT=gpurun_out/${TAG:-ablres}
mkdir -p $OUT
for r in 1 2; do
  for b in build build/abl4; do
    for f in attn_out ffn_down; do
      echo "## $b" >> $OUT/gemm.log
      BERT_LIB=$b/libbert.so timeout -k 10 120 python3 scripts/gemm_one.py $f 0 30 >> $OUT/gemm.log 2>&1 || exit $?
    done
  done
done
cat $OUT/gemm.log
