#!/bin/bash
# A/B of a GEMM change: GEMM kernel parity tests on the new build, the GEMM
# micro-benchmark (C3 M = 32768 and B = 1 M = 64) and the C3 forward, alternating
# build/libbert.so (new) with build/old/libbert.so; every step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-deqab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for r in 1 2; do
  for m in 32768 64; do
    for b in build build/old; do
      echo "## $b M=$m" >> $OUT/gemm.log
      SWEEP_M=$m BERT_LIB=$b/libbert.so timeout -k 10 120 python3 scripts/gemm_one.py all 0 30 >> $OUT/gemm.log 2>&1 || exit $?
    done
  done
done
cat $OUT/gemm.log
TAG=${TAG:-deqab}/fwd LIBS=old ROUNDS=2 bash scripts/gpu_lib_ab.sh
