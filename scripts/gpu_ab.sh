#!/bin/bash
# Forward A/B: the in-tree build against another build (LIB_A, default
# build/base/libbert.so = the last commit), alternating bench runs on one box;
# optional kernel tests (TESTS="-k gemm") and GEMM stamps first (STAMPS=1).
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
LIB_A=${LIB_A:-build/base/libbert.so}
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if [ -n "$TESTS" ]; then
  step 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/kt.log 2>&1 || { tail -30 $OUT/kt.log; exit 1; }
  tail -1 $OUT/kt.log
fi
if [ -n "$STAMPS" ]; then
  for s in "3072 768 1 2" "2304 768 0 2" "768 768 2 2" "768 3072 2 2"; do step 60 python -u scripts/gemm_stamps.py $s >> $OUT/stamps.log 2>&1 || exit 1; done
  grep -E "^N=|prologue|K loop  |epilogue" $OUT/stamps.log
fi
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: round(v['avg_us'], 1) for k, v in d['kernels'].items()})" "$@"; }
for r in 1 2; do
  BERT_LIB=$LIB_A step 300 python -u bench.py --no-cpu-baseline --no-probes --no-library > $OUT/bench_a$r.log 2>&1 || { tail -20 $OUT/bench_a$r.log; exit 1; }
  summ $OUT/bench_a$r.log A | tee -a $OUT/ab.log
  step 300 python -u bench.py --no-cpu-baseline --no-probes --no-library > $OUT/bench_b$r.log 2>&1 || { tail -20 $OUT/bench_b$r.log; exit 1; }
  summ $OUT/bench_b$r.log B | tee -a $OUT/ab.log
done
echo ab-ok
