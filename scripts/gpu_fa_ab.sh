#!/bin/bash
# A/B of the GEMM tile configs: cfg 2 (4 waves 256 x 128, 32 features per wave)
# against cfg 5 (4 waves 128 x 256, 64 features per wave): GEMM kernel tests of
# every form, the micro-bench on every C3 form, and the forward (alternating).
set -o pipefail
OUT=gpurun_out/${TAG:-fa}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
step 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm" > $OUT/kt.log 2>&1 || { tail -30 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log
for c in 2 5 2 5; do step 120 python -u scripts/gemm_one.py all $c 20 >> $OUT/micro.log 2>&1 || { tail $OUT/micro.log; exit 1; }; done
cat $OUT/micro.log
for c in 0 5 0 5; do
  BERT_GEMM_CFG=$c step 300 python -u bench.py --no-cpu-baseline --no-probes --no-library > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: round(v['avg_us'], 1) for k, v in d['kernels'].items()})" $OUT/bench_$c.log $c | tee -a $OUT/bench_ab.log
done
echo ab-ok
