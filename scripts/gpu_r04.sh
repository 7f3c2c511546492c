#!/bin/bash
# Round-4 GPU session: tests, bench (with its own rocprofv3 PMC passes), rocprofv3
# kernel stats of the bench, in-process multi-GPU, host throughput.  Every GPU
# step has its own limit; the chain stops at the first failure.  STEPS selects
# steps, TAG names the output directory gpurun_out/<TAG>.
set -o pipefail
TAG=${TAG:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PARITY_LOG=$OUT/parity.jsonl
STEPS=${STEPS:-"test bench prof tok"}
TESTS=${TESTS:-tests}
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if has test; then
  step 900 python -u -m pytest ${PYX:--x} -q -rf --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/gputest.log 2>&1
  rc=$?
  tail -3 $OUT/gputest.log
  # rc 1 = assertion failures only (no fault, no timeout): the later steps still run
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $OUT/gputest.log; exit 1; }
fi
if has bench; then
  step 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -c 600 $OUT/bench.log
fi
if has prof; then
  ( cd /tmp && step 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-pmc --no-library --steps 10 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
fi
if has inproc; then
  BERT_DEVICES=0,0,0,0,0,0,0,0 step 600 python -u bench.py --inproc --gpus 8 --steps 5 --warmup 1 > $OUT/inproc.log 2>&1 || { tail -20 $OUT/inproc.log; exit 1; }
  BERT_DEVICES=0 step 600 python -u bench.py --inproc --gpus 1 --steps 5 --warmup 1 >> $OUT/inproc.log 2>&1 || { tail -20 $OUT/inproc.log; exit 1; }
fi
if has tok; then step 300 python -u scripts/host_throughput.py tok --texts 4000 > $OUT/tok.log 2>&1 || exit 1; fi
if has server; then step 400 python -u scripts/host_throughput.py server > $OUT/server.log 2>&1 || { tail -20 $OUT/server.log; exit 1; }; fi
echo session-ok
