#!/bin/bash
# GPU session: selected gpu tests (args), then the bench.  Every GPU step has its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
export TMPDIR=/tmp PARITY_LOG=$OUT/parity.jsonl
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu "$@" > $OUT/gputest.log 2>&1
rc=$?
tail -5 $OUT/gputest.log
[ $rc -ne 0 ] && exit $rc
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
  tail -c 1500 $OUT/bench.log
fi
