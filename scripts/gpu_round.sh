#!/bin/bash
# One GPU session: gpu tests, bench, rocprof kernel stats.  Every GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 10 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 )
rc=$?
tail -3 $OUT/gputest.log; tail -c 600 $OUT/bench.log
exit $rc
