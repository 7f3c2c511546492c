#!/bin/bash
# Round-2 GPU session: tests, bench, in-process multi-GPU (two replicas on one
# GPU), host throughput (tokenizer, server), PMC traffic passes.  Every GPU step
# has its own limit; the chain stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-r02e}
mkdir -p $OUT
export TMPDIR=/tmp PARITY_LOG=$OUT/parity.jsonl
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
step 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
step 300 python scripts/host_throughput.py tok --texts 4000 > $OUT/tok.log 2>&1 || exit 1
step 400 python scripts/host_throughput.py server > $OUT/server.log 2>&1 || { tail -20 $OUT/server.log; exit 1; }
BERT_DEVICES=0,0 step 600 python bench.py --inproc --gpus 2 --steps 5 --warmup 1 > $OUT/inproc.log 2>&1 || { tail -20 $OUT/inproc.log; exit 1; }
if [ -n "$PMC" ]; then
  bash scripts/pmc.sh ${TAG:-r02e} > $OUT/pmc.log 2>&1 || exit 1
  python3 scripts/pmc_traffic.py gpurun_out/${TAG:-r02e}_pmc3 gpurun_out/${TAG:-r02e}_pmc4 $OUT/pmc_traffic.json > /dev/null || exit 1
fi
echo session-ok
