#!/bin/bash
# Chained forward A/B: optional GPU tests, then alternating bench runs over
# configurations CHAINS:LOCKSTEP (BERT_CHAINS 1 = one chain; BERT_LOCKSTEP k =
# chains wait for each other every k half-layers, 0 = free-running) on one box.
set -o pipefail
OUT=gpurun_out/${TAG:-chains}
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
CFGS=${CFGS:-"1:0 2:0 2:1 2:2"}
for r in ${ROUNDS:-1 2}; do
  for cfg in $CFGS; do
    c=${cfg%:*}; k=${cfg#*:}
    BERT_CHAINS=$c BERT_LOCKSTEP=$k timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --no-profile --steps 30 > $OUT/bench_c${c}_k${k}_r$r.log 2>&1 || { tail -20 $OUT/bench_c${c}_k${k}_r$r.log; exit 1; }
    python3 -c "import json,sys;l=[x for x in open('$OUT/bench_c${c}_k${k}_r$r.log') if x.startswith('{')][-1];d=json.loads(l);print('chains=$c lockstep=$k round=$r',d['value'],d['ms_per_step'])"
  done
done
