#!/bin/bash
# Chained forward A/B: GPU tests (default chains), then alternating bench runs
# over BERT_CHAINS (1 = one chain) and BERT_GRAPHS (0 = eager) on the same box.
set -o pipefail
OUT=gpurun_out/${TAG:-chains}
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
CFGS=${CFGS:-"1:1 2:1 4:1 1:0 2:0 4:0"}
for r in 1 2; do
  for cfg in $CFGS; do
    c=${cfg%:*}; g=${cfg#*:}
    BERT_CHAINS=$c BERT_GRAPHS=$g timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --no-profile --steps 30 > $OUT/bench_c${c}_g${g}_r$r.log 2>&1 || { tail -20 $OUT/bench_c${c}_g${g}_r$r.log; exit 1; }
    python3 -c "import json,sys;l=[x for x in open('$OUT/bench_c${c}_g${g}_r$r.log') if x.startswith('{')][-1];d=json.loads(l);print('chains=$c graphs=$g round=$r',d['value'],d['ms_per_step'])"
  done
done
