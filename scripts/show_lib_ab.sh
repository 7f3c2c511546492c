#!/usr/bin/env bash
# summary of gpu_lib_ab.sh: usage scripts/show_lib_ab.sh TAG v1 v2 ...
cd "$(dirname "$0")/.."
T="$1"; shift
for v in "$@"; do
  echo "== $v $(tail -n1 gpurun_out/${T}_${v}_t_kernels.log)"
  grep '^{' "gpurun_out/${T}_${v}_bench.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(' ', d['value'], {k: round(v['avg_us'], 1) for k, v in d['kernels'].items()})"
done
