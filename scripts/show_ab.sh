#!/usr/bin/env bash
# summary of a gpu_ab.sh run: test tails, bench value, per-kernel averages
T="${1:-ab}"
cd "$(dirname "$0")/.."
tail -1 "gpurun_out/${T}_t_kernels.log" 2>/dev/null
tail -1 "gpurun_out/${T}_t_gpu.log" 2>/dev/null
tail -1 "gpurun_out/${T}_bench.log" 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms/step', d['ms_per_step'], 'roofline frac', d['roofline']['frac'])
print({k: round(v['avg_us'], 1) for k, v in d['kernels'].items()})"
