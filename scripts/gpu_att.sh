#!/usr/bin/env bash
# attention parity (kernel-level) then the attention A/B micro-bench
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="${1:-att}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k attention --timeout 120 --timeout-method thread > "gpurun_out/${T}_t_att.log" 2>&1
VARIANTS="${VARIANTS:-0,2}" ROUNDS=2 timeout -k 10 200 python scripts/att_bench.py > "gpurun_out/${T}_att_bench.log" 2>&1
echo done
