#!/usr/bin/env bash
# kernel parity -> forward parity -> bench, each under its own limit; stops at
# the first failure.  usage: scripts/gpu_ab.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="${1:-ab}"
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -x -q > "gpurun_out/${T}_t_kernels.log" 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q --deselect tests/test_gpu_kernels.py > "gpurun_out/${T}_t_gpu.log" 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:-} > "gpurun_out/${T}_bench.log" 2>&1
echo done
