#!/usr/bin/env bash
# A/B of one environment variable on the bench (two rounds), kernel tests per value first.
# usage: scripts/gpu_env_ab.sh TAG VAR v1 v2 ...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="$1"; VAR="$2"; shift 2
for r in 1 2; do
  for v in "$@"; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        >> "gpurun_out/${T}_${v//,/_}_bench.log" 2>&1
  done
done
echo done
