#!/usr/bin/env bash
# A/B of BERT_GEMM16_FLAGS values on the bench (two rounds).  usage: scripts/gpu_flags_ab.sh TAG f1 f2 ...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="$1"; shift
for r in 1 2; do
  for f in "$@"; do
    BERT_GEMM16_FLAGS=$f timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        >> "gpurun_out/${T}_f${f}_bench.log" 2>&1
  done
done
echo done
