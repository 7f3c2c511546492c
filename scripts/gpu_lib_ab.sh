#!/usr/bin/env bash
# A/B of library builds (scripts/build_variant.sh): per variant, GEMM/attention
# kernel parity then the bench; "base" = build/libbert.so.  Two rounds.
# usage: scripts/gpu_lib_ab.sh TAG base pf2 pf4 ...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="$1"; shift
for v in "$@"; do
  lib="$(pwd)/build/libbert.so"; [ "$v" != base ] && lib="$(pwd)/build_ab/$v/libbert.so"
  BERT_LIB="$lib" timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > "gpurun_out/${T}_${v}_t_kernels.log" 2>&1
done
for r in 1 2; do
  for v in "$@"; do
    lib="$(pwd)/build/libbert.so"; [ "$v" != base ] && lib="$(pwd)/build_ab/$v/libbert.so"
    BERT_LIB="$lib" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        >> "gpurun_out/${T}_${v}_bench.log" 2>&1
  done
done
echo done
