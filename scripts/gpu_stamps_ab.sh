#!/usr/bin/env bash
# gemm16 stamps (scripts/gemm16_stamps.py) per library variant.  usage: scripts/gpu_stamps_ab.sh TAG base v1 v2 ...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="$1"; shift
for v in "$@"; do
  lib="$(pwd)/build/libbert.so"; [ "$v" != base ] && lib="$(pwd)/build_ab/$v/libbert.so"
  echo "#### $v" >> "gpurun_out/${T}_stamps.log"
  BERT_LIB="$lib" CFGS="${CFGS:-2}" timeout -k 10 200 python scripts/gemm16_stamps.py >> "gpurun_out/${T}_stamps.log" 2>&1
done
echo done
