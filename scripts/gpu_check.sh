#!/usr/bin/env bash
# One GPU session: parity tests, bench, rocprof kernel trace.  Every GPU step has
# its own time limit; the first failure ends the script (set -e).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-run}"
STEPS="${STEPS:-10}"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > "$OUT/${TAG}_t_kernels.log" 2>&1
  timeout -k 10 900 python -m pytest tests -m gpu -x -q --deselect tests/test_gpu_kernels.py > "$OUT/${TAG}_t_gpu.log" 2>&1
fi
timeout -k 10 400 python bench.py --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.log" 2>&1
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o prof --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-profile > "$OUT/${TAG}_prof.log" 2>&1
fi
echo done
