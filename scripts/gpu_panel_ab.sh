#!/usr/bin/env bash
# panel-LN hand-off A/B: kernel parity, then the bench per BERT_PANEL_VARIANT and
# with the separate LN kernel (BERT_PANEL_LN=0).  usage: scripts/gpu_panel_ab.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="${1:-pab}"
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > "gpurun_out/${T}_t_kernels.log" 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q --deselect tests/test_gpu_kernels.py > "gpurun_out/${T}_t_gpu.log" 2>&1
for v in 0 1 2; do
  BERT_PANEL_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      > "gpurun_out/${T}_v${v}_bench.log" 2>&1
done
BERT_PANEL_LN=0 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "gpurun_out/${T}_off_bench.log" 2>&1
echo done
