#!/usr/bin/env bash
# A/B of gemm16 flags (BERT_GEMM16_FLAGS) on the bench, then PMC passes of the
# default build on the forward.  usage: scripts/gpu_prio_ab.sh TAG
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="${1:-prio}"
for f in 0 1 0 1; do
  BERT_GEMM16_FLAGS=$f timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      >> "gpurun_out/${T}_f${f}_bench.log" 2>&1
done
KREGEX=gemmz PMC_GROUPS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM" \
  bash scripts/pmc.sh "${T}"
echo done
