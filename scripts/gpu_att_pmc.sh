#!/usr/bin/env bash
# attention A/B bench + PMC counters of the attention micro-bench (one pass per group)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"
mkdir -p gpurun_out
T="${1:-attp}"
VARIANTS="${VARIANTS:-0,2,3,4}" ROUNDS=2 timeout -k 10 200 python scripts/att_bench.py > "gpurun_out/${T}_att_bench.log" 2>&1
export TMPDIR=/tmp
cd /tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  VARIANTS=0,2 ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/gpurun_out/${T}_pmc$i" -o pmc \
      --kernel-include-regex attention -- python3 "$ROOT/scripts/att_bench.py" > "$ROOT/gpurun_out/${T}_pmc$i.log" 2>&1
done <<GROUPS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS
GROUPS
echo done
