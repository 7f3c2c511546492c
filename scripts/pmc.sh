#!/usr/bin/env bash
# PMC counter passes (one counter group per rocprofv3 run, no tracing domains
# besides kernel dispatch).  Output: gpurun_out/<tag>_pmc<i>/
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT="$(pwd)"
OUT="$ROOT/gpurun_out"
TAG="${1:-pmc}"
ARGS="${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-probes --no-library --no-pmc}"
# (--no-pmc: no nested rocprofv3 passes from the profiled process; bench.py's
# under_profiler() check is the second safeguard, not the only one)
# PMC_SCRIPT: profile that python script (repo-relative) instead of bench.py
TARGET="$ROOT/${PMC_SCRIPT:-bench.py}"
[ -n "${PMC_SCRIPT:-}" ] && ARGS="${PMC_SCRIPT_ARGS:-}"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${TAG}_pmc$i" -o pmc \
      ${KREGEX:+--kernel-include-regex "$KREGEX"} -- python3 "$TARGET" $ARGS > "$OUT/${TAG}_pmc$i.log" 2>&1
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum}
GROUPS
echo done
