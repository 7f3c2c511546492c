#!/bin/bash
# rocprofv3 counter passes (one group per run) over the GEMM micro-benchmark of one
# form (CASE) for the tile configs in CFGS; the counter list of the box first.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc3}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for cfg in ${CFGS:-2}; do
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/${cfg}_p$i -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/gemm_one.py ${CASE:-ffn_up} $cfg 10 > $OUT/${cfg}_p$i.log 2>&1 || exit $?
  done <<GROUPS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU
TA_TA_BUSY_sum TA_BUFFER_LOAD_WAVEFRONTS_sum
GROUPS
done
echo done
