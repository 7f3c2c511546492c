set -e
cd $GRAFT_REPO_ROOT
SWEEP_ROUNDS=1 VARIANTS=z0:0x1000,z1:0x1001,z3:0x1003 timeout -k 10 200 python scripts/gemm16_sweep.py > gpurun_out/sw1.log 2>&1
PMC_GROUPS=$'FETCH_SIZE\nWRITE_SIZE' bash scripts/pmc.sh r01e
echo ok
