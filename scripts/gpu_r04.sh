#!/bin/bash
# Round-4 GPU session: tests, bench (with its own rocprofv3 PMC passes), rocprofv3
# kernel stats of the bench, in-process multi-GPU, host throughput.  Every GPU
# step has its own limit; the chain stops at the first failure.  STEPS selects
# steps, TAG names the output directory gpurun_out/<TAG>.
set -o pipefail
TAG=${TAG:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PARITY_LOG=$OUT/parity.jsonl
STEPS=${STEPS:-"test bench prof tok"}
TESTS=${TESTS:-tests}
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if has test; then
  step 900 python -u -m pytest ${PYX:--x} -q -rf --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/gputest.log 2>&1
  rc=$?
  tail -3 $OUT/gputest.log
  # rc 1 = assertion failures only (no fault, no timeout): the later steps still run
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $OUT/gputest.log; exit 1; }
fi
if has bench; then
  step 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -c 600 $OUT/bench.log
fi
if has prof; then
  ( cd /tmp && step 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-pmc --no-library --steps 10 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
fi
if has inproc; then
  BERT_DEVICES=0,0,0,0,0,0,0,0 step 600 python -u bench.py --inproc --gpus 8 --steps 5 --warmup 1 > $OUT/inproc.log 2>&1 || { tail -20 $OUT/inproc.log; exit 1; }
  BERT_DEVICES=0 step 600 python -u bench.py --inproc --gpus 1 --steps 5 --warmup 1 >> $OUT/inproc.log 2>&1 || { tail -20 $OUT/inproc.log; exit 1; }
fi
if has attab; then
  # attention store order: after the S barrier (default) vs before it
  for r in 1 2; do
    for e in 0 1; do
      BERT_ATT_EARLY_STORE=$e step 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --no-pmc > $OUT/attab_${e}_${r}.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/attab_${e}_${r}.log').read().strip().splitlines()[-1]); print('early_store=$e', d['value'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})" | tee -a $OUT/attab.log
    done
  done
fi
if has smallab; then
  # the 64-row GEMM forms on the small-batch probes (C2, B 1 L 32), alternating
  for r in 1 2; do
    for c in ${SMALLC:-4 7 8}; do
      BERT_GEMM_SMALL=$c step 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-library --no-pmc --no-profile > $OUT/smallab_${c}_${r}.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/smallab_${c}_${r}.log').read().strip().splitlines()[-1]); p=d['probes']; print('small=$c', 'C2', p['f16_mfma']['sentences_per_s'], 'B1', p['q4_0_hbm']['latency_us'], p['q4_0_hbm']['kernel_avg_us'])" | tee -a $OUT/smallab.log
    done
  done
fi
if has gemmab; then
  # weight formats and tile configs of the C3 GEMM forms on random operands
  for f in 1 2; do SWEEP_FMT=$f step 120 python -u scripts/gemm_one.py all 0 20 >> $OUT/gemmab.log 2>&1 || exit 1; done
  SWEEP_FMT=2 step 120 python -u scripts/gemm_one.py all 5 20 >> $OUT/gemmab.log 2>&1 || exit 1
  cat $OUT/gemmab.log
fi
if has wide; then
  # 8-wave 256 x 256 tiles (cfg 9 NS 2, cfg 10 NS 3; one workgroup per CU) against production (2)
  for r in 1 2; do for c in 2 9 10; do step 120 python -u scripts/gemm_one.py all $c 20 >> $OUT/wide.log 2>&1 || exit 1; done; done
  for c in 2 9 10; do STAMPS_LIB=build/stamps/libbert.so step 120 python -u scripts/gemm_stamps.py 3072 768 1 $c >> $OUT/wide_stamps.log 2>&1 || exit 1; done
  cat $OUT/wide.log
fi
if has dmastamp; then
  for a in "3072 768 1" "2304 768 0" "768 3072 2"; do STAMPS_LIB=build/stamps/libbert.so step 120 python -u scripts/gemm_stamps.py $a 2 >> $OUT/dma_stamps.log 2>&1 || exit 1; done
  cat $OUT/dma_stamps.log
fi
if has xi; then
  # X pieces interleaved among the MFMAs (cfg 11) against the burst in front of them (2)
  for r in 1 2; do for c in 2 11 12; do step 120 python -u scripts/gemm_one.py all $c 20 >> $OUT/xi.log 2>&1 || exit 1; done; done
  for r in 1 2; do for c in 0 11 12; do
    BERT_GEMM_CFG=$c step 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --no-pmc > $OUT/xi_${c}_${r}.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/xi_${c}_${r}.log').read().strip().splitlines()[-1]); print('cfg=$c', d['value'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})" | tee -a $OUT/xi.log
  done; done
  cat $OUT/xi.log
fi
if has xismall; then
  # interleaved X pieces on the 128- and 64-row forms (BERT_GEMM_XI=1) on the probes, alternating
  for r in 1 2; do for e in 0 1; do
    BERT_GEMM_XI=$e step 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-library --no-pmc --no-profile > $OUT/xismall_${e}_${r}.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/xismall_${e}_${r}.log').read().strip().splitlines()[-1]); p=d['probes']; print('xi=$e', 'C3', d['value'], 'C2', p['f16_mfma']['sentences_per_s'], 'B1', p['q4_0_hbm']['latency_us'])" | tee -a $OUT/xismall.log
  done; done
fi
if has b1stamp; then
  for a in "2304 768 0" "768 768 2" "3072 768 1" "768 3072 2"; do SWEEP_M=64 STAMPS_LIB=build/stamps/libbert.so step 120 python -u scripts/gemm_stamps.py $a ${B1CFG:-16} >> $OUT/b1_stamps.log 2>&1 || exit 1; done
  ( cd /tmp && step 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/b1prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/b1_trace.py 32 50 > $GRAFT_REPO_ROOT/$OUT/b1_trace.log 2>&1 ) || exit 1
  cat $OUT/b1_stamps.log
fi
if has ntab; then
  # non-temporal output stores of the 256-row GEMM tiles (default) vs plain stores (BERT_GEMM_NT=0), alternating
  for r in 1 2; do
    for n in -1 0; do
      BERT_GEMM_NT=$n step 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --no-pmc > $OUT/ntab_${n}_${r}.log 2>&1 || exit 1
      python3 -c "import json; d=json.loads(open('$OUT/ntab_${n}_${r}.log').read().strip().splitlines()[-1]); print('nt=$n', d['value'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})" | tee -a $OUT/ntab.log
    done
  done
fi
if has c2sweep; then
  # every GEMM on one tile config (BERT_GEMM_CFG) against the heuristic (0): the small-batch probes
  for c in ${SWEEPC:-0 3 4 7 13 14 16 0}; do
    BERT_GEMM_CFG=$c step 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-library --no-pmc > $OUT/c2sweep_${c}.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/c2sweep_${c}.log').read().strip().splitlines()[-1]); p=d['probes']; print('cfg=$c', 'C2', p['f16_mfma']['sentences_per_s'], p['f16_mfma']['kernel_avg_us'], 'B1', p['q4_0_hbm']['latency_us'])" | tee -a $OUT/c2sweep.log
  done
fi
if has poolab; then
  # one-launch pool over <= 4 chunks (default) vs the two launches (BERT_POOL_ONE=0), alternating: C2 probe
  for r in 1 2; do for e in 1 0; do
    BERT_POOL_ONE=$e step 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-library --no-pmc > $OUT/poolab_${e}_${r}.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/poolab_${e}_${r}.log').read().strip().splitlines()[-1]); p=d['probes']; print('pool_one=$e', 'C2', p['f16_mfma']['sentences_per_s'], p['f16_mfma']['kernel_avg_us'], 'B1', p['q4_0_hbm']['latency_us'])" | tee -a $OUT/poolab.log
  done; done
fi
if has tok; then step 300 python -u scripts/host_throughput.py tok --texts 4000 > $OUT/tok.log 2>&1 || exit 1; fi
if has server; then step 400 python -u scripts/host_throughput.py server > $OUT/server.log 2>&1 || { tail -20 $OUT/server.log; exit 1; }; fi
echo session-ok
