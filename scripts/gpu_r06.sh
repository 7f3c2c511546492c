#!/bin/bash
# Round-6 GPU session.  STEPS selects (test smoke bench prof pmc rehearsal b1trace
# c2trace envelope stamps share tok),
# TAG names gpurun_out/<TAG>.  Every GPU step has its own limit; a fault, abort or
# time limit ends the script.
set -o pipefail
TAG=${TAG:-r06a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp PARITY_LOG=$OUT/parity.jsonl
STEPS=${STEPS:-"test bench prof"}
TESTS=${TESTS:-tests}
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() { local lim=$1; shift; timeout -k 10 $lim "$@"; }
if has test; then
  step ${TEST_LIMIT:-900} python -u -m pytest ${PYX:--x} -q -rf --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/gputest.log 2>&1
  rc=$?
  tail -3 $OUT/gputest.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $OUT/gputest.log; exit 1; }
fi
if has smoke; then
  step 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if has bench; then
  step 400 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -c 600 $OUT/bench.log
fi
if has prof; then
  ( cd /tmp && step 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-pmc --no-library --no-encode --no-probes --steps 10 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 ) || { tail -20 $OUT/prof.log; exit 1; }
fi
if has pmc; then
  # one counter group per rocprofv3 pass over a short bench (scripts/pmc.sh passes
  # --no-pmc itself), then the per-class summary
  step 900 bash scripts/pmc.sh ${TAG}pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
  python3 scripts/pmc_classes.py "$TAG tree, C3 bench under rocprofv3 --pmc" gpurun_out/${TAG}pmc_pmc* > $OUT/pmc_summary.txt 2>&1 || true
fi
if has rehearsal; then
  # the N-rank launch path on this one-GPU box: bench.py --gpus 2 starts its two
  # ranks itself; both drive GPU 0 (BENCH_SHARED_DEVICE=1, gloo timing collectives)
  BENCH_SHARED_DEVICE=1 step 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-probes --no-pmc --no-library --no-encode > $OUT/rehearsal.log 2>&1 || { tail -20 $OUT/rehearsal.log; exit 1; }
fi
if has b1trace; then
  # GPU-side kernel durations of the B = 1, L = 32 forward (graph replay)
  ( cd /tmp && step 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/b1prof -o b1 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/b1_trace.py 32 200 > $GRAFT_REPO_ROOT/$OUT/b1trace.log 2>&1 ) || { tail -20 $OUT/b1trace.log; exit 1; }
fi
if has c2trace; then
  # GPU-side kernel durations of the C2 forward (MiniLM f16, B 32, L 128, graph replay)
  ( cd /tmp && step 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/c2prof -o c2 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/b1_trace.py 128 200 32 all-MiniLM-L6-v2 f16 > $GRAFT_REPO_ROOT/$OUT/c2trace.log 2>&1 ) || { tail -20 $OUT/c2trace.log; exit 1; }
fi
if has envelope; then
  step 600 python -u scripts/q8_envelope.py --out $OUT/q8_envelope.jsonl > $OUT/envelope.log 2>&1 || { tail -20 $OUT/envelope.log; exit 1; }
fi
if has stamps; then
  # the shipped 256 x 128 form (cfg 2) at C3 for the four GEMMs: N K epi
  for shp in "2304 768 0" "768 768 2" "3072 768 1" "768 3072 2"; do
    STAMPS_LIB=build/stamps/libbert.so step 120 python -u scripts/gemm_stamps.py $shp 2 >> $OUT/stamps.log 2>&1 || { tail -20 $OUT/stamps.log; exit 1; }
  done
fi
if has share; then
  step 300 python -u scripts/share_curve.py --out $OUT/share_curve.jsonl > $OUT/share.log 2>&1 || { tail -20 $OUT/share.log; exit 1; }
fi
if has load; then
  # load time + peak RSS, 1 vs 8 replicas, this build vs round 5's (build/ab_r05)
  step 600 python -u scripts/load_profile.py --libs new:build/libbert.so${LOAD_OLD:+,r05:build/ab_r05/libbert.so} --out $OUT/load_profile.jsonl > $OUT/load.log 2>&1 || { tail -20 $OUT/load.log; exit 1; }
fi
if has tok; then step 300 python -u scripts/host_throughput.py tok --texts 4000 > $OUT/tok.log 2>&1 || exit 1; fi
echo session-ok
