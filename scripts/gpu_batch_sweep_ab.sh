# A/B of two builds over scripts/batch_sweep.py, alternating twice on one box.
# LIBS = the builds' libbert.so paths; output gpurun_out/<TAG>/sweep.jsonl
set -o pipefail
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
for r in 1 2; do
  for lib in $LIBS; do
    BERT_LIB=$lib timeout -k 10 300 python -u scripts/batch_sweep.py >> $OUT/sweep.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  done
done
