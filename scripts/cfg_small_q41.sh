# q4_1 (C4's format) in the two small-batch tile forms (4 vs 16), as
# scripts/cfg_small_sweep.sh for the other formats.
set -e
for M in 256 512 1024 2048; do
  for a in "1024 1024 2" "1024 4096 2" "3072 1024 0" "4096 1024 1"; do
    n=${a%% *}; rest=${a#* }; k=${rest%% *}; e=${rest#* }
    timeout -k 10 60 python -u scripts/gemm_shape.py 3 $n $k $M $e 0,4,16 100
  done
done
