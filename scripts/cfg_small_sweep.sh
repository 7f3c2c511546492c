# The two small-batch tile forms (4: 2-wave 64 x 64, 16: 4-wave 64 x 64 with
# wave-private X rings) per weight format and GEMM width, M 64 .. 2048.
set -e
for M in 64 128 256 512 1024 2048; do
  for fmt in 1 2 8; do
    if [ $fmt = 1 ]; then set -- "384 384 2" "384 1536 2" "1152 384 0" "1536 384 1"; else set -- "768 768 2" "768 3072 2" "2304 768 0" "3072 768 1"; fi
    for a in "$@"; do
      n=${a%% *}; rest=${a#* }; k=${rest%% *}; e=${rest#* }
      timeout -k 10 60 python -u scripts/gemm_shape.py $fmt $n $k $M $e 0,4,16 100
    done
  done
done
