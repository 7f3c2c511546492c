# (configs 20 / 21 existed only in the round-6 experiment build: profiles/r06_gemm_128x192_ab.log)
# The 128 x 192 tile configs (20: 8 waves, 21: 4 waves) against 128 x 128 (3) at
# C2's widths and at tile counts either side of one per CU.
set -e
for fmt in 1 2; do
  for args in "1152 384 4096 0" "1536 384 4096 1" "1152 384 3584 0" "1536 384 2560 1" "2304 768 2048 0" "3072 768 2048 1"; do
    timeout -k 10 60 python -u scripts/gemm_shape.py $fmt $args 3,20,21 200
  done
done
