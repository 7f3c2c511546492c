# The residual GEMMs (epi 2: O-proj, FFN-down) at mid-size M: the tile configs the
# heuristic chooses among (3: 128 x 128, 4: 2-wave 64 x 64, 16: 4-wave 64 x 64).
set -e
for M in 512 1024 2048 3072 4096; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 384 384 $M 2 0,3,4,16 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 384 1536 $M 2 0,3,4,16 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 2 768 768 $M 2 0,3,4,16 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 2 768 3072 $M 2 0,3,4,16 200
done
