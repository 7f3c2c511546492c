# 128 x 128 (cfg 3) against 64 x 64 (cfg 4) below one 128 x 128 tile per CU, where
# the heuristic takes 64 x 64: the crossover in M for MiniLM (f16, d 384) and
# bge-base (q4_0, d 768) widths.
set -e
for M in 1024 1536 2048 2560 3072 3584; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 1152 384 $M 0 3,4 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 1536 384 $M 1 3,4 200
done
for M in 512 768 1024 1536 1792; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 2 2304 768 $M 0 3,4 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 2 3072 768 $M 1 3,4 200
done
