# 256 x 128 (cfg 2) against 128 x 128 (cfg 3) where 128 x 128 tiles number one to
# two per CU (the heuristic takes 3 there): MiniLM (f16) and bge-base (q4_0) widths.
set -e
for M in 3072 4096 5120 6144 7168; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 1152 384 $M 0 2,3 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 1536 384 $M 1 2,3 200
done
for M in 2048 2560 3072 3584; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 2 2304 768 $M 0 2,3 200
  timeout -k 10 60 python -u scripts/gemm_shape.py 2 3072 768 $M 1 2,3 200
done
