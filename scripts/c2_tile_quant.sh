# GEMM time vs tile count (cfg 3, 128 x 128 tiles, f16 weights) at C2's widths:
# where the one-tile-per-CU step falls.  Output: one line per shape.
set -e
for M in 2048 2304 2560 2688 2816 2944 3072 3328 3584 3840 4096; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 1536 384 $M 1 3 200
done
for M in 3072 3328 3456 3584 3712 3840 4096; do
  timeout -k 10 60 python -u scripts/gemm_shape.py 1 1152 384 $M 0 3 200
done
python -c "import torch; p=torch.cuda.get_device_properties(0); print('CUs', p.multi_processor_count)"
