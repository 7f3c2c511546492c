set -o pipefail
mkdir -p gpurun_out/tq8
BERT_LIB=build/tq8/libbert.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemm" > gpurun_out/tq8/tests.log 2>&1 || { tail -30 gpurun_out/tq8/tests.log; exit 1; }
tail -1 gpurun_out/tq8/tests.log
for lib in build/libbert.so build/tq8/libbert.so; do
  n=$(echo $lib | tr '/' '_')
  BERT_LIB=$lib timeout -k 10 200 python -u scripts/ab_bits.py gpurun_out/tq8/$n.q8.npy bge-base-zh-v1.5 q8_0 > /dev/null 2>&1 || exit 1
  BERT_LIB=$lib timeout -k 10 200 python -u scripts/ab_bits.py gpurun_out/tq8/$n.q8s.npy all-MiniLM-L6-v2 q8_0 > /dev/null 2>&1 || exit 1
done
python3 -c "
import numpy as np
for t in ('q8','q8s'):
    a=np.load('gpurun_out/tq8/build_libbert.so.%s.npy'%t); b=np.load('gpurun_out/tq8/build_tq8_libbert.so.%s.npy'%t)
    print(t, a.shape, 'bitwise equal', np.array_equal(a.view(np.uint32), b.view(np.uint32)))
"
for M in 32768; do
  for lib in build/libbert.so build/tq8/libbert.so; do
    BERT_LIB=$lib timeout -k 10 60 python -u scripts/gemm_shape.py 8 768 3072 $M 2 0 100 | sed "s|^|$lib |"
    BERT_LIB=$lib timeout -k 10 60 python -u scripts/gemm_shape.py 8 3072 768 $M 1 0 100 | sed "s|^|$lib |"
    BERT_LIB=$lib timeout -k 10 60 python -u scripts/gemm_shape.py 8 2304 768 $M 0 0 100 | sed "s|^|$lib |"
  done
done
TAG=tq8ab VAR=BERT_LIB VALS="build/libbert.so build/tq8/libbert.so" bash scripts/gpu_ab_env_probes.sh
