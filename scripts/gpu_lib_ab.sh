#!/bin/bash
# Library A/B at C3: alternating bench runs of build/libbert.so and the builds
# named in LIBS (BERT_LIB=build/<name>/libbert.so), ROUNDS rounds.
set -o pipefail
OUT=gpurun_out/${TAG:-libab}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in base ${LIBS}; do
    if [ $lib = base ]; then L=build/libbert.so; else L=build/$lib/libbert.so; fi
    BERT_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --steps 30 > $OUT/${lib}_r$r.log 2>&1 || { tail -20 $OUT/${lib}_r$r.log; exit 1; }
    python3 -c "import json;l=[x for x in open('$OUT/${lib}_r$r.log') if x.startswith('{')][-1];d=json.loads(l);k=d['kernels'];print('$lib r$r',d['value'],' '.join(f'{n}={v[\"avg_us\"]:.1f}' for n,v in k.items()))"
  done
done
