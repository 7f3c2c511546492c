#!/bin/bash
# Library A/B with the small-batch probes: alternating bench runs (C3 + the B = 1 and
# C2 probes, no PMC) of build/libbert.so ("new") and build/old/libbert.so.
set -o pipefail
OUT=gpurun_out/${TAG:-libabp}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in new old; do
    if [ $lib = new ]; then L=${NEW:-build}/libbert.so; else L=${OLD:-build/old}/libbert.so; fi
    BERT_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc --no-library --steps 30 > $OUT/${lib}_r$r.log 2>&1 || { tail -20 $OUT/${lib}_r$r.log; exit 1; }
    python3 -c "
import json;l=[x for x in open('$OUT/${lib}_r$r.log') if x.startswith('{')][-1];d=json.loads(l);k=d['kernels']
p=d.get('probes',{});c2=p.get('f16_mfma',{});b1=p.get('q4_0_hbm',{});c1=p.get('c1_f32',{})
print('$lib r$r',d['value'],' '.join(f'{n}={v[\"avg_us\"]:.1f}' for n,v in k.items()))
print('   C2',c2.get('sentences_per_s'),c2.get('kernel_avg_us'),' B1',b1.get('latency_us'),b1.get('kernel_avg_us'))
print('   C1',c1.get('latency_us'),c1.get('kernel_avg_us'))"
  done
done
