#!/bin/bash
# Environment A/B at C3: alternating bench runs over ENVS (";"-separated
# assignments, "-" = none), ROUNDS rounds, per-kernel averages printed.
set -o pipefail
OUT=gpurun_out/${TAG:-envab}
mkdir -p $OUT
IFS=';' read -ra CFG <<< "${ENVS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for i in "${!CFG[@]}"; do
    e=${CFG[$i]}; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-probes --no-library --steps 30 > $OUT/c${i}_r$r.log 2>&1 || { tail -20 $OUT/c${i}_r$r.log; exit 1; }
    python3 -c "import json;l=[x for x in open('$OUT/c${i}_r$r.log') if x.startswith('{')][-1];d=json.loads(l);k=d['kernels'];print('[${CFG[$i]}] r$r',d['value'],' '.join(f'{n}={v[\"avg_us\"]:.1f}' for n,v in k.items()))"
  done
done
