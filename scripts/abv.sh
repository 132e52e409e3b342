#!/bin/bash
# A/B over env settings of the headline bench: VARIANTS="A=1 B=2;C=3" (';'
# separates variants, an empty variant = defaults).  BENCH_ARGS extra flags.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "${VS[@]}"; do
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 10 --no-cpu-baseline --mcmc-iters ${MCMC:-0} ${BENCH_ARGS} > gpurun_out/abv_$i.json 2> gpurun_out/abv_$i.err
  rc=$?
  [ $rc -eq 0 ] || { echo "variant '$v' rc=$rc"; tail -5 gpurun_out/abv_$i.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/abv_$i.json')); c=d['config']; s=c.get('single_chain') or {}
print('[$v]', 'C=%d'%c['chains_per_gpu'], round(d['value']), 'single', round(s.get('value',0)), 'kernel_us', round(d['roofline']['kernel_avg_us'],1), 'frac', round(d['roofline']['frac'],4))"
  i=$((i+1))
done
