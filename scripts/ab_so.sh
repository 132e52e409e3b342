#!/bin/bash
# A/B of library builds on one box (diagnostic): lib/libnngp_<v>.so copied over lib/libnngp.so in turn
# (the box's scratch copy), the default bench without CPU baseline / MCMC for each, variants interleaved.
# usage: ab_so.sh REPS v1 v2 ...   (extra bench args in AB_ARGS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
reps=$1; shift
cp lib/libnngp.so lib/libnngp_cur.so
for r in $(seq 1 $reps); do
  for v in "$@"; do
    cp lib/libnngp_$v.so lib/libnngp.so
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --mcmc-iters 0 --sustained-s 0 --no-rebuild-calls $AB_ARGS > gpurun_out/ab_so_${v}_$r.json 2> gpurun_out/ab_so_${v}_$r.err || { tail -5 gpurun_out/ab_so_${v}_$r.err; cp lib/libnngp_cur.so lib/libnngp.so; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_so_${v}_$r.json').read().strip().splitlines()[-1]); c=d['config']
print('rep $r $v', round(d['value']), 'single', round(c['single_chain']['value']) if c.get('single_chain') else None,
      'cold', round(c['cold_calls']['value']), 'kernel_us', round(d['roofline']['kernel_avg_us'], 1))"
  done
done
cp lib/libnngp_cur.so lib/libnngp.so
