#!/bin/bash
# round 6: does the rebuild-calls measurement (a second 3-chain context) change the live kernel timing
# that follows it?  And the stream-after-scatter variant (i) against h.
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for rb in 0 1; do
    a="--no-rebuild-calls"; [ $rb = 1 ] && a=""
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --mcmc-iters 0 $a > gpurun_out/rb_${rb}_$r.json 2> gpurun_out/rb_${rb}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/rb_${rb}_$r.json').read().strip().splitlines()[-1])
print('rebuild_calls=$rb rep $r', round(d['value']), 'kernel_us', round(d['roofline']['kernel_avg_us'], 1))"
  done
done
bash scripts/ab_so.sh 2 h i
