#!/bin/bash
# the driver's bench line at --warmup 5 against --warmup 20 (same 20 timed steps), interleaved: every call shape
# of the timed region is captured before t0, so the warmup count must not move the number
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 5 20 5 20; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup $w --no-cpu-baseline --mcmc-iters 0 > gpurun_out/wu_$w.json 2> gpurun_out/wu_$w.err || { tail -20 gpurun_out/wu_$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/wu_$w.json').read().strip().splitlines()[-1]); print('warmup=$w', round(d['value'],1), round(d['ms_per_step'],5), round(d['roofline']['kernel_avg_us'],1))"
done
