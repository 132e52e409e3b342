#!/bin/bash
# round 4 experiment 6: grouped refresh items (parity subset), async vs synced sweep calls (driver-shape bench
# line, no CPU baseline), MCMC kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mcmc.py tests/test_gpu_warm_calls.py -x -q \
  --timeout 300 --timeout-method thread -k "tiles-default or mcmc or warm or accept" > gpurun_out/exp6_tests.log 2>&1 || { tail -40 gpurun_out/exp6_tests.log; exit 1; }
tail -2 gpurun_out/exp6_tests.log
for v in 1 0 1 0; do
  NNGP_SWEEP_SYNC=$v timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --mcmc-iters 0 > gpurun_out/b6_$v.json 2> gpurun_out/b6_$v.err || { tail -20 gpurun_out/b6_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/b6_$v.json').read().strip().splitlines()[-1]); print('sync=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
bash scripts/mcmc_prof.sh || exit 1
