#!/bin/bash
# round 4 experiment 7: batched residual sums / obs reductions (parity subset), bench line, MCMC kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mcmc.py tests/test_gpu_capi_sequence.py tests/test_gpu_warm_calls.py tests/test_heavy_metals.py -x -q \
  --timeout 300 --timeout-method thread -k "tiles-default or mcmc or warm or accept or lockstep or heavy or ssr or ratio or mu" > gpurun_out/exp7_tests.log 2>&1 || { tail -40 gpurun_out/exp7_tests.log; exit 1; }
tail -2 gpurun_out/exp7_tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_exp7.json 2> gpurun_out/bench_exp7.err || { tail -20 gpurun_out/bench_exp7.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_exp7.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['secondary'] and (d['secondary']['value'], d['secondary'].get('ms_per_iteration')))"
bash scripts/mcmc_prof.sh || exit 1
