#!/bin/bash
# round 4 experiment 5: driver-shape bench, MCMC kernel trace, A/B of async sweep calls
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_exp5.json 2> gpurun_out/bench_exp5.err || { tail -20 gpurun_out/bench_exp5.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_exp5.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['cold_calls'], d['config']['single_chain']['value'], d['roofline'], d['secondary'] and (d['secondary']['value'], d['secondary'].get('ms_per_iteration')), d['cpu_baseline']['value'])"
bash scripts/mcmc_prof.sh || exit 1
