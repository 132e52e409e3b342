#!/bin/bash
# round 4 experiment 3: wave-local batches by default at 3+ chains (42-slot cap) against the exchange wave alone,
# 2 chains both ways, configs[4]'s per-GPU share at 3 chains (r in global memory with and without wave-local
# batches), r-in-global wave-local parity, pair log-likelihood / heavy-metals tests, n = 1e7 on one GPU, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_env.py 3 200 2 'xw:NNGP_TILE_WL=0' 'wl:' > gpurun_out/ab3_c3.txt 2>&1 || { tail -20 gpurun_out/ab3_c3.txt; exit 1; }
grep rep gpurun_out/ab3_c3.txt
timeout -k 10 200 python -u scripts/ab_env.py 2 200 1 'xw:' 'wl:NNGP_TILE_WL=1' > gpurun_out/ab3_c2.txt 2>&1 || { tail -20 gpurun_out/ab3_c2.txt; exit 1; }
grep rep gpurun_out/ab3_c2.txt
NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 300 python -u scripts/ab_env.py 3 100 1 'auto:' 'rgwl:NNGP_TILE_R=global' > gpurun_out/ab3_c4share.txt 2>&1 || { tail -20 gpurun_out/ab3_c4share.txt; exit 1; }
grep rep gpurun_out/ab3_c4share.txt
NNGP_TILE_WL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "r_in_global_memory" > gpurun_out/rgwl_tests.log 2>&1 || { tail -30 gpurun_out/rgwl_tests.log; exit 1; }
tail -2 gpurun_out/rgwl_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_mcmc.py tests/test_heavy_metals.py -x -q -s --timeout 250 --timeout-method thread \
  -k "pair or heavy_metals_device" > gpurun_out/mcmc_tests.log 2>&1 || { tail -30 gpurun_out/mcmc_tests.log; exit 1; }
grep -E "heavy metals|passed|failed" gpurun_out/mcmc_tests.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --mcmc-iters 20 > gpurun_out/bench_exp3.json 2> gpurun_out/bench_exp3.err || { tail -20 gpurun_out/bench_exp3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_exp3.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['cold_calls'], d['config']['single_chain']['value'], d['roofline']['kernel_avg_us'], d['secondary'] and d['secondary']['value'])"
NNGP_AB_N=10000000 NNGP_AB_M=20 timeout -k 10 600 python -u scripts/ab_env.py 1 40 1 'col:NNGP_ENGINE=colors' 'rgwl:NNGP_TILE_R=global,NNGP_TILE_WL=1' 'rg:NNGP_TILE_R=global' > gpurun_out/ab3_1e7.txt 2>&1 || { tail -20 gpurun_out/ab3_1e7.txt; exit 1; }
grep -E "rep|workload" gpurun_out/ab3_1e7.txt
