#!/bin/bash
# round 4 experiment 1: wave-local batches (NNGP_TILE_WL=1) and the exchange-wave L2 prefetch
# (NNGP_TILE_PF) against the default at the headline; parity subsets; warm-call pins; configs[4] share
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u scripts/ab_env.py 3 200 2 'base:NNGP_TILE_PF=0' 'wl:NNGP_TILE_WL=1' 'pf3:NNGP_TILE_PF=3' 'pf7:NNGP_TILE_PF=7' > gpurun_out/ab_c3.txt 2>&1 || { tail -20 gpurun_out/ab_c3.txt; exit 1; }
grep rep gpurun_out/ab_c3.txt
timeout -k 10 240 python -u scripts/ab_env.py 1 200 1 'base:NNGP_TILE_PF=0' 'wl:NNGP_TILE_WL=1' 'pf7:NNGP_TILE_PF=7' > gpurun_out/ab_c1.txt 2>&1 || { tail -20 gpurun_out/ab_c1.txt; exit 1; }
grep rep gpurun_out/ab_c1.txt
NNGP_TILE_WL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "headline or sweep_matches_masked or batched_chains_bitwise or single_chain_sweep_inside or philox or graph_replay" > gpurun_out/wl_tests.log 2>&1 || { tail -30 gpurun_out/wl_tests.log; exit 1; }
tail -2 gpurun_out/wl_tests.log
NNGP_TILE_WL=1 timeout -k 10 200 python -u scripts/timeline.py 1000000 15 3 10 > gpurun_out/r04_tl3_wl.txt 2>&1 || { tail -20 gpurun_out/r04_tl3_wl.txt; exit 1; }
head -12 gpurun_out/r04_tl3_wl.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_warm_calls.py -v --timeout 300 --timeout-method thread > gpurun_out/warm_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/warm_tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 300 python -u scripts/ab_env.py 3 100 1 'col:NNGP_ENGINE=colors' 'rg:NNGP_TILE_R=global' > gpurun_out/ab_c4share_c3.txt 2>&1 || { tail -20 gpurun_out/ab_c4share_c3.txt; exit 1; }
grep rep gpurun_out/ab_c4share_c3.txt
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --mcmc-iters 20 > gpurun_out/bench_exp1.json 2> gpurun_out/bench_exp1.err || { tail -20 gpurun_out/bench_exp1.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_exp1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['cold_calls'], d['config']['single_chain']['value'], d['roofline']['kernel_avg_us'], d['secondary'] and d['secondary']['value'])"
