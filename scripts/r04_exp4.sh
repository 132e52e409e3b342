#!/bin/bash
# round 4 experiment 4: one-sync MH steps (tests, MCMC kernel trace, bench), interior-first wave-local tiles
# (parity, A/B at 3 and 4 chains, timeline)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_mcmc.py tests/test_gpu_capi_sequence.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "mh_step or pair or lockstep or interior_first_wave_local or r_in_global_wave_local or coinciding" \
  > gpurun_out/exp4_tests.log 2>&1 || { tail -40 gpurun_out/exp4_tests.log; exit 1; }
tail -2 gpurun_out/exp4_tests.log
timeout -k 10 300 python -u scripts/ab_env.py 3 200 2 'wl:' 'wlib:NNGP_TILE_SPLIT=1' 'xw:NNGP_TILE_WL=0' > gpurun_out/ab4_c3.txt 2>&1 || { tail -20 gpurun_out/ab4_c3.txt; exit 1; }
grep rep gpurun_out/ab4_c3.txt
timeout -k 10 200 python -u scripts/ab_env.py 4 100 1 'wl:' 'wlib:NNGP_TILE_SPLIT=1' 'xw:NNGP_TILE_WL=0' > gpurun_out/ab4_c4.txt 2>&1 || { tail -20 gpurun_out/ab4_c4.txt; exit 1; }
grep rep gpurun_out/ab4_c4.txt
NNGP_TILE_SPLIT=1 timeout -k 10 200 python -u scripts/timeline.py 1000000 15 3 10 > gpurun_out/r04_tl3_wlib.txt 2>&1 || { tail -20 gpurun_out/r04_tl3_wlib.txt; exit 1; }
head -14 gpurun_out/r04_tl3_wlib.txt
bash scripts/mcmc_prof.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_exp4.json 2> gpurun_out/bench_exp4.err || { tail -20 gpurun_out/bench_exp4.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_exp4.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['cold_calls'], d['config']['single_chain']['value'], d['roofline']['kernel_avg_us'], d['secondary'] and (d['secondary']['value'], d['secondary'].get('ms_per_iteration')))"
