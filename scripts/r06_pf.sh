#!/bin/bash
# round 6: records/rescue GPU tests, then the L2-prefetch A/B of the tile sweep (NNGP_TILE_PF) and its timeline
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_robustness.py \
  tests/test_gpu_mcmc.py tests/test_gpu_warm_calls.py -k "records or rescue or tri_solve or timeout or beta0 or invalidated" > gpurun_out/r06_pf_tests.txt 2>&1 || { tail -30 gpurun_out/r06_pf_tests.txt; exit 1; }
tail -3 gpurun_out/r06_pf_tests.txt; grep "oversub" gpurun_out/r06_pf_tests.txt | head
timeout -k 10 400 python -u scripts/ab_env.py 3 200 3 'base:' 'pf:NNGP_TILE_PF=1' > gpurun_out/r06_pf_ab.txt 2>&1 || { tail -20 gpurun_out/r06_pf_ab.txt; exit 1; }
cat gpurun_out/r06_pf_ab.txt
NNGP_TILE_PF=1 timeout -k 10 300 python -u scripts/timeline.py > gpurun_out/r06_pf_timeline.txt 2>&1 || exit 1
tail -22 gpurun_out/r06_pf_timeline.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "lane_groups or factor_matches" > gpurun_out/r06_factor_lanes_tests.txt 2>&1 || { tail -30 gpurun_out/r06_factor_lanes_tests.txt; exit 1; }
tail -2 gpurun_out/r06_factor_lanes_tests.txt
ROOTDIR=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_factor -o run -- python3 $ROOTDIR/scripts/factor_lanes_ab.py > $ROOTDIR/gpurun_out/r06_factor_lanes_ab.txt 2>&1) || { tail -20 gpurun_out/r06_factor_lanes_ab.txt; exit 1; }
cat gpurun_out/r06_factor_lanes_ab.txt | tail -9
f=$(find gpurun_out/prof_factor -name "*kernel_stats.csv" | head -1); grep -i "factor" "$f" | cut -c1-220
