#!/bin/bash
# colour engine on 21 lanes at 3 chains (columns longer than 256 entries, m = 20): parity, then configs[4]'s
# per-GPU share and configs[4] on one GPU -- colour engine (default now) against r-in-global tiles
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "21_lanes" > gpurun_out/c21_tests.log 2>&1 || { tail -30 gpurun_out/c21_tests.log; exit 1; }
tail -1 gpurun_out/c21_tests.log
NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 300 python -u scripts/ab_env.py 3 50 1 'auto:' 'rg:NNGP_TILE_R=global' > gpurun_out/ab_c21_share.txt 2>&1 || { tail -20 gpurun_out/ab_c21_share.txt; exit 1; }
grep rep gpurun_out/ab_c21_share.txt
NNGP_AB_N=10000000 NNGP_AB_M=20 timeout -k 10 700 python -u scripts/ab_env.py 3 20 1 'auto:' 'rg:NNGP_TILE_R=global' > gpurun_out/ab_c21_1e7.txt 2>&1 || { tail -20 gpurun_out/ab_c21_1e7.txt; exit 1; }
grep -E "rep|workload" gpurun_out/ab_c21_1e7.txt
