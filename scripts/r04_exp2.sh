#!/bin/bash
# round 4 experiment 2: r-in-global tiles on wave-local batches (n = 1e7 on one GPU), their bitwise parity with
# LDS tiles, the pair log-likelihood and heavy-metals tolerance tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NNGP_TILE_WL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "r_in_global_memory" > gpurun_out/rgwl_tests.log 2>&1 || { tail -30 gpurun_out/rgwl_tests.log; exit 1; }
tail -2 gpurun_out/rgwl_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_mcmc.py tests/test_heavy_metals.py -x -q -s --timeout 250 --timeout-method thread \
  -k "pair or heavy_metals_device" > gpurun_out/mcmc_tests.log 2>&1 || { tail -30 gpurun_out/mcmc_tests.log; exit 1; }
grep -E "heavy metals|passed|failed" gpurun_out/mcmc_tests.log
NNGP_AB_N=10000000 NNGP_AB_M=20 timeout -k 10 700 python -u scripts/ab_env.py 1 40 1 'col:NNGP_ENGINE=colors' 'rgwl:NNGP_TILE_R=global,NNGP_TILE_WL=1' 'rg:NNGP_TILE_R=global' > gpurun_out/ab_1e7.txt 2>&1 || { tail -20 gpurun_out/ab_1e7.txt; exit 1; }
grep -E "rep|workload" gpurun_out/ab_1e7.txt
