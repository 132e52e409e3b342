#!/bin/bash
# round 4: exchange-wave L2 prefetch (NNGP_TILE_PF) -- parity subset with it on, interleaved A/B at the headline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_warm_calls.py -v --timeout 300 --timeout-method thread > gpurun_out/warm_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/warm_tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
NNGP_TILE_PF=7 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "headline or sweep_matches_masked or multipass or philox" > gpurun_out/pf_tests.log 2>&1 || { tail -30 gpurun_out/pf_tests.log; exit 1; }
tail -2 gpurun_out/pf_tests.log
timeout -k 10 500 python -u scripts/ab_env.py 3 200 2 'pf0:NNGP_TILE_PF=0' 'pf1:NNGP_TILE_PF=1' 'pf3:NNGP_TILE_PF=3' 'pf7:NNGP_TILE_PF=7' > gpurun_out/ab_pf_c3.txt 2>&1 || { tail -20 gpurun_out/ab_pf_c3.txt; exit 1; }
grep rep gpurun_out/ab_pf_c3.txt
timeout -k 10 300 python -u scripts/ab_env.py 1 200 1 'pf0:NNGP_TILE_PF=0' 'pf7:NNGP_TILE_PF=7' > gpurun_out/ab_pf_c1.txt 2>&1 || { tail -20 gpurun_out/ab_pf_c1.txt; exit 1; }
grep rep gpurun_out/ab_pf_c1.txt
NNGP_TILE_PF=7 timeout -k 10 300 python -u scripts/timeline.py 1000000 15 3 10 > gpurun_out/r04_tl3_pf7.txt 2>&1 || { tail -20 gpurun_out/r04_tl3_pf7.txt; exit 1; }
head -12 gpurun_out/r04_tl3_pf7.txt
# configs[4] per-GPU share (n = 1.25e6, m = 20: one rank of eight): colour engine vs RG tiles at 3 chains, LDS tiles at 2
NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 400 python -u scripts/ab_env.py 3 100 1 'col:NNGP_ENGINE=colors' 'rg:NNGP_TILE_R=global' > gpurun_out/ab_c4share_c3.txt 2>&1 || { tail -20 gpurun_out/ab_c4share_c3.txt; exit 1; }
grep rep gpurun_out/ab_c4share_c3.txt
NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 300 python -u scripts/ab_env.py 2 100 1 'lds:NNGP_TILE_XW=1' 'rg:NNGP_TILE_R=global' > gpurun_out/ab_c4share_c2.txt 2>&1 || { tail -20 gpurun_out/ab_c4share_c2.txt; exit 1; }
grep rep gpurun_out/ab_c4share_c2.txt
