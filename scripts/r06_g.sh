#!/bin/bash
# round 6: ghost adds as the hand-off's dw arrive (g) against e and the round-5 build (a)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_warm_calls.py tests/test_gpu_tile_shard.py tests/test_gpu_robustness.py > gpurun_out/r06_g_tests.txt 2>&1 || { tail -30 gpurun_out/r06_g_tests.txt; exit 1; }
tail -2 gpurun_out/r06_g_tests.txt
bash scripts/ab_so.sh 3 e g || exit 1
NNGP_TIMELINE_KEEP=gpurun_out/r06_g_timeline.bin timeout -k 10 300 python -u scripts/timeline.py > gpurun_out/r06_g_timeline.txt 2>&1 || exit 1
tail -48 gpurun_out/r06_g_timeline.txt
