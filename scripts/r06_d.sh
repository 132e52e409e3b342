#!/bin/bash
# round 6: the fused beta_0 shift + rsqrt prep + log_unit + fma sums (d) against the round-5 build (a):
# warm-call tests, parity subset, A/B, per-colour timeline of d
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_warm_calls.py tests/test_gpu_parity.py -k "warm or beta0 or invalidated or normals or headline or tile_engine" > gpurun_out/r06_d_tests.txt 2>&1 || { tail -30 gpurun_out/r06_d_tests.txt; exit 1; }
tail -2 gpurun_out/r06_d_tests.txt
bash scripts/ab_so.sh 3 a d || exit 1
NNGP_TIMELINE_KEEP=gpurun_out/r06_d_timeline.bin timeout -k 10 300 python -u scripts/timeline.py > gpurun_out/r06_d_timeline.txt 2>&1 || exit 1
tail -45 gpurun_out/r06_d_timeline.txt
