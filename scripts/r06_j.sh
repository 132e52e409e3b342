#!/bin/bash
# round 6: hand-off granules padded to 4 per slot at 3 chains (j) against h: tests, A/B, PMC request sizes
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tile_shard.py tests/test_gpu_warm_calls.py -k "tile or warm or headline or shard" > gpurun_out/r06_j_tests.txt 2>&1 || { tail -30 gpurun_out/r06_j_tests.txt; exit 1; }
tail -2 gpurun_out/r06_j_tests.txt
AB_ARGS="--no-single-chain" bash scripts/ab_so.sh 3 h j || exit 1
cp lib/libnngp_j.so lib/libnngp.so
bash scripts/pmc_sizes.sh > gpurun_out/r06_j_pmc.txt 2>&1 || { tail -5 gpurun_out/r06_j_pmc.txt; exit 1; }
tail -4 gpurun_out/r06_j_pmc.txt
