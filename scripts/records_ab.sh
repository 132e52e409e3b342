#!/bin/bash
# streamed field records: their GPU tests, the C client, then the MCMC metric with and
# without streaming (scripts/mcmc_ab.py) -> gpurun_out/rs_*.txt
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mcmc.py tests/test_gpu_capi_sequence.py -k "records or capi or sequence" > gpurun_out/rs_tests.txt 2>&1; rc=$?; tail -12 gpurun_out/rs_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u scripts/mcmc_ab.py NNGP_RECORDS_STREAM 1 0 3 > gpurun_out/rs_ab.txt 2>&1; rc=$?; tail -9 gpurun_out/rs_ab.txt; exit $rc
