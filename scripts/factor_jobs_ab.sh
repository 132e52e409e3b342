#!/bin/bash
# multi-chain factor launches: the factor tests, then the MCMC metric with
# NNGP_FACTOR_JOBS=1 / 0 (scripts/mcmc_ab.py) and a kernel trace of the jobs path
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
ROOTDIR=$(pwd)
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_mcmc.py tests/test_gpu_capi_sequence.py tests/test_gpu_parity.py -k "factor or step or capi or sequence" > gpurun_out/fj_tests.txt 2>&1; rc=$?; tail -14 gpurun_out/fj_tests.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u scripts/mcmc_ab.py NNGP_FACTOR_JOBS 1 0 3 > gpurun_out/fj_ab.txt 2>&1; rc=$?; tail -8 gpurun_out/fj_ab.txt; [ $rc = 0 ] || exit $rc
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $ROOTDIR/gpurun_out/prof_fj -o run -- python3 $ROOTDIR/scripts/mcmc_prof.py --no-cprofile > $ROOTDIR/gpurun_out/prof_fj.log 2>&1) || exit 1
python3 scripts/trace_iters.py $(find gpurun_out/prof_fj -name "*kernel_trace.csv" | head -1) 3 > gpurun_out/fj_iters.txt; head -20 gpurun_out/fj_iters.txt
