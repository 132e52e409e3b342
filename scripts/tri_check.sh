# sync-free triangular solve (NNGP_TRI=dag): parity subset, then a kernel
# trace of the MCMC iterations (diagnostic)
cd $GRAFT_REPO_ROOT
export NNGP_TRI=dag
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_predict.py -x -q --timeout 120 --timeout-method thread -k "tri or ancillary or predict or initialize or mcmc" > gpurun_out/tri_tests.log 2>&1
rc=$?; tail -4 gpurun_out/tri_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_mcmc.sh > /dev/null || exit 1
grep value gpurun_out/prof_mcmc.log | head -1 | cut -c1-200
python3 scripts/trace_window.py gpurun_out/prof_mcmc/run_kernel_trace.csv 99 10
