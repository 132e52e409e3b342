cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./scripts/micro/dpfma || exit 1
export NNGP_TRI=dag
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "refresh or accept or tile or precision" > gpurun_out/r3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_mcmc.sh > /dev/null || exit 1
grep value gpurun_out/prof_mcmc.log | head -1 | cut -c100-250
python3 scripts/trace_window.py gpurun_out/prof_mcmc/run_kernel_trace.csv 99 10 | head -8
