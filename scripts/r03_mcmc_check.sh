# MCMC-path parity subset + the secondary metric + a kernel trace of its iterations
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mcmc.py tests/test_gpu_parity.py tests/test_heavy_metals.py -x -q --timeout 120 --timeout-method thread -k "loglik or ancillary or tri or mcmc or heavy or lockstep or beta0 or ratio" > gpurun_out/mcmc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mcmc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/mcmc_bench.json 2> gpurun_out/mcmc_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/mcmc_bench.json').read().strip().splitlines()[-1]); print(round(d['value']), d['secondary'])"
bash scripts/r03_mcmc_prof.sh
