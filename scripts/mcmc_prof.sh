# kernel trace of 10 MCMC iterations (3 chains, 1e6/m15) + per-iteration breakdown
cd $GRAFT_REPO_ROOT
bash scripts/prof_mcmc.sh > /dev/null || exit 1
grep value gpurun_out/prof_mcmc.log | head -1 | cut -c1-300
f=$(find gpurun_out/prof_mcmc -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_iters.py $f 3 > gpurun_out/mcmc_iters.txt; cat gpurun_out/mcmc_iters.txt
