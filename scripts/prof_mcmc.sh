# rocprofv3 kernel trace of the bench's MCMC iterations (3 chains, 1e6/m15;
# scripts/mcmc_prof.py: 2 warm-up + 10 timed iterations under cProfile)
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_mcmc -o run -- python3 $ROOTDIR/scripts/mcmc_prof.py > $ROOTDIR/gpurun_out/prof_mcmc.log 2>&1) || exit 1
f=$(find gpurun_out/prof_mcmc -name "*kernel_stats.csv" | head -1); head -20 "$f" | cut -c1-200
