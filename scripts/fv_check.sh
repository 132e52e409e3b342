cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_fv -o run -- python3 $ROOTDIR/scripts/factor_variants.py > $ROOTDIR/gpurun_out/fv.log 2>&1) || exit 1
grep "max rel" gpurun_out/fv.log
f=$(find gpurun_out/prof_fv -name "*kernel_stats.csv" | head -1); grep factor_kernel "$f" | cut -c1-200
export NNGP_TRI=dag
bash scripts/prof_mcmc.sh > /dev/null || exit 1
grep value gpurun_out/prof_mcmc.log | head -1 | cut -c100-250
python3 scripts/trace_window.py gpurun_out/prof_mcmc/run_kernel_trace.csv 99 10 | head -8
