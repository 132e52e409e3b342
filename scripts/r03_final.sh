# final round-3 tree: full GPU suite, smoke + default bench, rocprofv3 kernel trace of the bench
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_full.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu_full.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.txt
bash scripts/full_check.sh > /dev/null || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_final -o run -- python3 $ROOTDIR/bench.py --steps 60 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > $ROOTDIR/gpurun_out/bench_prof_final.json 2> $ROOTDIR/gpurun_out/bench_prof_final.err) || exit 1
f=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-200
