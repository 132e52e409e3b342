# Round-end check on one box: the full GPU suite, smoke + default bench, a
# rocprofv3 kernel-trace/stats run of the bench command; outputs in gpurun_out/
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 660 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.txt 2>&1 || { tail -20 gpurun_out/pytest_gpu_full.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.txt
bash scripts/full_check.sh || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_tiles -o run -- python3 $ROOTDIR/bench.py --steps 60 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > $ROOTDIR/gpurun_out/bench_prof.json 2> $ROOTDIR/gpurun_out/bench_prof.err) || exit 1
f=$(find gpurun_out/prof_tiles -name "*kernel_stats.csv" | head -1); head -8 "$f" | cut -c1-220
