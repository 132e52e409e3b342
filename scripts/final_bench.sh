# Round deliverable: default bench line + rocprofv3 kernel trace/stats of the
# same workload (shorter step count), both under gpurun_out/.
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit 1
cat gpurun_out/bench_final.json
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_final -o run -- python3 $ROOTDIR/bench.py --steps 60 --warmup 10 --no-cpu-baseline > $ROOTDIR/gpurun_out/bench_prof.json 2> $ROOTDIR/gpurun_out/bench_prof.err) || exit 1
f=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1); head -14 "$f" | cut -c1-200
cat gpurun_out/bench_prof.json
