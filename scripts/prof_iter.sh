cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_iter -o run -- python3 $ROOTDIR/scripts/iter_bench.py > $ROOTDIR/gpurun_out/prof_iter.log 2>&1) || exit 1
f=$(find gpurun_out/prof_iter -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-160
