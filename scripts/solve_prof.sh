# Kernel trace of the batched ancillary proposal (scripts/solve_prof.py).
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd)
export TMPDIR=/tmp
rm -rf gpurun_out/solve_prof
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/gpurun_out/solve_prof" -o run -- \
    python3 "$ROOTDIR/scripts/solve_prof.py" > "$ROOTDIR/gpurun_out/solve_prof.log" 2>&1) || exit 1
f=$(find gpurun_out/solve_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/solve_stats.csv
t=$(find gpurun_out/solve_prof -name "*kernel_trace.csv" | head -1)
python3 scripts/solve_gaps.py "$t" > gpurun_out/solve_gaps.txt
