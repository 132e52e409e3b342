# Round deliverables: PMC passes of the tile sweep kernel (HBM traffic), then a
# rocprofv3 kernel-trace/stats run of the bench command; outputs in gpurun_out/.
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc.sh || exit 1
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_tiles -o run -- python3 $ROOTDIR/bench.py --steps 60 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > $ROOTDIR/gpurun_out/bench_prof.json 2> $ROOTDIR/gpurun_out/bench_prof.err) || exit 1
f=$(find gpurun_out/prof_tiles -name "*kernel_stats.csv" | head -1); head -8 "$f" | cut -c1-220
cat gpurun_out/bench_prof.json | cut -c1-400
