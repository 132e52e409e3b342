# Tile-engine parity subset + a rocprofv3 kernel-trace/stats run of the bench; outputs in gpurun_out/
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tile_shard.py -k 'tile or headline' -m gpu > gpurun_out/tile_test.log 2>&1 || { tail -20 gpurun_out/tile_test.log; exit 1; }
tail -1 gpurun_out/tile_test.log
rm -rf gpurun_out/prof_tiles
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_tiles -o run -- python3 $ROOTDIR/bench.py --steps 60 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > $ROOTDIR/gpurun_out/bench_prof.json 2> $ROOTDIR/gpurun_out/bench_prof.err) || exit 1
f=$(find gpurun_out/prof_tiles -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-200
