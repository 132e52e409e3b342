#!/bin/bash
# the driver's bench command, the default bench, rocprofv3 kernel stats of the bench and the PMC
# FETCH/WRITE passes of the sweep kernel (scripts/pmc.sh) and the request-size passes
# (scripts/pmc_sizes.sh) -> gpurun_out/
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_shape.json 2> gpurun_out/bench_driver_shape.err || { tail -20 gpurun_out/bench_driver_shape.err; exit 1; }
cut -c1-600 gpurun_out/bench_driver_shape.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cut -c1-300 gpurun_out/bench_default.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_final -o run -- python3 $ROOTDIR/bench.py --steps 60 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > $ROOTDIR/gpurun_out/bench_prof_final.json 2> $ROOTDIR/gpurun_out/bench_prof_final.err) || exit 1
f=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1); head -6 "$f" | cut -c1-200
bash scripts/pmc.sh && bash scripts/pmc_sizes.sh
