#!/bin/bash
# configs[4] (n = 1e7, m = 20, 3 chains) on ONE GPU: the bench line under a rocprofv3 kernel-trace/stats run
# (colour engine on 21-lane chunks since the end of round 4; before that r in global memory: 240 MB of r
# cannot live in 40 MB of LDS)
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_c4 -o run -- python3 $ROOTDIR/bench.py --gpus 1 --workload configs4 --steps 20 --warmup 5 --no-cpu-baseline --no-single-chain --mcmc-iters 0 > $ROOTDIR/gpurun_out/bench_c4_one_gpu.json 2> $ROOTDIR/gpurun_out/bench_c4_one_gpu.err) || { tail -20 gpurun_out/bench_c4_one_gpu.err; exit 1; }
tail -1 gpurun_out/bench_c4_one_gpu.json | cut -c1-700
f=$(find gpurun_out/prof_c4 -name "*kernel_stats.csv" | head -1); head -5 "$f" | cut -c1-200
