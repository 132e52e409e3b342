#!/bin/bash
# copy the final evidence of a round from gpurun_out/ into profiles/<tag>_* (run here after
# scripts/gpu_suite.sh and scripts/final_bench.sh).  Usage: bash scripts/collect.sh r05
cd "$(dirname "$0")/.."
set -e
T=${1:?usage: collect.sh <round tag, e.g. r05>}
cp gpurun_out/bench_driver_shape.json profiles/${T}_bench_driver_shape.json
cp gpurun_out/bench_default.json profiles/${T}_bench_default.json
cp gpurun_out/bench_prof_final.json profiles/${T}_bench_under_rocprof_final.json
cp "$(find gpurun_out/prof_final -name '*kernel_stats.csv' | head -1)" profiles/${T}_kernel_stats_final.csv
cp gpurun_out/pmc/summary.json profiles/${T}_pmc_tiles_c3_final.json
[ -f gpurun_out/pmcs/summary.json ] && cp gpurun_out/pmcs/summary.json profiles/${T}_pmc_sizes_tiles_c3_final.json
[ -f gpurun_out/pytest_gpu_full.txt ] && tail -3 gpurun_out/pytest_gpu_full.txt > profiles/${T}_pytest_gpu_full_final.txt
[ -f gpurun_out/smoke.log ] && cp gpurun_out/smoke.log profiles/${T}_smoke.txt
ls -la profiles/${T}_*
