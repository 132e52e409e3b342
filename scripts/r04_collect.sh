#!/bin/bash
# copy the round-4 final evidence from gpurun_out/ into profiles/ (run here after the final GPU calls)
cd "$(dirname "$0")/.."
set -e
cp gpurun_out/bench_driver_shape.json profiles/r04_bench_driver_shape.json
cp gpurun_out/bench_default.json profiles/r04_bench_default.json
cp gpurun_out/bench_prof_final.json profiles/r04_bench_under_rocprof_final.json
cp "$(find gpurun_out/prof_final -name '*kernel_stats.csv' | head -1)" profiles/r04_kernel_stats_final.csv
cp gpurun_out/pmc/summary.json profiles/r04_pmc_tiles_c3_final.json
[ -f gpurun_out/pytest_gpu_full.txt ] && tail -3 gpurun_out/pytest_gpu_full.txt > profiles/r04_pytest_gpu_full_final.txt
[ -f gpurun_out/smoke.log ] && cp gpurun_out/smoke.log profiles/r04_smoke.txt
ls -la profiles/r04_*
