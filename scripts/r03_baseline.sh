cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --mcmc-iters 20 > gpurun_out/r03_base_bench.json 2> gpurun_out/r03_base_bench.err || exit 1
timeout -k 10 300 python scripts/timeline.py 1000000 15 3 10 > gpurun_out/r03_base_tl3.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/timeline.py 1000000 15 1 10 > gpurun_out/r03_base_tl1.txt 2>&1 || exit 1
