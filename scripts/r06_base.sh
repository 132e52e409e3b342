cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06_base_bench.json 2> gpurun_out/r06_base_bench.err || exit 1
cut -c1-400 gpurun_out/r06_base_bench.json
timeout -k 10 300 python -u scripts/timeline.py > gpurun_out/r06_base_timeline.txt 2>&1 || exit 1
tail -30 gpurun_out/r06_base_timeline.txt
