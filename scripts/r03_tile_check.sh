# tile-sweep parity subset, two default bench runs, the 3-chain timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tile_shard.py -x -q --timeout 200 --timeout-method thread -k "tile or headline or sweep or batched or chains" > gpurun_out/tile_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tile_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --mcmc-iters 0 > gpurun_out/tb$r.json 2> gpurun_out/tb$r.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/tb$r.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['config']['single_chain']['value']), d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
done
timeout -k 10 300 python scripts/timeline.py 1000000 15 3 10 > gpurun_out/tl3.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/tl3.txt | head -13
