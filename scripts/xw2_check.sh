# exchange-wave tiles, second form (NNGP_TILE_XW=2): parity subset, A/B bench, timeline;
# then the configs[4] tile-shard test (r in global memory, 8 ranks x 32 tiles)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "xw2 or residency" > gpurun_out/xw2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/xw2_tests.log; [ $rc -eq 0 ] || exit $rc
for x in 2 1 2 1; do
  NNGP_TILE_XW=$x timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > gpurun_out/xw_b$x.json 2> gpurun_out/xw_b$x.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/xw_b$x.json').read().strip().splitlines()[-1]); print('xw=$x', round(d['value']), round(d['config']['single_chain']['value']), d['roofline']['kernel_avg_us'])"
done
NNGP_TILE_XW=2 timeout -k 10 300 python scripts/timeline.py 1000000 15 3 10 > gpurun_out/xw2_tl3.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/xw2_tl3.txt | head -14
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 800 --timeout-method thread -k "tile_shard" > gpurun_out/c4_tile.log 2>&1
rc=$?; tail -3 gpurun_out/c4_tile.log; tail -4 gpurun_out/test_progress.log; exit $rc
