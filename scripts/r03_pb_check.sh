# exchange wave with 6 granule polls in flight per lane: tile parity subset + two default benches
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "tile or headline" > gpurun_out/pb_tests.log 2>&1
rc=$?; tail -2 gpurun_out/pb_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --mcmc-iters 0 > gpurun_out/pb$r.json 2> gpurun_out/pb$r.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/pb$r.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['config']['single_chain']['value']), d['roofline']['kernel_avg_us'])"
done
