# one chain: 1024-thread tiles (no exchange wave) vs the default 512-thread exchange-wave tiles
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for nt in 1024 512; do
  NNGP_TILE_NT=$nt timeout -k 10 300 python bench.py --chains 1 --no-single-chain --steps 200 --warmup 20 --no-cpu-baseline --mcmc-iters 0 > gpurun_out/nt$nt.json 2> gpurun_out/nt$nt.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/nt$nt.json').read().strip().splitlines()[-1]); print('nt=$nt', round(d['value']), d['roofline']['kernel_avg_us'])"
done
