# Exchange-wave tiles (NNGP_TILE_XW=1) vs default: remaining checks, benches; outputs in gpurun_out/
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tile_shard.py -m gpu \
  -k 'chain_split or shard' > gpurun_out/xw_test2.log 2>&1
tail -3 gpurun_out/xw_test2.log
for XW in 0 1; do
NNGP_TILE_XW=$XW timeout -k 10 300 python bench.py --steps 50 --warmup 10 --mcmc-iters 0 --no-cpu-baseline > gpurun_out/xw${XW}_bench.json 2> gpurun_out/xw${XW}_bench.err || { tail -20 gpurun_out/xw${XW}_bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("gpurun_out/xw${XW}_bench.json").read().strip().splitlines()[-1])
print("XW=$XW bench", d["value"], d["roofline"]["frac"], d["roofline"]["kernel_avg_us"], d["config"].get("single_chain", {}).get("value"))
PY
done
