# Tile-kernel iteration check: parity subset, bench (3 chains + single chain), per-phase timelines; outputs in gpurun_out/
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k 'headline or masked_reference or batched_chains_bitwise or multipass or philox_stream or graph_replay or accept_factor or residency or r_in_global' \
  > gpurun_out/perf_test.log 2>&1 || { tail -30 gpurun_out/perf_test.log; exit 1; }
tail -1 gpurun_out/perf_test.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --mcmc-iters 0 --no-cpu-baseline > gpurun_out/perf_bench.json 2> gpurun_out/perf_bench.err || { tail -20 gpurun_out/perf_bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("gpurun_out/perf_bench.json").read().strip().splitlines()[-1])
print("bench", d["value"], d["roofline"]["frac"], d["roofline"]["kernel_avg_us"], d["config"].get("single_chain", {}).get("value"))
PY
timeout -k 10 200 python scripts/timeline.py 1000000 15 3 10 > gpurun_out/perf_tl3.txt 2>&1 || exit 1
timeout -k 10 200 python scripts/timeline.py 1000000 15 1 10 > gpurun_out/perf_tl1.txt 2>&1 || exit 1
grep -v "^0:" gpurun_out/perf_tl3.txt | head -12
