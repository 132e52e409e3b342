# tri-solve tests + a short default bench (diagnostic)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tri_solve or ancillary" > gpurun_out/tri2.log 2>&1
rc=$?; tail -2 gpurun_out/tri2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench_r3a.json 2> gpurun_out/bench_r3a.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_r3a.json").read().strip().splitlines()[-1])
print(d["value"], d.get("ms_per_step"))
print(json.dumps(d.get("secondary"))[:500])
PY
