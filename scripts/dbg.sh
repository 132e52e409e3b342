# GPU tests + a short bench (single-chain and 3-chain lines)
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/dbg_bench.json 2> gpurun_out/dbg_bench.err || exit 1
grep graph gpurun_out/dbg_bench.err
python -c "
import json; d=json.load(open('gpurun_out/dbg_bench.json')); print(d['value'], d['config']['single_chain'], d['roofline'])"
