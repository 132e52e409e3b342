cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for mode in launch persistent; do
  NNGP_SWEEP=$mode timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/dbg_$mode.json 2> gpurun_out/dbg_$mode.err
  echo "mode=$mode rc=$?"; grep graph gpurun_out/dbg_$mode.err; python -c "
import json; d=json.load(open('gpurun_out/dbg_$mode.json')); print(d['value'], d['roofline'])"
done
