# GPU: parity tests, then bench (1 and 3 chains) with/without L2 prefetch, then in-kernel stamps
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for PF in ${PFS:-1 0}; do
  NNGP_PREFETCH=$PF timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/dbg_bench_$PF.json 2> gpurun_out/dbg_bench_$PF.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/dbg_bench_$PF.json')); print('prefetch $PF: C=3', round(d['value']), 'single', round(d['config']['single_chain']['value']), 'kernel_avg_us', round(d['roofline']['kernel_avg_us'],2))"
done
[ -n "$STAMPS" ] && bash scripts/stamps.sh
true
