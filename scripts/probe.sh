cd $GRAFT_REPO_ROOT
for P in 0 1 2 3 4; do
  NNGP_SWEEP=launch NNGP_PROBE=$P timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/probe_$P.json 2> gpurun_out/probe_$P.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/probe_$P.json')); print('probe $P', round(d['value']), 'kernel_us', round(d['roofline']['kernel_avg_us'],2))"
done
