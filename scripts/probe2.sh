cd $GRAFT_REPO_ROOT
for P in 0 4 5 7 8; do
  NNGP_PROBE=$P timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-single-chain --chains 1 > gpurun_out/p2_$P.json 2> gpurun_out/p2_$P.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/p2_$P.json')); print('probe $P', round(d['value']), 'us/sweep', round(1e6/d['value'],1), 'kernel_avg_us', round(d['roofline']['kernel_avg_us'],2))"
done
