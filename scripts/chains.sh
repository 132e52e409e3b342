cd $GRAFT_REPO_ROOT
for C in 2 3 4; do
  timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-single-chain --chains $C > gpurun_out/ch_$C.json 2> gpurun_out/ch_$C.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/ch_$C.json')); print('chains $C', round(d['value']), 'kernel_avg_us', round(d['roofline']['kernel_avg_us'],2), 'frac', round(d['roofline']['frac'],3))"
done
