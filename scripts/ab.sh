# A/B of an env switch on the bench (1 and 3 chains): variant 0 = unset, 1 = set to 1
cd $GRAFT_REPO_ROOT
for V in 0 1; do
  if [ $V = 1 ]; then export $AB=1; else unset $AB; fi
  timeout -k 10 400 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/ab_$V.json')); print('$AB=$V C=3', round(d['value']), 'single', round(d['config']['single_chain']['value']), 'kernel_avg_us', round(d['roofline']['kernel_avg_us'],2))"
done
