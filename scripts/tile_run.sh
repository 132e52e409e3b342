cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 5 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_mcmc.py -k "tiles" -m gpu -q -x > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || { grep -E "^E|Error" gpurun_out/pt.log | head; exit 1; }
for ex in 0 3; do NNGP_TILE_EXP=$ex timeout -k 10 400 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --mcmc-iters 0 > gpurun_out/bench_tiles.json 2> gpurun_out/bench_tiles.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_tiles.json')); print('exp=$ex tiles value', round(d['value']), 'single', round(d['config']['single_chain']['value']), 'kernel us', round(d['roofline']['kernel_avg_us']), 'entries', d['config']['n_entries'])"; done
