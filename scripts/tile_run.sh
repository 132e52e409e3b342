cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 5 500 python -m pytest tests/test_gpu_parity.py -k "tiles and sweep" -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit 1
for NT in ${NTS:-512}; do for C in 1 3; do echo "NT=$NT C=$C"; NNGP_TILE_NT=$NT timeout -k 5 200 python scripts/tile_probe.py 1000000 15 $C 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1; done; done
for NT in ${NTS:-512}; do NNGP_TILE_NT=$NT timeout -k 10 400 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --mcmc-iters 0 --no-kernel-timing > gpurun_out/bench_tiles.json 2> gpurun_out/bench_tiles.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/bench_tiles.json')); print('NT=$NT tiles value', d['value'], 'single', d['config']['single_chain']['value'])"; done
