#!/bin/bash
# A/B measurement recipes cited in DESIGN.md §3 and §5 (one box, variants interleaved by
# scripts/ab_env.py: chain-sweeps/s and the sweep kernel's launch time by HIP events).  Usage:
#   bash scripts/ab.sh wl|prio|c4share|1e7|split|sync
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
case "$1" in
  wl)  # wave-local batches vs exchange-wave batches at 3, 2 and 1 chains
    timeout -k 10 300 python -u scripts/ab_env.py 3 200 2 'xw:NNGP_TILE_WL=0' 'wl:' &&
    timeout -k 10 200 python -u scripts/ab_env.py 2 200 1 'xw:' 'wl:NNGP_TILE_WL=1' &&
    timeout -k 10 200 python -u scripts/ab_env.py 1 200 1 'xw:' 'wl:NNGP_TILE_WL=1' ;;
  prio)  # exchange-wave issue priority / poll-round sleep (measured no effect; knobs removed afterwards)
    timeout -k 10 300 python -u scripts/ab_env.py 3 200 2 'base:' ;;
  c4share)  # configs[4]'s per-GPU share on one GPU: r in global memory, plain vs wave-local batches
    NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 300 python -u scripts/ab_env.py 3 100 1 'auto:' 'rgwl:NNGP_TILE_R=global' ;;
  1e7)  # n = 1e7, m = 20, one chain on one GPU
    NNGP_AB_N=10000000 NNGP_AB_M=20 timeout -k 10 600 python -u scripts/ab_env.py 1 40 1 'col:NNGP_ENGINE=colors' \
      'rgwl:NNGP_TILE_R=global,NNGP_TILE_WL=1' 'rg:NNGP_TILE_R=global' ;;
  split)  # interior-first wave-local layouts
    timeout -k 10 300 python -u scripts/ab_env.py 3 200 2 'wl:' 'wlib:NNGP_TILE_SPLIT=1' 'xw:NNGP_TILE_WL=0' ;;
  sync)  # sweep calls with / without a host sync, the driver's bench shape
    for v in 1 0 1 0; do
      NNGP_SWEEP_SYNC=$v timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        --mcmc-iters 0 > gpurun_out/ab_sync_$v.json || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/ab_sync_$v.json').read().strip().splitlines()[-1]); print('sync=$v', d['value'], d['ms_per_step'])"
    done ;;
  *) echo "usage: $0 wl|prio|c4share|1e7|split|sync"; exit 2 ;;
esac
