#!/bin/bash
# Two tile-shard ranks on ONE GPU (two processes, HIP IPC) at configs[4]'s
# per-rank tile shape: n = 2 x 625,000, m = 20, 3 chains, 256 tiles (128 per
# rank, ~4.9k locations per tile as at n = 1e7 over 8 GPUs).  NNGP_SPLIT_CHAINS=1
# (default): the chains as a 2-chain and a 1-chain shard with r in LDS;
# =0: one 3-chain shard with r in global memory.  Bench JSON lines in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sp in 1 0; do
  NNGP_SPLIT_CHAINS=$sp NNGP_BENCH_DEVICE=0 NNGP_TILES=256 timeout -k 10 450 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951$sp \
    bench.py --gpus 2 --n-locs 625000 --neighbours 20 --steps 20 --warmup 5 --mcmc-iters 0 --no-cpu-baseline \
    > gpurun_out/shard2_split$sp.json 2> gpurun_out/shard2_split$sp.err || { tail -20 gpurun_out/shard2_split$sp.err; exit 1; }
  python3 - "$sp" <<'PY'
import json, sys
sp = sys.argv[1]
d = json.loads(open(f"gpurun_out/shard2_split{sp}.json").read().strip().splitlines()[-1])
c = d["config"]
print("split" if sp == "1" else "joint", d["value"], c.get("chain_sweeps_per_s"), c.get("chain_groups"),
      c["parity_check"], c.get("engine_note_rank0"))
PY
done
