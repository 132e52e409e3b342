"""Colour-sharded sweep over RCCL with 2 ranks (diagnostic): every rank sweeps
its half of every colour and all-gathers the colour's {dw, w_new} through
RCCL; rank 0 checks the field against a 1-rank shard of the same inputs
(bitwise).  Launch: python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 --master-port P scripts/rccl_two_rank.py [device_per_rank]
(device_per_rank=0 puts both ranks on device 0, for a 1-GPU box)."""
import os
import sys

import numpy as np
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _pkgload  # noqa: E402

P = _pkgload.load()
from nngp_amd.shard import ShardContext, init_shard_comm  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = int(os.environ["LOCAL_RANK"]) if (len(sys.argv) < 2 or sys.argv[1] != "0") else 0
dist.init_process_group("gloo")
rng = np.random.default_rng(5)
n, m, C = 20000, 10, 2
locs = rng.uniform(size=(n, 2))
locs = locs[P.order_maxmin(locs) - 1]
NN = P.find_ordered_nn(locs, m)
col = P.naive_greedy_coloring(NN)
lm = np.arange(1, n + 1, dtype=np.int32)
y = rng.normal(size=n)
fields = [rng.normal(size=n) for _ in range(C)]
args = ([0.1, 0.2], [0.0, 0.1], [-0.2, 0.0], [3, 4], [0, 0])


def setup(ctx):
    for k in range(C):
        ctx.select(k)
        ctx.factor(0, "exponential_isotropic", [1.0, 0.05, 0.0])
        ctx.set_field(fields[k])
        ctx.set_mu(None, args[0][k])
    ctx.select(0)


ctx = ShardContext(locs, NN, col, lm, y, n_ranks=world, rank=rank, device=dev, n_chains=C)
init_shard_comm(ctx, dist)
setup(ctx)
ctx.sweep_chains(4, *args)
got = []
for k in range(C):
    ctx.select(k)
    got.append(ctx.get_field())
ctx.close()
dist.barrier()
if rank == 0:
    ref = ShardContext(locs, NN, col, lm, y, n_ranks=1, rank=0, device=dev, n_chains=C)
    setup(ref)
    ref.sweep_chains(4, *args)
    ok = True
    for k in range(C):
        ref.select(k)
        ok &= bool(np.array_equal(ref.get_field(), got[k]))
    ref.close()
    print(f"rccl {world}-rank shard == 1 rank bitwise: {ok}", flush=True)
    if not ok:
        sys.exit(1)
dist.barrier()
dist.destroy_process_group()
