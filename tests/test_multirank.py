"""The bench's N>1 paths on CPU, world_size-2 gloo processes (127.0.0.1):
the contract's timed region reports the MAX elapsed over ranks on every
rank; --multi replicas gives every rank its own workload and chain seeds;
the sharded sweep's bootstrap (RCCL id, IPC handles of the tile shard's
granule buffers) is agreed over the group; and a sharded measurement that
fails on any rank prints a null value on rank 0 (no replicas substituted).
The sharded sweep itself -- tile shard: device-initiated granule stores into
the peers' buffers over xGMI; colour shard: one RCCL all-gather per colour --
needs GPUs (tests/test_gpu_tile_shard.py, tests/test_gpu_shard.py)."""
import os
import sys
import time
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, str(ROOT))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    delay = 0.05 * (rank + 1)

    def run(n, ctr):
        for _ in range(n):
            time.sleep(delay / 10)
        return ctr + n

    el, ctr = bench.timed_region(run, 10, 2, dist)
    q.put((rank, el, ctr))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_timed_region_reports_max_over_ranks():
    world, port = 2, 29000 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    els = {r: el for r, el, _ in out}
    assert abs(els[0] - els[1]) < 1e-12           # all_reduce(MAX): identical on every rank
    assert els[0] >= 0.1 * 0.9                      # the slower rank's 10 x 10 ms dominates
    assert all(ctr == 12 for _, _, ctr in out)      # warmup 2 + timed 10 steps


def _seed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, str(ROOT))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    wseed, seeds = bench.replica_seeds(dist.get_rank(), 3)
    mine = torch.tensor([wseed] + seeds, dtype=torch.int64)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    q.put((rank, [v.tolist() for v in allv]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_rank_workloads_differ():
    """--multi replicas: the ranks' workload seeds and chain seeds (bench.replica_seeds,
    what bench.main uses) gathered over the group are pairwise distinct."""
    world, port = 2, 31500 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_seed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert out[0] == out[1]
    flat = [x for v in out[0] for x in v]
    assert len(set(flat)) == len(flat)


def _shard_fail_worker(rank, world, port, q):
    import contextlib
    import io

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    import bench

    def fake_shard_main(P, args, world, rank, local_rank, dist, scaling):
        if rank == 1:
            raise RuntimeError("hipIpcOpenMemHandle: invalid argument")
        return {"metric": bench.METRIC, "value": 123.0}

    bench.shard_main = fake_shard_main
    sys.argv = ["bench.py", "--gpus", str(world)]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main()
    q.put((rank, buf.getvalue()))


@pytest.mark.timeout(180)
def test_failed_shard_prints_null_value():
    """bench.py at N = 2 (default --multi shard-weak): the sharded measurement
    fails on rank 1; rank 0 prints ONE line with a null value, the error, and
    no replicas measurement in its place."""
    import json

    world, port = 2, 32500 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=170) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert out[1].strip() == ""
    lines = out[0].strip().splitlines()
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["value"] is None and d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert "failed" in d["config"]["error"]


def _bcast_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, str(ROOT))
    import _pkgload

    P = _pkgload.load()
    import nngp_amd.shard as S

    # the RCCL id needs a GPU; the bootstrap logic is what runs here
    S.shard_unique_id = lambda: bytes(range(128)) if rank == 0 else bytes(128)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q.put((rank, S.broadcast_unique_id(dist)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_shard_unique_id_broadcast_two_ranks():
    """The colour-sharded path's communicator bootstrap: rank 0's RCCL id
    reaches every rank over a gloo group (bench.py --shard)."""
    world, port = 2, 29500 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bcast_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert out[0] == out[1] == bytes(range(128))


class _FakeTileShard:
    """Stands in for a tile-shard ShardContext (the IPC and RCCL calls need a
    GPU): records what init_shard_comm hands it."""

    def __init__(self, rank, fail_open=False):
        self.n_ranks, self.rank, self.tile_shard, self.fail_open = 2, rank, True, fail_open
        self.uid = self.opened = None

    def comm_init(self, uid):
        self.uid = uid

    def ipc_handle(self):
        return bytes([self.rank + 1]) * 192

    def ipc_open(self, handles):
        if self.fail_open:
            raise RuntimeError("hipIpcOpenMemHandle: invalid argument")
        self.opened = list(handles)


def _init_worker(rank, world, port, q, fail_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, str(ROOT))
    import _pkgload

    _pkgload.load()
    import nngp_amd.shard as S

    S.shard_unique_id = lambda: bytes(range(128))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = _FakeTileShard(rank, fail_open=(rank == fail_rank))
    try:
        S.init_shard_comm(ctx, dist)
        q.put((rank, "ok", ctx.uid, ctx.opened))
    except RuntimeError as e:
        q.put((rank, "raised", str(e), None))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_tile_shard_init_two_ranks(fail_rank):
    """Tile-shard bootstrap over gloo: the RCCL id from rank 0, then the IPC
    handles of the granule buffers in rank order on every rank; a failure on
    one rank (here rank 1's ipc_open) raises on EVERY rank, so no rank goes on
    to a sweep whose peers never come."""
    world, port = 2, 30500 + os.getpid() % 1000 + (fail_rank + 1) * 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_init_worker, args=(r, world, port, q, fail_rank)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: (st, a, b) for r, st, a, b in (q.get(timeout=100) for _ in range(world))}
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    if fail_rank < 0:
        for r in range(world):
            st, uid, opened = out[r]
            assert st == "ok" and uid == bytes(range(128))
            assert opened == [bytes([1]) * 192, bytes([2]) * 192]
    else:
        for r in range(world):
            st, msg, _ = out[r]
            assert st == "raised" and "rank 1" in msg and "hipIpcOpenMemHandle" in msg


def _groups_worker(rank, world, port, q, diverge):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, str(ROOT))
    import _pkgload

    _pkgload.load()
    import nngp_amd.shard as S

    dist.init_process_group("gloo", rank=rank, world_size=world)
    groups = [[0, 1], [2]] if (diverge and rank == 1) else [[0, 1, 2]]
    try:
        q.put((rank, "ok", S._same_everywhere(dist, groups, "the chain groups")))
    except RuntimeError as e:
        q.put((rank, "raised", str(e)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("diverge", [False, True])
def test_chain_groups_agreed_across_ranks(diverge):
    """bench.py's sharded path: the chain groups each rank chose
    (context.split_groups, a rank-local decision) are compared over the
    group; ranks that disagree all raise instead of waiting for shards that
    never pair up."""
    world, port = 2, 29700 + os.getpid() % 200 + (50 if diverge else 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_groups_worker, args=(r, world, port, q, diverge)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: rest for r, *rest in (q.get(timeout=100) for _ in range(world))}
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    if diverge:
        assert all(o[0] == "raised" and "disagree" in o[1] for o in out.values())
    else:
        assert all(o == ["ok", [[0, 1, 2]]] for o in out.values())
