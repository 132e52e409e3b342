"""Tile shard at the headline size: the n = 1e6,
m = 15, Matern 3/2, 3-chain workload of bench.py with its 256 tiles split
over G = 2, 4, 8 ranks (every rank its own context, buffers and granule
buffer; the ranks' tiles in one launch on device 0, so a draw crosses ranks
only through the remote puts into the reader rank's buffer), against the
single-GPU context with the same 256 tiles: every rank's field bitwise equal
after each of two calls (the tile partition, batches and summation order are
the same; only the hand-off path differs)."""
import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def headline(P):
    return make_problem(P, 1_000_000, 15, seed=7)


def _setup(ctx, fields, cps):
    for k in range(len(fields)):
        ctx.select(k)
        ctx.factor(0, "matern15_isotropic", cps[k])
        ctx.set_field(fields[k])
        ctx.set_mu(None, 0.1 * k)
    ctx.select(0)


def _fields(ctx, C):
    out = []
    for k in range(C):
        ctx.select(k)
        out.append(ctx.get_field())
    ctx.select(0)
    return out


@pytest.mark.parametrize("G", [2, 4, 8])
def test_tile_shard_headline_equals_single_gpu_bitwise(P, headline, monkeypatch, G):
    monkeypatch.setenv("NNGP_TILES", "256")
    # the one-GPU side rebuilds r = B w every call, as shard calls do (a warm
    # call starts from the r the last call left: the same chain, last bits apart)
    monkeypatch.setenv("NNGP_SWEEP_WARM", "0")
    locs, NN, col, lm, y = headline
    n, C = len(locs), 3
    cps = [[1.0, 0.05, 0.0], [1.2, 0.04, 0.0], [0.8, 0.06, 0.0]]
    rng = np.random.default_rng(5)
    fields = [rng.normal(size=n) for _ in range(C)]
    calls = [([0.0, 0.1, 0.2], [0.0, 0.2, -0.1], [-0.5, -0.4, -0.6], [11, 12, 13], [0, 0, 0], 3),
             ([0.05, 0.1, 0.15], [0.1, 0.0, -0.2], [-0.3, -0.5, -0.4], [21, 22, 23], [3, 3, 3], 2)]
    want = []
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ref:
        assert ref.info["sweep_engine"] == 1 and ref.info["n_tiles"] == 256
        _setup(ref, fields, cps)
        for b0, ls, lnv, seed, cb, ns in calls:
            ref.sweep_chains(ns, b0, ls, lnv, seed, cb)
            want.append(_fields(ref, C))
    ctxs = [P.ShardContext(locs, NN, col, lm, y, n_ranks=G, rank=g, device=0, n_chains=C) for g in range(G)]
    try:
        inf = [c.info for c in ctxs]
        assert all(i["sweep_engine"] == 1 and i["n_tiles"] == 256 and i["n_ranks"] == G for i in inf)
        assert sum(i["shard_owned"] for i in inf) == n
        assert inf[0]["shard_exchange_slots"] > 0
        for c in ctxs:
            _setup(c, fields, cps)
        for (b0, ls, lnv, seed, cb, ns), w in zip(calls, want):
            P.sweep_chains_group(ctxs, ns, b0, ls, lnv, seed, cb)
            for g, c in enumerate(ctxs):
                for k, f in enumerate(_fields(c, C)):
                    np.testing.assert_array_equal(f, w[k], err_msg=f"G={G} rank {g} chain {k}")
    finally:
        for c in ctxs:
            c.close()


def test_tile_shard_two_processes_one_gpu_ipc():
    """The multi-process path of the tile shard (HIP IPC mappings across
    processes, remote granule stores into the other process's buffer, call ids
    in step, w by peer copies + device flags) with 2 ranks on the one GPU:
    tests/mp/tile_shard_ipc_check.py under torch.distributed.run, bitwise equal
    to one context with the same 32 tiles.  (RCCL itself refuses two ranks on
    one GPU; its broadcasts replace the copies on an 8-GPU node.)"""
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    port = 29900 + os.getpid() % 97
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(root / "tests/mp/tile_shard_ipc_check.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(root))
    assert out.returncode == 0 and "ok tile shard over 2 processes" in out.stdout, out.stdout[-2000:] + out.stderr[-4000:]
