"""Two processes, one GPU: the tile shard's multi-process path without RCCL
(which refuses two ranks on one GPU).  Run under torch.distributed.run with
2 ranks; both ranks use device 0.  Each rank maps the other's granule
buffer, w replica and flag words through HIP IPC (handles all-gathered over
gloo), runs its half of the tiles, stores the draws the other rank's tiles
read into the other's buffer, and exchanges its slots of w by peer copies and
device flags.  Rank 0 also sweeps the same problem alone with the same tiles
and checks every chain bitwise.  Prints "ok ..." on rank 0."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np
import torch.distributed as dist

import _pkgload

TILES = int(os.environ.get("TILE_SHARD_TILES", "32"))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["NNGP_TILES"] = str(TILES)
    # the one-GPU reference rebuilds r = B w every call, as shard calls do
    # (a warm call would start from the carried-over r: last bits apart)
    os.environ["NNGP_SWEEP_WARM"] = "0"
    P = _pkgload.load()
    from conftest import make_problem
    from nngp_amd.shard import ShardContext, init_shard_comm

    dist.init_process_group("gloo")
    n, m, C = 20000, 10, 3
    locs, NN, col, lm, y = make_problem(P, n, m, seed=31)
    rng = np.random.default_rng(4)
    fields = [rng.normal(size=n) for _ in range(C)]
    calls = [([0.1, 0.2, 0.3], [0.0, 0.1, -0.1], [-0.5, -0.3, -0.4], [5, 6, 7], [0, 0, 0], 3),
             ([0.2, 0.1, 0.0], [0.1, 0.0, 0.2], [-0.4, -0.6, -0.5], [8, 9, 10], [3, 3, 3], 2)]

    def setup(ctx):
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", [1.0, 0.1 + 0.01 * k, 0.0])
            ctx.set_field(fields[k])
            ctx.set_mu(None, calls[0][0][k])

    def read(ctx):
        out = []
        for k in range(C):
            ctx.select(k)
            out.append(ctx.get_field())
        return out

    ctx = ShardContext(locs, NN, col, lm, y, n_ranks=world, rank=rank, device=0, n_chains=C)
    info = ctx.info
    assert info["sweep_engine"] == 1 and info["n_ranks"] == world and info["n_tiles"] == TILES, info
    init_shard_comm(ctx, dist, rccl=False)
    setup(ctx)
    # the calls back to back, nothing read in between: the second call's
    # prologue runs on replicas that only the halo-only exchange after the
    # first call updated (no full exchange until the read below syncs); then
    # one more call after that full exchange
    for b0, ls, lnv, seed, cb, ns in calls:
        ctx.sweep_chains(ns, b0, ls, lnv, seed, cb)
    stale = True
    try:  # the library refuses to read a stale replica (nngp_shard_sync is explicit)
        from nngp_amd._lib import NNGPError, lib

        st = lib.nngp_get_field(ctx._h, np.zeros(n))
        stale = st != 0
    except NNGPError:
        pass
    assert stale, "a stale replica was read without nngp_shard_sync"
    got = [read(ctx)]  # ShardContext readers sync first (collective)
    b0, ls, lnv, seed, cb, ns = calls[0]
    ctx.sweep_chains(ns, b0, ls, lnv, seed, [x + 5 for x in cb])
    got.append(read(ctx))
    # the R drop-in's order on the raw C ABI (rpkg/R/mcmc_nngp_update_Gaussian.R:
    # sweep_chains, nngp_shard_sync, sum_squared_residuals_chains; no hidden
    # sync in the readers): the SSR read after the explicit sync succeeds
    # and equals the one-context SSR; without it the reader refuses
    mask = (1 << C) - 1
    ctx.sweep_chains(ns, b0, ls, lnv, seed, [x + 9 for x in cb])
    ssr = np.zeros(C)
    assert lib.nngp_sum_squared_residuals_chains(ctx._h, mask, np.asarray(b0, np.float64), ssr) != 0
    assert lib.nngp_shard_sync(ctx._h) == 0
    assert lib.nngp_sum_squared_residuals_chains(ctx._h, mask, np.asarray(b0, np.float64), ssr) == 0
    got.append(read(ctx))
    dist.barrier()
    ctx.close()
    if rank == 0:
        ref = P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C)
        assert ref.info["n_tiles"] == TILES
        setup(ref)
        for b0, ls, lnv, seed, cb, ns in calls:
            ref.sweep_chains(ns, b0, ls, lnv, seed, cb)
        for k, f in enumerate(read(ref)):
            assert np.array_equal(f, got[0][k]), (k, np.abs(f - got[0][k]).max())
        b0, ls, lnv, seed, cb, ns = calls[0]
        ref.sweep_chains(ns, b0, ls, lnv, seed, [x + 5 for x in cb])
        for k, f in enumerate(read(ref)):
            assert np.array_equal(f, got[1][k]), (k, np.abs(f - got[1][k]).max())
        ref.sweep_chains(ns, b0, ls, lnv, seed, [x + 9 for x in cb])
        for k, f in enumerate(read(ref)):
            assert np.array_equal(f, got[2][k]), (k, np.abs(f - got[2][k]).max())
        ssr_ref = ref.sum_squared_residuals_chains(mask, b0)
        assert np.array_equal(ssr_ref, ssr), (ssr_ref, ssr)
        ref.close()
        print(f"ok tile shard over {world} processes on one GPU == one context, bitwise "
              f"(n={n}, {C} chains, {TILES} tiles, {info['shard_exchange_slots']} exchanged slots)", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
