"""Sharded sweep on the GPU, through the C ABI,
for both shard engines (every test runs twice):
 - tiles: the tile shard -- the ranks' tiles run in ONE launch on device 0
   (each rank with its own context, buffers and granule buffer; a draw read
   by another rank's tile reaches it only through the remote put into that
   rank's buffer, exactly as across GPUs), then device copies of every
   rank's slots instead of the RCCL broadcasts.  NNGP_TILES fixes the tile
   count, so 1 rank and G ranks share one layout;
 - colors: the colour shard -- the exchange of each colour is a device copy
   of the other ranks' segments instead of the RCCL all-gather.
The per-rank kernels and plans are the ones the multi-process path uses; the
multi-process transport itself needs one GPU per rank (8-GPU node).

Bars: every rank's field == the 1-rank shard field, bitwise (the ranks apply
the same updates in the same order); the 1-rank shard vs the oracle's
masked-form sweep with the same Philox normals within the sweep tolerance of
test_gpu_parity.py (rtol 1e-8, atol 1e-9 after 2-3 sweeps).
"""
import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu

CP = [1.0, 0.08, 0.0]


@pytest.fixture(autouse=True, params=["tiles", "colors"])
def engine(request, monkeypatch):
    monkeypatch.setenv("NNGP_ENGINE", request.param)
    monkeypatch.setenv("NNGP_TILES", "120")  # divisible by every G below; <= the CUs of one device
    return request.param


def _shards(P, prob, G, C, fields, b0):
    locs, NN, col, lm, y = prob
    ctxs = [P.ShardContext(locs, NN, col, lm, y, n_ranks=G, rank=g, device=0, n_chains=C) for g in range(G)]
    for ctx in ctxs:
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", CP)
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0[k])
        ctx.select(0)
    return ctxs


def _fields(ctx, C):
    out = []
    for k in range(C):
        ctx.select(k)
        out.append(ctx.get_field())
    ctx.select(0)
    return out


@pytest.mark.parametrize("n,m,G,C", [(6000, 10, 2, 1), (6000, 10, 3, 3), (20000, 15, 8, 1), (3000, 5, 5, 2),
                                     (40, 3, 4, 1)])
def test_group_shard_equals_single_rank_bitwise(P, engine, n, m, G, C):
    prob = make_problem(P, n, m, seed=n + G)
    rng = np.random.default_rng(G)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0 = [0.1 * (k + 1) for k in range(C)]
    args = (b0, [0.2 - 0.1 * k for k in range(C)], [-0.3 + 0.05 * k for k in range(C)],
            [11 + k for k in range(C)], [5] * C)
    ref = _shards(P, prob, 1, C, fields, b0)[0]
    ref.sweep_chains(3, *args)
    want = _fields(ref, C)
    ctxs = _shards(P, prob, G, C, fields, b0)
    info = ctxs[0].info
    assert info["n_ranks"] == G and info["sweep_engine"] == (1 if engine == "tiles" else 0)
    if engine == "tiles":
        assert info["n_tiles"] == min(120, n) and ref.info["n_tiles"] == info["n_tiles"]
        assert G == 1 or n < 100 or info["shard_exchange_slots"] > 0
    assert sum(c.info["shard_owned"] for c in ctxs) == n
    P.sweep_chains_group(ctxs, 3, *args)
    for g, ctx in enumerate(ctxs):
        for k, f in enumerate(_fields(ctx, C)):
            np.testing.assert_array_equal(f, want[k], err_msg=f"rank {g} chain {k}")
    # a second call continues from the replicas (r = B w rebuilt per call)
    P.sweep_chains_group(ctxs, 2, *args[:4], [8] * C)
    ref.sweep_chains(2, *args[:4], [8] * C)
    want = _fields(ref, C)
    for ctx in ctxs:
        for k, f in enumerate(_fields(ctx, C)):
            np.testing.assert_array_equal(f, want[k])
    for c in ctxs + [ref]:
        c.close()


def test_single_rank_shard_matches_oracle(P, O):
    n, m = 2500, 10
    locs, NN, col, lm, y = make_problem(P, n, m, seed=9)
    field = np.random.default_rng(3).normal(size=n)
    seed, base = 987654321, 40
    with P.ShardContext(locs, NN, col, lm, y, n_ranks=1, rank=0, device=0) as ctx:
        ctx.factor(0, "exponential_isotropic", CP)
        ctx.set_field(field)
        ctx.set_mu(None, 0.1)
        ctx.sweep(3, 0.1, 0.0, 0.1, seed, base)
        got = ctx.get_field()
        # the other entry points keep working on a shard context
        Lo = O.vecchia_linv("exponential_isotropic", CP, locs, NN)
        assert abs(ctx.loglik(0, 0.1, 0.0) - O.loglik(Lo, got - 0.1, NN, 0.0)) < 1e-9 * abs(ctx.loglik(0, 0.1, 0.0))
    z = O.sweep_normals(seed, base, 3, n)
    ref = O.sweep("masked", field, Lo, NN, col, O.precision_diag(Lo, NN), np.ones(n, np.int32), y,
                  np.full(n, 0.1), lm, 0.1, 0.0, 0.1, z)
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9)


def test_shard_refreshes_ghost_values_on_accept(P, O):
    """nngp_accept_factor refreshes the ghost cells' B values too: after a
    new factor, the sharded sweep still equals the single rank bitwise."""
    n, m, G = 5000, 10, 3
    prob = make_problem(P, n, m, seed=4)
    field = np.random.default_rng(1).normal(size=n)
    out = []
    for g_count in (1, G):
        ctxs = _shards(P, prob, g_count, 1, [field], [0.0])
        for c in ctxs:
            c.factor(1, "exponential_isotropic", [1.0, 0.15, 0.0])
            c.accept_factor()
        P.sweep_chains_group(ctxs, 2, [0.0], [0.0], [0.0], [3], [0])
        out.append([c.get_field() for c in ctxs])
        for c in ctxs:
            c.close()
    for f in out[1]:
        np.testing.assert_array_equal(f, out[0][0])


def test_shard_sweep_needs_communicator(P):
    prob = make_problem(P, 500, 5, seed=2)
    with P.ShardContext(*prob, n_ranks=2, rank=0, device=0) as ctx:
        ctx.factor(0, "exponential_isotropic", CP)
        ctx.set_field(np.zeros(500))
        ctx.set_mu(None, 0.0)
        with pytest.raises(P.NNGPError, match="communicator"):
            ctx.sweep(1, 0.0, 0.0, 0.0, 1, 0)
        with pytest.raises(P.NNGPError, match="injected"):
            ctx.sweep(1, 0.0, 0.0, 0.0, 1, 0, z=np.zeros((1, 500)))


def test_rccl_single_rank_communicator(P):
    """RCCL loads and initialises on the box: a 1-rank communicator."""
    from nngp_amd.shard import shard_unique_id

    prob = make_problem(P, 800, 5, seed=3)
    field = np.random.default_rng(0).normal(size=800)
    res = []
    for use_comm in (False, True):
        with P.ShardContext(*prob, n_ranks=1, rank=0, device=0) as ctx:
            if use_comm:
                ctx.comm_init(shard_unique_id())
            ctx.factor(0, "exponential_isotropic", CP)
            ctx.set_field(field)
            ctx.set_mu(None, 0.0)
            ctx.sweep_chains(2, [0.0], [0.0], [0.0], [7], [0])
            res.append(ctx.get_field())
    np.testing.assert_array_equal(res[0], res[1])


def test_group_shard_with_duplicated_observations_and_mu_vector(P):
    """Locations with several observations (Heavy_metals-like, n_obs > n) and
    a per-observation mean: the per-slot residual sums and observation counts
    are replicated on every rank; still bitwise equal to one rank."""
    n, m, G = 4000, 10, 4
    locs, NN, col, lm, y = make_problem(P, n, m, seed=21, dup_frac=0.15)
    rng = np.random.default_rng(4)
    field = rng.normal(size=n)
    mu = 0.2 + 0.05 * rng.normal(size=len(y))
    out = []
    for g_count in (1, G):
        ctxs = [P.ShardContext(locs, NN, col, lm, y, n_ranks=g_count, rank=g, device=0) for g in range(g_count)]
        for c in ctxs:
            c.factor(0, "matern15_isotropic", [1.0, 0.07, 0.0])
            c.set_field(field)
            c.set_mu(mu, 0.2)
        P.sweep_chains_group(ctxs, 3, [0.2], [0.1], [-0.4], [9], [2])
        out.append([c.get_field() for c in ctxs])
        for c in ctxs:
            c.close()
    for f in out[1]:
        np.testing.assert_array_equal(f, out[0][0])
