"""BASELINE configs[4] on the one-GPU box: n = 1e7 locations, m = 20, Matern
3/2 (the `matern15_isotropic` extension), colour classes sharded
over 8 ranks (north_star).  All 8 ranks run in this process
(nngp_sweep_chains_group: the per-colour exchange is a device copy instead of
the RCCL all-gather; the kernels, plan and exchange layout are the RCCL
path's).  Bars: the 8-rank field == the 1-rank field bitwise after one call;
the 1-rank field vs the oracle's local-form sweep with the same Philox normals
on the device factor (1e-9, one sweep); the log-likelihood vs the oracle's on
that factor (1e-10); sampled factor rows vs the dense conditional (the
kriging form of vecchia_Linv) within DESIGN §4's conditioning bound.

Engines: the colour shard (NNGP_ENGINE=colors) in the first test; the tile
shard (the default multi-GPU engine) in the second, with 256 tiles of r in
global memory split 8 x 32 over the ranks (the node's own plan, 256 LDS tiles
per GPU, needs 2048 resident workgroups: one device holds 256) -- bitwise
equal to the single-GPU context with the same tiles."""
import time
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
PROGRESS = Path(__file__).resolve().parent.parent / "gpurun_out" / "test_progress.log"


def _progress(capfd, t0, msg):
    """A progress line past pytest's capture (and into gpurun_out/): this test
    runs for minutes, and a silent GPU run is taken for a hung one."""
    line = f"[configs4 {time.time() - t0:7.1f}s] {msg}"
    with capfd.disabled():
        print(line, flush=True)
    try:
        PROGRESS.parent.mkdir(exist_ok=True)
        with open(PROGRESS, "a") as f:
            f.write(line + "\n")
    except OSError:
        pass


def _dense_row(O, covfun, cp, locs, nn_row):
    """Row of GpGp::vecchia_Linv from the dense local covariance: for self s
    and neighbours N, Linv = [1, -C_NN^{-1} C_Ns] / sqrt(C_ss - C_sN C_NN^{-1} C_Ns)."""
    idx = nn_row[nn_row != O.NA] - 1
    Cm = O.covmat(covfun, cp, locs[idx])
    if len(idx) == 1:
        return np.array([1.0 / np.sqrt(Cm[0, 0])]), 1.0
    wts = np.linalg.solve(Cm[1:, 1:], Cm[1:, 0])
    cv = Cm[0, 0] - Cm[0, 1:] @ wts
    return np.concatenate([[1.0], -wts]) / np.sqrt(cv), np.linalg.cond(Cm)


@pytest.fixture(scope="module")
def c4(P):
    """configs[4]'s inputs (built once for the module: ~75 s of host graph
    preparation at n = 1e7)."""
    t0 = time.time()
    n, m = 10_000_000, 20
    rng = np.random.default_rng(2024)
    locs = rng.uniform(size=(n, 2))
    locs = locs[P.order_maxmin(locs) - 1]
    NN = P.find_ordered_nn(locs, m)
    col = P.naive_greedy_coloring(NN)
    lm = np.arange(1, n + 1, dtype=np.int32)
    y = 1.0 + rng.normal(size=n)
    field = 1.0 + rng.normal(size=n)
    return {"locs": locs, "NN": NN, "col": col, "lm": lm, "y": y, "field": field, "rng": rng,
            "prep_s": time.time() - t0}


def test_configs4_1e7_m20_matern15_eight_rank_shard(P, O, c4, capfd, monkeypatch):
    monkeypatch.setenv("NNGP_ENGINE", "colors")
    t0 = time.time()
    n, G = 10_000_000, 8
    locs, NN, col, lm, y, field, rng = (c4[k] for k in ("locs", "NN", "col", "lm", "y", "field", "rng"))
    _progress(capfd, t0, f"inputs ({col.max()} colours, host prep {c4['prep_s']:.0f} s)")
    covfun, cp = "matern15_isotropic", [1.0, 0.02, 0.0]
    b0, ls, lnv, seed, cb = 1.0, 0.1, np.log(0.25), 4242, 7

    ref = P.ShardContext(locs, NN, col, lm, y, n_ranks=1, rank=0, device=0)
    ref.factor(0, covfun, cp)
    ref.set_field(field)
    ref.set_mu(None, b0)
    ll = ref.loglik(0, b0, ls)
    Linv = ref.get_linv(0)
    ref.sweep_chains(1, [b0], [ls], [lnv], [seed], [cb])
    want = ref.get_field()
    ref.close()
    _progress(capfd, t0, "1-rank context: factor, log-likelihood, one sweep")

    llo = O.loglik(Linv, field - b0, NN, ls)
    assert abs(ll - llo) <= 1e-10 * abs(llo), (ll, llo)
    for i in np.concatenate([np.arange(5), rng.choice(n, 400, replace=False)]):
        row, kappa = _dense_row(O, covfun, cp, locs, NN[i])
        got = Linv[i, :len(row)]
        assert np.abs(got - row).max() <= max(1e-10, 1e-14 * kappa) * np.abs(row).max(), (i, kappa)
    z = O.sweep_normals(seed, cb, 1, n)
    exp = O.sweep("local", field, Linv, NN, col, O.precision_diag(Linv, NN), np.ones(n, np.int32), y,
                  np.full(n, b0), lm, b0, ls, lnv, z)
    np.testing.assert_allclose(want, exp, rtol=1e-9, atol=1e-9)
    del Linv, exp, z
    _progress(capfd, t0, "oracle: factor rows, log-likelihood, local-form sweep")

    ctxs = []
    for g in range(G):
        ctxs.append(P.ShardContext(locs, NN, col, lm, y, n_ranks=G, rank=g, device=0))
        _progress(capfd, t0, f"shard context {g + 1}/{G}")
    assert sum(c.info["shard_owned"] for c in ctxs) == n
    for c in ctxs:
        c.factor(0, covfun, cp)
        c.set_field(field)
        c.set_mu(None, b0)
    P.sweep_chains_group(ctxs, 1, [b0], [ls], [lnv], [seed], [cb])
    for g, c in enumerate(ctxs):
        np.testing.assert_array_equal(c.get_field(), want, err_msg=f"rank {g}")
        c.close()


def test_configs4_tile_shard_r_global_eight_ranks_bitwise(P, c4, capfd, monkeypatch):
    """The default multi-GPU engine (the tile shard) at
    configs[4]'s geometry: n = 1e7, m = 20, Matern 3/2, 256 tiles split over
    8 ranks x 32 (the 8-GPU node's tile count per GPU would be 256 x 8, which
    one device cannot hold resident; 32 per rank keeps all 8 ranks' tiles in
    one launch here).  Tiles of ~39k locations exceed a CU's LDS, so their r
    lives in global memory (NNGP_TILE_R=global, the RG tiles).  Every rank's
    field after two calls (2 + 1 sweeps) is bitwise equal to the single-GPU
    context with the same 256 RG tiles -- the rank split changes only where a
    granule is stored (peer buffers through the ranks' remote puts)."""
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.setenv("NNGP_TILE_R", "global")
    monkeypatch.setenv("NNGP_TILES", "256")
    monkeypatch.setenv("NNGP_SWEEP_WARM", "0")  # shard calls rebuild r = B w every call: so does the reference
    t0 = time.time()
    n, G = 10_000_000, 8
    locs, NN, col, lm, y, field = (c4[k] for k in ("locs", "NN", "col", "lm", "y", "field"))
    covfun, cp = "matern15_isotropic", [1.0, 0.02, 0.0]
    calls = [(1.0, 0.1, np.log(0.25), 4242, 7, 2), (0.9, 0.0, np.log(0.3), 4343, 9, 1)]
    want = []
    with P.ChainContext(locs, NN, col, lm, y, device=0) as ref:
        inf = ref.info
        assert inf["sweep_engine"] == 1 and inf["n_tiles"] == 256 and inf["tile_r_global"] == 1, inf
        ref.factor(0, covfun, cp)
        ref.set_field(field)
        ref.set_mu(None, 1.0)
        for b0, ls, lnv, seed, cb, ns in calls:
            ref.sweep_chains(ns, [b0], [ls], [lnv], [seed], [cb])
            want.append(ref.get_field())
    _progress(capfd, t0, "single-GPU context, 256 RG tiles: two calls")
    ctxs = []
    try:
        for g in range(G):
            ctxs.append(P.ShardContext(locs, NN, col, lm, y, n_ranks=G, rank=g, device=0))
            _progress(capfd, t0, f"tile shard context {g + 1}/{G}")
        inf = [c.info for c in ctxs]
        assert all(i["sweep_engine"] == 1 and i["n_tiles"] == 256 and i["n_ranks"] == G and i["tile_r_global"] == 1
                   for i in inf), inf[0]
        assert sum(i["shard_owned"] for i in inf) == n
        for c in ctxs:
            c.factor(0, covfun, cp)
            c.set_field(field)
            c.set_mu(None, 1.0)
        for (b0, ls, lnv, seed, cb, ns), w in zip(calls, want):
            P.sweep_chains_group(ctxs, ns, [b0], [ls], [lnv], [seed], [cb])
            for g, c in enumerate(ctxs):
                np.testing.assert_array_equal(c.get_field(), w, err_msg=f"rank {g}")
        _progress(capfd, t0, "8-rank tile shard == single GPU, bitwise, after each call")
    finally:
        for c in ctxs:
            c.close()
