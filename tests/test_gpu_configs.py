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

Engine: the colour shard (NNGP_ENGINE=colors).  The tile shard of this size
has 2048 tiles (256 per GPU), which only an 8-GPU node holds resident; its
cross-rank logic is checked at the headline size (test_gpu_tile_shard.py)
and by bench.py's cross-GPU parity check on the node."""
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


def test_configs4_1e7_m20_matern15_eight_rank_shard(P, O, capfd, monkeypatch):
    monkeypatch.setenv("NNGP_ENGINE", "colors")
    t0 = time.time()
    n, m, G = 10_000_000, 20, 8
    rng = np.random.default_rng(2024)
    locs = rng.uniform(size=(n, 2))
    locs = locs[P.order_maxmin(locs) - 1]
    _progress(capfd, t0, "max-min order")
    NN = P.find_ordered_nn(locs, m)
    _progress(capfd, t0, "ordered NN")
    col = P.naive_greedy_coloring(NN)
    _progress(capfd, t0, f"colouring ({col.max()} colours)")
    lm = np.arange(1, n + 1, dtype=np.int32)
    y = 1.0 + rng.normal(size=n)
    field = 1.0 + rng.normal(size=n)
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
