"""HIP path vs the CPU oracle, through the C ABI (needs an MI355X).

Tolerances (fp64 everywhere; the oracle is a textbook-order restatement, the
device uses a different summation / factorisation order):
  * Vecchia factor Linv ........ rtol 1e-9, atol 1e-10 (error grows with the
                                  local condition number); 1e-8 general Matern
  * log-likelihood ............. rel 1e-10
  * chromatic sweep field ...... rtol 1e-9, atol 1e-10 after one sweep; 1e-8 after
                                  2-3 sweeps (each sweep is a linear map whose gain
                                  amplifies last-bit differences of the inputs)
  * neighbour indices, colours . bit-exact (integer)
"""
import numpy as np
import pytest

from conftest import make_problem

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("engine")]

COVS = {
    "exponential_isotropic": [1.0, 0.08, 0.0],
    "matern15_isotropic": [1.0, 0.05, 0.0],
    "matern_isotropic": [1.0, 0.06, 0.7, 0.0],
}


def _ctx(P, locs, NN, col, lm, y):
    return P.ChainContext(locs, NN, col, lm, y, device=0)


def test_device_normals_match_oracle(P, O):
    from nngp_amd.context import device_normals

    for seed, sweep in [(0, 0), (12345678901234, 7), (2 ** 64 - 1, 2 ** 40 + 3)]:
        z = device_normals(seed, sweep, 4096)
        zo = O.normals(seed, sweep, 4096)
        assert np.allclose(z, zo, rtol=1e-14, atol=1e-14)
        assert abs(z.mean()) < 0.1 and abs(z.std() - 1) < 0.05


@pytest.mark.parametrize("m", [1, 5, 10, 15, 20, 31])
@pytest.mark.parametrize("covfun", list(COVS))
def test_factor_matches_oracle(P, O, m, covfun):
    locs, NN, col, lm, y = make_problem(P, 700, m, seed=m)
    cp = COVS[covfun]
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        got = ctx.get_linv(0)
        ref = O.vecchia_linv(covfun, cp, locs, NN)
        # relative error amplified by the local condition number: rtol 1e-9
        # plus atol 1e-10 (|Linv| entries are O(1e-2..1e2) here)
        tol = 1e-8 if covfun == "matern_isotropic" else 1e-9
        np.testing.assert_allclose(got, ref, rtol=tol, atol=tol * 1e-1)
        # unfilled (NA) entries are exactly 0 like GpGp's zeros(n, m)
        assert np.all(got[NN == O.NA] == 0.0)
        np.testing.assert_allclose(ctx.precision_diag(), O.precision_diag(ref, NN), rtol=1e-10)


@pytest.mark.parametrize("covfun", ["exponential_isotropic", "matern15_isotropic"])
@pytest.mark.parametrize("m", [12, 15])
def test_factor_lane_pairs_match_oracle(P, O, covfun, m, monkeypatch):
    """The opt-in lane-pair factor kernel (NNGP_FACTOR_PAIR=1, two lanes per
    Vecchia row, kernels.hip factor_pair_kernel; BM = 16 blocks: m = 15, and
    m = 12 padded in front) against the oracle's GpGp::vecchia_Linv
    restatement, at the one-lane kernel's tolerance."""
    monkeypatch.setenv("NNGP_FACTOR_PAIR", "1")
    locs, NN, col, lm, y = make_problem(P, 900, m, seed=40 + m)
    cp = COVS[covfun]
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        got = ctx.get_linv(0)
    ref = O.vecchia_linv(covfun, cp, locs, NN)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)
    assert np.all(got[NN == O.NA] == 0.0)


@pytest.mark.parametrize("m", [1, 5, 10, 15])
@pytest.mark.parametrize("covfun", [c for c in COVS if c != "matern_isotropic"])
def test_factor_lane_groups_match_oracle(P, O, m, covfun, monkeypatch):
    """The opt-in 16-lane-group factor kernel (NNGP_FACTOR_LANES=16: one DPP
    row of 16 lanes per Vecchia row, lane q owning point q and column q of the
    local block, right-looking Cholesky by row broadcasts; kernels.hip
    factor_lanes_kernel; b <= 16, so m <= 15) against the oracle's
    GpGp::vecchia_Linv restatement at test_factor_matches_oracle's tolerance,
    every covariance family it serves (the general Matern keeps the
    run-time-b kernel); and the multi-chain launch (three jobs with different
    parameters in one launch) row for row against one job at a time."""
    monkeypatch.setenv("NNGP_FACTOR_LANES", "16")
    locs, NN, col, lm, y = make_problem(P, 700, m, seed=m)
    cp = COVS[covfun]
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        got = ctx.get_linv(0)
        ref = O.vecchia_linv(covfun, cp, locs, NN)
        np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)
        assert np.all(got[NN == O.NA] == 0.0)
        np.testing.assert_allclose(ctx.precision_diag(), O.precision_diag(ref, NN), rtol=1e-10)
    if covfun == "matern15_isotropic":
        cps = [[1.0 + 0.2 * k] + list(cp[1:]) for k in range(3)]
        cps[2][1] *= 1.3
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=3) as ctx:
            st = ctx.factor_chains(0, 7, covfun, cps)
            assert (st == 0).all()
            jobs = [ctx.select(k).get_linv(0) for k in range(3)]
            for k in range(3):
                ctx.select(k).factor(0, covfun, cps[k])
                np.testing.assert_array_equal(ctx.get_linv(0), jobs[k])


@pytest.mark.parametrize("covfun", ["exponential_isotropic", "matern15_isotropic"])
def test_factor_with_coinciding_points_matches_oracle(P, O, covfun):
    """Two locations at distance 0 (correlation 1) with a nugget: a positive
    definite local covariance that GpGp factors; the device's distance
    (sqrt_pos at s = 0) must be 0, not 0 x inf."""
    locs, NN, col, lm, y = make_problem(P, 3000, 10, seed=71)
    locs = locs.copy()
    for k0 in (100, 1500, 2999):
        locs[k0] = locs[NN[k0, 1] - 1]
    cp = [1.0, 0.08, 0.1]
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        got = ctx.get_linv(0)
    ref = O.vecchia_linv(covfun, cp, locs, NN)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("covfun,cp,d", [
    ("exponential_scaledim", [1.3, 0.1, 0.3, 0.0], 2),
    ("exponential_spacetime", [0.7, 0.1, 0.5, 0.0], 3),
    ("matern_scaledim", [1.0, 0.1, 0.2, 1.4, 0.0], 2),
    ("matern_spacetime", [1.0, 0.1, 0.3, 0.9, 0.0], 3),
    ("exponential_isotropic", [2.0, 0.2, 0.1], 3),  # nugget + variance
    ("matern_isotropic", [1.0, 0.1, 2.6, 0.0], 2),
])
def test_factor_other_covfuns(P, O, covfun, cp, d):
    locs, NN, col, lm, y = make_problem(P, 500, 10, d=d, seed=3)
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        _assert_rows_close(O, covfun, cp, locs, NN, ctx.get_linv(0), O.vecchia_linv(covfun, cp, locs, NN))


def _assert_rows_close(O, covfun, cp, locs, NN, got, ref, eps=1e-14):
    """Per-row tolerance eps * cond(local covariance) * max|row| (forward
    error bound of a backward-stable Cholesky + triangular solve)."""
    for i in range(NN.shape[0]):
        idx = NN[i][NN[i] != O.NA] - 1
        kappa = np.linalg.cond(O.covmat(covfun, cp, locs[idx])) if len(idx) > 1 else 1.0
        tol = max(1e-10, eps * kappa) * np.abs(ref[i]).max()
        assert np.abs(got[i] - ref[i]).max() <= tol, (i, kappa, np.abs(got[i] - ref[i]).max())


def test_factor_sphere(P, O):
    rng = np.random.default_rng(5)
    locs = np.column_stack([rng.uniform(-124, -67, 800), rng.uniform(25, 49, 800)])
    locs = locs[P.order_maxmin(locs) - 1]
    NN = P.find_ordered_nn(locs, 5)
    col = P.naive_greedy_coloring(NN)
    lm = np.arange(1, 801, dtype=np.int32)
    for covfun, cp in [("exponential_sphere", [1.0, 0.05, 0.0]), ("matern_sphere", [1.0, 0.05, 0.8, 0.0])]:
        with _ctx(P, locs, NN, col, lm, rng.normal(size=800)) as ctx:
            ctx.factor(0, covfun, cp)
            _assert_rows_close(O, covfun, cp, locs, NN, ctx.get_linv(0), O.vecchia_linv(covfun, cp, locs, NN))


def test_factor_not_pd_reports_row(P):
    locs, NN, col, lm, y = make_problem(P, 200, 5, seed=1)
    locs = locs.copy()
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        # absurdly long range -> numerically singular local covariances
        with pytest.raises(P.NNGPError) as e:
            ctx.factor(0, "matern15_isotropic", [1.0, 1e9, 0.0])
        assert e.value.status == 3 and "row" in str(e.value)


@pytest.mark.parametrize("covfun", ["exponential_isotropic", "matern15_isotropic"])
def test_loglik_matches_oracle(P, O, covfun):
    locs, NN, col, lm, y = make_problem(P, 1500, 10, seed=2)
    cp = COVS[covfun]
    field = np.random.default_rng(0).normal(size=1500) + 0.7
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        ctx.set_field(field)
        for ls in [-0.3, 0.0, 1.2]:
            got = ctx.loglik(0, 0.7, ls)
            ref = O.loglik(O.vecchia_linv(covfun, cp, locs, NN), field - 0.7, NN, ls)
            assert abs(got - ref) <= 1e-10 * abs(ref)


def _sweep_case(P, O, n, m, n_sweeps, dup, mu_vec, covfun="exponential_isotropic", seed=0, form="masked"):
    locs, NN, col, lm, y = make_problem(P, n, m, seed=seed, dup_frac=dup)
    cp = COVS[covfun]
    rng = np.random.default_rng(seed + 1)
    field = rng.normal(size=n)
    beta0, ls, lnv = 0.4, 0.3, -0.2
    mu = (beta0 + 0.1 * rng.normal(size=len(lm))) if mu_vec else np.full(len(lm), beta0)
    z = rng.normal(size=(n_sweeps, n))
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, covfun, cp)
        ctx.set_field(field)
        ctx.set_mu(mu if mu_vec else None, beta0)
        ctx.sweep(n_sweeps, beta0, ls, lnv, 1, 0, z=z)
        got = ctx.get_field()
        Lo = ctx.get_linv(0)  # the sweep is checked on the device's own factor
    np.testing.assert_allclose(Lo, O.vecchia_linv(covfun, cp, locs, NN), rtol=1e-6, atol=1e-8)
    D = O.precision_diag(Lo, NN)
    opl = np.bincount(lm - 1, minlength=n).astype(np.int32)
    ref = O.sweep(form, field, Lo, NN, col, D, opl, y, mu, lm, beta0, ls, lnv, z)
    return got, ref


@pytest.mark.parametrize("n,m,dup,mu_vec", [(2000, 5, 0.0, False), (3000, 10, 0.1, True),
                                            (1500, 15, 0.0, True), (900, 20, 0.05, False)])
def test_sweep_matches_masked_reference_form(P, O, n, m, dup, mu_vec):
    got, ref = _sweep_case(P, O, n, m, 3, dup, mu_vec)
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9)
    got1, ref1 = _sweep_case(P, O, n, m, 1, dup, mu_vec)
    np.testing.assert_allclose(got1, ref1, rtol=1e-9, atol=1e-10)


def test_sweep_matern15_local_form(P, O):
    got, ref = _sweep_case(P, O, 20000, 15, 2, 0.0, False, covfun="matern15_isotropic", form="local")
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9)


def test_sweep_philox_stream_matches_oracle(P, O):
    locs, NN, col, lm, y = make_problem(P, 2500, 10, seed=9)
    cp = COVS["exponential_isotropic"]
    field = np.random.default_rng(3).normal(size=2500)
    seed, base = 987654321, 40
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "exponential_isotropic", cp)
        ctx.set_field(field)
        ctx.set_mu(None, 0.1)
        ctx.sweep(3, 0.1, 0.0, 0.1, seed, base)  # graph-captured path
        got = ctx.get_field()
        ctx.set_field(field)
        ctx.sweep(3, 0.1, 0.0, 0.1, seed, base)  # replay of the cached graph
        np.testing.assert_array_equal(ctx.get_field(), got)  # deterministic replay
    Lo = O.vecchia_linv("exponential_isotropic", cp, locs, NN)
    z = O.sweep_normals(seed, base, 3, 2500)
    ref = O.sweep("masked", field, Lo, NN, col, O.precision_diag(Lo, NN), np.ones(2500, np.int32), y,
                  np.full(2500, 0.1), lm, 0.1, 0.0, 0.1, z)
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9)


def test_graph_replay_sees_new_scalars(P, O):
    """Scalars (beta0, scales, counter) live in device memory: a replayed graph
    must use the current values, not the captured ones."""
    locs, NN, col, lm, y = make_problem(P, 1200, 8, seed=4)
    cp = COVS["exponential_isotropic"]
    field = np.random.default_rng(8).normal(size=1200)
    Lo = O.vecchia_linv("exponential_isotropic", cp, locs, NN)
    D = O.precision_diag(Lo, NN)
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "exponential_isotropic", cp)
        for (b0, ls, lnv, base) in [(0.1, 0.0, 0.1, 0), (-0.5, 0.4, -0.3, 10)]:
            ctx.set_field(field)
            ctx.set_mu(None, b0)
            ctx.sweep(2, b0, ls, lnv, 5, base)
            z = O.sweep_normals(5, base, 2, 1200)
            ref = O.sweep("masked", field, Lo, NN, col, D, np.ones(1200, np.int32), y, np.full(1200, b0), lm,
                          b0, ls, lnv, z)
            np.testing.assert_allclose(ctx.get_field(), ref, rtol=1e-8, atol=1e-9)


def test_accept_factor_refreshes_sweep_values(P, O):
    locs, NN, col, lm, y = make_problem(P, 1500, 10, seed=6)
    c0, c1 = [1.0, 0.05, 0.0], [1.0, 0.12, 0.0]
    field = np.random.default_rng(2).normal(size=1500)
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "exponential_isotropic", c0)
        ctx.set_field(field)
        ctx.set_mu(None, 0.0)
        ctx.sweep(1, 0.0, 0.0, 0.0, 3, 0)  # captures a graph on factor 0
        ctx.set_field(field)
        ctx.factor(1, "exponential_isotropic", c1)
        ctx.accept_factor()
        ctx.sweep(1, 0.0, 0.0, 0.0, 3, 0)
        got = ctx.get_field()
        np.testing.assert_allclose(ctx.precision_diag(), O.precision_diag(O.vecchia_linv("exponential_isotropic", c1, locs, NN), NN), rtol=1e-10)
    L1 = O.vecchia_linv("exponential_isotropic", c1, locs, NN)
    z = O.sweep_normals(3, 0, 1, 1500)
    ref = O.sweep("masked", field, L1, NN, col, O.precision_diag(L1, NN), np.ones(1500, np.int32), y,
                  np.zeros(1500), lm, 0.0, 0.0, 0.0, z)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)


def test_mh_building_blocks(P, O):
    locs, NN, col, lm, y = make_problem(P, 1800, 10, seed=11, dup_frac=0.1)
    n = 1800
    rng = np.random.default_rng(4)
    field = rng.normal(size=n) + 1.0
    beta0, lnv = 1.0, -0.4
    mu = beta0 + 0.2 * rng.normal(size=len(lm))
    c0, c1 = [1.0, 0.05, 0.0], [1.0, 0.09, 0.0]
    L0 = O.vecchia_linv("exponential_isotropic", c0, locs, NN)
    L1 = O.vecchia_linv("exponential_isotropic", c1, locs, NN)
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "exponential_isotropic", c0)
        ctx.factor(1, "exponential_isotropic", c1)
        ctx.set_field(field)
        ctx.set_mu(mu, beta0)
        # ancillary proposal: beta0 + exp(dls/2) B1^{-1} B0 (field - beta0)  (update_Gaussian.R:127)
        ctx.ancillary_propose(beta0, 0.3)
        w = O.tri_solve(L1, NN, O.linv_mult(L0, field - beta0, NN))
        prop = beta0 + np.exp(0.15) * w
        ratio = ctx.field_response_ratio(beta0, lnv)
        sd = np.exp(0.5 * lnv)
        ll = lambda f: -0.5 * ((y - (f[lm - 1] + mu - beta0)) / sd) ** 2
        np.testing.assert_allclose(ratio, (ll(prop) - ll(field)).sum(), rtol=1e-8)
        ssr = ctx.sum_squared_residuals(beta0)
        np.testing.assert_allclose(ssr, ((y - field[lm - 1] - mu + beta0) ** 2).sum(), rtol=1e-11)
        oqo, oqf = ctx.beta0_stats()
        u1 = O.linv_mult(L0, np.ones(n), NN)
        uf = O.linv_mult(L0, field, NN)
        np.testing.assert_allclose([oqo, oqf], [u1 @ u1, u1 @ uf], rtol=1e-11)
        X = rng.normal(size=(n, 3))
        np.testing.assert_allclose(ctx.spmv(1, X), np.column_stack([O.linv_mult(L1, X[:, k], NN) for k in range(3)]),
                                   rtol=1e-12, atol=1e-12)
        u = rng.normal(size=n)
        np.testing.assert_allclose(ctx.tri_solve(0, u), O.tri_solve(L0, NN, u), rtol=1e-9, atol=1e-10)
        ctx.accept_field()
        np.testing.assert_allclose(ctx.get_field(), prop, rtol=1e-9, atol=1e-10)


def test_edge_cases(P, O):
    # n <= m+1 (every row short), single-location colours, m = 0 neighbourhood impossible (b>=1)
    for n, m in [(1, 3), (2, 3), (5, 10), (40, 1)]:
        locs, NN, col, lm, y = make_problem(P, n, m, seed=n)
        got, ref = None, None
        with _ctx(P, locs, NN, col, lm, y) as ctx:
            ctx.factor(0, "exponential_isotropic", [1.0, 0.3, 0.0])
            Lo = O.vecchia_linv("exponential_isotropic", [1.0, 0.3, 0.0], locs, NN)
            np.testing.assert_allclose(ctx.get_linv(0), Lo, rtol=1e-11, atol=1e-13)
            f = np.linspace(-1, 1, n)
            ctx.set_field(f)
            ctx.set_mu(None, 0.0)
            z = np.ones((1, n))
            ctx.sweep(1, 0.0, 0.0, 0.0, 0, 0, z=z)
            got = ctx.get_field()
        ref = O.sweep("masked", f, Lo, NN, col, O.precision_diag(Lo, NN), np.ones(n, np.int32), y,
                      np.zeros(n), lm, 0.0, 0.0, 0.0, z)
        np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)


def test_bad_inputs_fail_loudly(P):
    locs, NN, col, lm, y = make_problem(P, 300, 5, seed=2)
    bad = col.copy()
    bad[:] = 1  # not a proper colouring
    with pytest.raises(P.NNGPError):
        P.ChainContext(locs, NN, bad, lm, y, device=0)
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        with pytest.raises(P.NNGPError):
            ctx.sweep(1, 0.0, 0.0, 0.0, 0, 0)  # no factor yet
        with pytest.raises(P.NNGPError):
            ctx.factor(0, "exponential_isotropic", [1.0, 0.1])  # wrong covparms length


def test_size_independent_properties_large(P, O):
    """n = 2e5, m = 15: local-form oracle agreement + stationarity of the
    sweep map (zero noise, huge noise variance => Gibbs on the prior is a
    contraction towards 0)."""
    n, m = 200_000, 15
    locs, NN, col, lm, y = make_problem(P, n, m, seed=21)
    cp = COVS["matern15_isotropic"]
    rng = np.random.default_rng(1)
    field = rng.normal(size=n)
    z = rng.normal(size=(1, n))
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "matern15_isotropic", cp)
        ctx.set_field(field)
        ctx.set_mu(None, 0.0)
        ctx.sweep(1, 0.0, 0.0, 0.0, 0, 0, z=z)
        got = ctx.get_field()
        info = ctx.info
        Lo = ctx.get_linv(0)
    ref = O.sweep("local", field, Lo, NN, col, O.precision_diag(Lo, NN), np.ones(n, np.int32), y,
                  np.zeros(n), lm, 0.0, 0.0, 0.0, z)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-10)
    assert info["nnz"] == n * (m + 1) - m * (m + 1) // 2


@pytest.mark.parametrize("n,m,C", [(3000, 10, 2), (3000, 10, 3), (60000, 15, 4), (60000, 15, 3)])
def test_batched_chains_bitwise_equal_single_chain_contexts(P, O, n, m, C):
    """nngp_sweep_chains on a C-chain context (chains share the wavefronts)
    gives, for every chain, exactly the bits of the same context's chain
    swept alone; a 1-chain context agrees to rounding; chain 0 matches the
    oracle."""
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + C)
    rng = np.random.default_rng(C)
    cps = [[1.0 + 0.2 * k, 0.05 + 0.01 * k, 0.1 * k] for k in range(C)]
    fields = [rng.normal(size=n) for _ in range(C)]
    b0 = [0.2 * k for k in range(C)]
    ls = [0.1 - 0.05 * k for k in range(C)]
    lnv = [-0.3 + 0.1 * k for k in range(C)]
    seeds = [99 + k for k in range(C)]
    bases = [7 + 3 * k for k in range(C)]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        info = ctx.info
        assert info["n_chains"] == C
        if info["sweep_engine"] == 0:
            assert info["lanes_per_chain"] == {2: 32, 3: 16, 4: 16}[C]
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "matern15_isotropic", cps[k])
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0[k])
        ctx.sweep_chains(4, b0, ls, lnv, seeds, bases)
        got = [ctx.select(k).get_field() for k in range(C)]
        Lo0 = ctx.select(0).get_linv(0)
    # same context layout, chains swept one at a time: bitwise identical
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as seq:
        for k in range(C):
            seq.select(k)
            seq.factor(0, "matern15_isotropic", cps[k])
            seq.set_field(fields[k])
            seq.set_mu(None, b0[k])
        for k in range(C):
            seq.select(k).sweep(4, b0[k], ls[k], lnv[k], seeds[k], bases[k])
        for k in range(C):
            np.testing.assert_array_equal(got[k], seq.select(k).get_field())
    # a 1-chain context (64-lane layout: other lane splits => other summation
    # order inside a column): equal to rounding
    for k in range(C):
        with _ctx(P, locs, NN, col, lm, y) as one:
            one.factor(0, "matern15_isotropic", cps[k])
            one.set_field(fields[k])
            one.set_mu(None, b0[k])
            one.sweep(4, b0[k], ls[k], lnv[k], seeds[k], bases[k])
            np.testing.assert_allclose(got[k], one.get_field(), rtol=1e-11, atol=1e-12)
    z = O.sweep_normals(seeds[0], bases[0], 4, n)
    ref = O.sweep("local", fields[0], Lo0, NN, col, O.precision_diag(Lo0, NN), np.ones(n, np.int32), y,
                  np.full(n, b0[0]), lm, b0[0], ls[0], lnv[0], z)
    np.testing.assert_allclose(got[0], ref, rtol=1e-7, atol=1e-8)


@pytest.mark.parametrize("n,m", [(6000, 20), (60000, 15)])
def test_colour_engine_21_lanes_three_chains(P, O, monkeypatch, n, m):
    """The colour engine at 3 chains on 21 lanes per chain (its layout when a
    column of B is longer than the 16-lane chunk's 256 entries: m = 20 at
    n >= ~1e6, configs[4] on one GPU; forced here by NNGP_COLOUR_LANES=21):
    every chain bitwise equal to the same context's chain swept alone, equal
    to rounding to a 1-chain context, chain 0 to the oracle."""
    monkeypatch.setenv("NNGP_ENGINE", "colors")
    monkeypatch.setenv("NNGP_COLOUR_LANES", "21")
    C = 3
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + m)
    rng = np.random.default_rng(m)
    cps = [[1.0 + 0.2 * k, 0.05 + 0.01 * k, 0.1 * k] for k in range(C)]
    fields = [rng.normal(size=n) for _ in range(C)]
    b0, ls, lnv = [0.2 * k for k in range(C)], [0.1 - 0.05 * k for k in range(C)], [-0.3 + 0.1 * k for k in range(C)]
    seeds, bases = [99 + k for k in range(C)], [7 + 3 * k for k in range(C)]

    def setup(ctx):
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "matern15_isotropic", cps[k])
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0[k])

    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        assert ctx.info["sweep_engine"] == 0 and ctx.info["lanes_per_chain"] == 21, ctx.info
        setup(ctx)
        ctx.sweep_chains(4, b0, ls, lnv, seeds, bases)
        got = [ctx.select(k).get_field() for k in range(C)]
        Lo0 = ctx.select(0).get_linv(0)
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as seq:
        setup(seq)
        for k in range(C):
            seq.select(k).sweep(4, b0[k], ls[k], lnv[k], seeds[k], bases[k])
        for k in range(C):
            np.testing.assert_array_equal(got[k], seq.select(k).get_field())
    for k in range(C):
        with P.ChainContext(locs, NN, col, lm, y, device=0) as one:
            one.factor(0, "matern15_isotropic", cps[k])
            one.set_field(fields[k])
            one.set_mu(None, b0[k])
            one.sweep(4, b0[k], ls[k], lnv[k], seeds[k], bases[k])
            np.testing.assert_allclose(got[k], one.get_field(), rtol=1e-11, atol=1e-12)
    z = O.sweep_normals(seeds[0], bases[0], 4, n)
    ref = O.sweep("local", fields[0], Lo0, NN, col, O.precision_diag(Lo0, NN), np.ones(n, np.int32), y,
                  np.full(n, b0[0]), lm, b0[0], ls[0], lnv[0], z)
    np.testing.assert_allclose(got[0], ref, rtol=1e-7, atol=1e-8)


def test_single_chain_sweep_inside_batched_context(P, O):
    """nngp_sweep on one chain of a 3-chain context leaves the other chains
    untouched and equals the oracle (injected normals)."""
    n, m = 4000, 8
    locs, NN, col, lm, y = make_problem(P, n, m, seed=3)
    rng = np.random.default_rng(8)
    fields = [rng.normal(size=n) for _ in range(3)]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=3) as ctx:
        for k in range(3):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", [1.0, 0.1, 0.05])
            ctx.set_field(fields[k])
            ctx.set_mu(None, 0.0)
        z = rng.normal(size=(2, n))
        ctx.select(1).sweep(2, 0.0, 0.0, 0.0, 0, 0, z=z)
        got = [ctx.select(k).get_field() for k in range(3)]
        Lo = ctx.select(1).get_linv(0)
    np.testing.assert_array_equal(got[0], fields[0])
    np.testing.assert_array_equal(got[2], fields[2])
    ref = O.sweep("local", fields[1], Lo, NN, col, O.precision_diag(Lo, NN), np.ones(n, np.int32), y,
                  np.zeros(n), lm, 0.0, 0.0, 0.0, z)
    np.testing.assert_allclose(got[1], ref, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("plan", ["dag", "levels"])
@pytest.mark.parametrize("n,m", [(5000, 5), (120000, 15)])
def test_blocked_tri_solve_equals_level_schedule(P, O, n, m, plan, monkeypatch):
    """The sync-free one-launch solve (default, `dag`) and the blocked plan
    (`levels`: runs of small DAG levels in one workgroup) give exactly the
    bits of one launch per level, repeatedly, and match the oracle."""
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + 1)
    cp = COVS["matern15_isotropic"]
    rng = np.random.default_rng(3)
    us = [rng.normal(size=n) for _ in range(3)]
    monkeypatch.setenv("NNGP_TRI", plan)
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "matern15_isotropic", cp)
        got = [ctx.tri_solve(0, u) for u in us]
        Lo = ctx.get_linv(0)
    monkeypatch.setenv("NNGP_TRI", "level")
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "matern15_isotropic", cp)
        ref = [ctx.tri_solve(0, u) for u in us]
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_allclose(got[0], O.tri_solve(Lo, NN, us[0]), rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("n,m,C,mask", [(5000, 5, 3, 0b101), (120000, 15, 4, 0b1111), (3000, 10, 2, 0b11)])
def test_batched_ancillary_bitwise_equal_per_chain(P, O, n, m, C, mask):
    """nngp_ancillary_propose_chains (one solve schedule for the masked
    chains) gives every masked chain exactly the proposal of
    nngp_ancillary_propose on that chain alone; chain 0 matches the oracle
    form beta0 + exp(dls/2) B1^{-1} B0 (field - beta0) (update_Gaussian.R:127)."""
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + C + 5)
    rng = np.random.default_rng(C + 11)
    c0s = [[1.0 + 0.1 * k, 0.05 + 0.01 * k, 0.0] for k in range(C)]
    c1s = [[1.2 + 0.1 * k, 0.06 + 0.01 * k, 0.0] for k in range(C)]
    fields = [rng.normal(size=n) + 0.5 * k for k in range(C)]
    b0 = np.array([0.3 * k for k in range(C)])
    dls = np.array([0.2 - 0.1 * k for k in range(C)])

    def setup(ctx):
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", c0s[k])
            ctx.factor(1, "exponential_isotropic", c1s[k])
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0[k])

    chains = [k for k in range(C) if (mask >> k) & 1]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        setup(ctx)
        ctx.ancillary_propose_chains(mask, b0, dls)
        got = {}
        for k in chains:
            ctx.select(k).accept_field()
            got[k] = ctx.get_field()
        untouched = [ctx.select(k).get_field() for k in range(C) if k not in chains]
        L0, L1 = ctx.select(0).get_linv(0), ctx.select(0).get_linv(1)
    for f, k in zip(untouched, [k for k in range(C) if k not in chains]):
        np.testing.assert_array_equal(f, fields[k])
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as seq:
        setup(seq)
        for k in chains:
            seq.select(k).ancillary_propose(b0[k], dls[k])
            seq.accept_field()
            np.testing.assert_array_equal(got[k], seq.get_field())
    w = O.tri_solve(L1, NN, O.linv_mult(L0, fields[0] - b0[0], NN))
    np.testing.assert_allclose(got[0], b0[0] + np.exp(0.5 * dls[0]) * w, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("m", [3, 7, 15, 20, 31])
def test_tri_solve_every_row_width(P, O, m):
    """The solve's row kernel is specialised on b = m+1 (<= 8, 16, 32):
    each variant matches the oracle, batched over chains too."""
    n = 6000
    locs, NN, col, lm, y = make_problem(P, n, m, seed=m)
    rng = np.random.default_rng(m)
    u = rng.normal(size=n)
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=2) as ctx:
        for k in range(2):
            ctx.select(k).factor(0, "exponential_isotropic", [1.0, 0.08 + 0.02 * k, 0.01])
        got = [ctx.select(k).tri_solve(0, u) for k in range(2)]
        Ls = [ctx.select(k).get_linv(0) for k in range(2)]
    for g, L in zip(got, Ls):
        np.testing.assert_allclose(g, O.tri_solve(L, NN, u), rtol=1e-9, atol=1e-10)


def test_configs1_synthetic_1e5_m10_exponential(P, O):
    """BASELINE configs[1]: synthetic 2-D, n = 1e5, m = 10, exponential
    covariance -- factor, log-likelihood and two chromatic sweeps (default
    engine, Philox normals) against the oracle."""
    n, m = 100_000, 10
    locs, NN, col, lm, y = make_problem(P, n, m, seed=101)
    cp = [1.0, 0.1, 0.0]
    field = np.random.default_rng(2).normal(size=n)
    seed, base = 4242, 3
    with _ctx(P, locs, NN, col, lm, y) as ctx:
        ctx.factor(0, "exponential_isotropic", cp)
        Linv = ctx.get_linv(0)
        ctx.set_field(field)
        ctx.set_mu(None, 0.5)
        ll = ctx.loglik(0, 0.5, 0.3)
        ctx.sweep(2, 0.5, 0.3, -1.0, seed, base)
        got = ctx.get_field()
    Lo = O.vecchia_linv("exponential_isotropic", cp, locs, NN)
    np.testing.assert_allclose(Linv, Lo, rtol=1e-9, atol=1e-10)
    llo = O.loglik(Lo, field - 0.5, NN, 0.3)
    assert abs(ll - llo) <= 1e-10 * abs(llo)
    z = O.sweep_normals(seed, base, 2, n)
    ref = O.sweep("local", field, Lo, NN, col, O.precision_diag(Lo, NN), np.ones(n, np.int32), y,
                  np.full(n, 0.5), lm, 0.5, 0.3, -1.0, z)
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9)


def test_headline_size_1e6_m15_three_chains(P, O):
    """The headline workload itself (n = 1e6, m = 15, Matern 3/2, 3 chains in
    one context, the default engine): every chain's field after one call of 2
    sweeps against the oracle's local-form sweep with the same Philox normals
    and the device's own factor (isolates the sweep), its log-likelihood
    against the oracle's on that factor (1e-10), and the factor against the
    oracle's per row within DESIGN §4's bound max(1e-10, 1e-14 cond(C_i)) x
    max|row| (at this density, range 0.04 over 1e6 points, many local
    covariances are near-singular)."""
    n, m, C = 1_000_000, 15, 3
    locs, NN, col, lm, y = make_problem(P, n, m, seed=7)
    cps = [[1.0, 0.05, 0.0], [1.2, 0.04, 0.0], [0.8, 0.06, 0.0]]
    rng = np.random.default_rng(5)
    fields = [rng.normal(size=n) for _ in range(C)]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "matern15_isotropic", cps[k])
            ctx.set_field(fields[k])
            ctx.set_mu(None, 0.1 * k)
        Ls = []
        for k in range(C):
            ctx.select(k)
            Ls.append(ctx.get_linv(0))
        ctx.select(1)
        L1 = Ls[1]
        ll = ctx.loglik(0, 0.1, 0.2)
        b0s, lss, lnvs, seeds = [0.0, 0.1, 0.2], [0.0, 0.2, -0.1], [-0.5, -0.4, -0.6], [11, 12, 13]
        ctx.sweep_chains(2, b0s, lss, lnvs, seeds, [0, 0, 0])
        got = []
        for k in range(C):
            ctx.select(k)
            got.append(ctx.get_field())
    llo = O.loglik(L1, fields[1] - 0.1, NN, 0.2)
    assert abs(ll - llo) <= 1e-10 * abs(llo)
    for k in range(C):  # every chain of the batched call
        z = O.sweep_normals(seeds[k], 0, 2, n)
        ref = O.sweep("local", fields[k], Ls[k], NN, col, O.precision_diag(Ls[k], NN), np.ones(n, np.int32), y,
                      np.full(n, 0.1 * k), lm, b0s[k], lss[k], lnvs[k], z)
        np.testing.assert_allclose(got[k], ref, rtol=1e-8, atol=1e-9, err_msg=f"chain {k}")
    Lo = O.vecchia_linv("matern15_isotropic", cps[1], locs, NN)
    err = np.abs(L1 - Lo).max(axis=1)
    scale = np.abs(Lo).max(axis=1)
    bad = np.nonzero(err > 1e-10 * scale)[0]
    if len(bad):
        covs = np.stack([O.covmat("matern15_isotropic", cps[1], locs[NN[i][NN[i] != O.NA] - 1]) for i in bad
                         if (NN[i] != O.NA).sum() == m + 1])
        full = np.array([i for i in bad if (NN[i] != O.NA).sum() == m + 1])
        kappa = np.linalg.cond(covs)
        assert np.all(err[full] <= np.maximum(1e-10, 1e-14 * kappa) * scale[full])
        short = np.setdiff1d(bad, full)  # the first m rows (fewer neighbours)
        for i in short:
            idx = NN[i][NN[i] != O.NA] - 1
            k = np.linalg.cond(O.covmat("matern15_isotropic", cps[1], locs[idx]))
            assert err[i] <= max(1e-10, 1e-14 * k) * scale[i]


@pytest.mark.parametrize("C", [1, 3])
def test_tile_engine_multipass_ghost_cells(P, O, C, monkeypatch):
    """Tile engine with 1024-thread tiles (NNGP_TILE_NT=1024: one ghost
    register per thread, 1024 ghost cells per pass) on 32 tiles at n = 1e5,
    m = 20: some (tile, colour) holds more ghost cells than a pass, so the
    hand-off applies them in several passes -- double-buffered at 1 chain, one
    register set at 3 chains.  Every chain against the oracle's local-form
    sweep with the same Philox normals (2 sweeps, 1e-8)."""
    monkeypatch.setenv("NNGP_TILES", "32")
    monkeypatch.setenv("NNGP_TILE_NT", "1024")
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    n, m = 100_000, 20
    locs, NN, col, lm, y = make_problem(P, n, m, seed=21)
    cps = [[1.0, 0.1, 0.0], [0.7, 0.05, 0.0], [1.3, 0.08, 0.0]][:C]
    rng = np.random.default_rng(2)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0s, lss, lnvs, seeds = [0.1, -0.2, 0.3][:C], [0.0, 0.2, -0.3][:C], [-0.5, -0.2, -0.9][:C], [5, 6, 7][:C]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        info = ctx.info
        assert info["sweep_engine"] == 1 and info["n_tiles"] == 32
        assert info["tile_ghost_cells_max"] > info["tile_ghost_pass"] == 1024, info
        Ls = []
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", cps[k])
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0s[k])
            Ls.append(ctx.get_linv(0))
        ctx.sweep_chains(2, b0s, lss, lnvs, seeds, [3] * C)
        got = []
        for k in range(C):
            ctx.select(k)
            got.append(ctx.get_field())
    for k in range(C):
        z = O.sweep_normals(seeds[k], 3, 2, n)
        ref = O.sweep("local", fields[k], Ls[k], NN, col, O.precision_diag(Ls[k], NN), np.ones(n, np.int32), y,
                      np.full(n, b0s[k]), lm, b0s[k], lss[k], lnvs[k], z)
        np.testing.assert_allclose(got[k], ref, rtol=1e-8, atol=1e-9, err_msg=f"chain {k}")


@pytest.mark.parametrize("xw", ["0", "1"])
def test_tile_residency_fallback(P, O, monkeypatch, xw):
    """More tiles than the device holds at once (NNGP_TILES = 2 x CUs): the
    persistent tile sweep spins on its neighbours' granules, so it needs
    every workgroup resident.  The occupancy query at creation sees that the
    grid does not fit and the context runs the colour engine instead, saying
    why (engine_fallback 2, the note names the residency) -- no spin timeout --
    and the sweep still equals the oracle's."""
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.setenv("NNGP_TILE_XW", xw)
    n, m = 40_000, 10
    locs, NN, col, lm, y = make_problem(P, n, m, seed=33)
    with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
        cus = ctx.info["device_cus"]
    assert cus > 0
    monkeypatch.setenv("NNGP_TILES", str(2 * cus))
    field = np.random.default_rng(3).normal(size=n)
    with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
        info = ctx.info
        assert info["sweep_engine"] == 0 and info["engine_fallback"] == 2, info
        assert "residency" in info["engine_note"], info["engine_note"]
        ctx.factor(0, "exponential_isotropic", [1.0, 0.1, 0.0])
        L = ctx.get_linv(0)
        ctx.set_field(field)
        ctx.set_mu(None, 0.2)
        ctx.sweep_chains(2, [0.2], [0.1], [-0.4], [9], [0])
        got = ctx.get_field()
    z = O.sweep_normals(9, 0, 2, n)
    ref = O.sweep("local", field, L, NN, col, O.precision_diag(L, NN), np.ones(n, np.int32), y, np.full(n, 0.2), lm,
                  0.2, 0.1, -0.4, z)
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9)
    # at one tile per CU the tile engine runs, with its occupancy on record
    monkeypatch.setenv("NNGP_TILES", str(cus))
    with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
        info = ctx.info
        assert info["sweep_engine"] == 1 and info["engine_fallback"] == 0, info
        assert info["tile_resident_per_cu"] >= 1 and info["tile_exchange_wave"] == int(xw), info
        assert "tiles:" in info["engine_note"], info["engine_note"]


@pytest.mark.parametrize("n,m,C", [(20000, 10, 1), (60000, 15, 3), (3000, 5, 2), (40000, 20, 4)])
def test_tile_engine_r_in_global_memory_equals_lds_bitwise(P, engine, monkeypatch, n, m, C):
    """Tiles whose r lives in global memory (the layout beyond the LDS: n = 1e7
    on one GPU; NNGP_TILE_R=global forces it) run the same arithmetic in the
    same order as the LDS tiles: every chain's field bitwise equal after two
    calls (3 + 2 sweeps)."""
    if engine != "tiles-default":
        pytest.skip("sets the engine itself")
    # the same 512-thread cell layout on both sides (exchange-wave tiles cut
    # their batches for 448 cell threads, and r in global memory has none)
    monkeypatch.setenv("NNGP_TILE_XW", "0")
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + C)
    rng = np.random.default_rng(C)
    fields = [rng.normal(size=n) for _ in range(C)]
    out = []
    for rg in (False, True):
        if rg:
            monkeypatch.setenv("NNGP_TILE_R", "global")
        else:
            monkeypatch.delenv("NNGP_TILE_R", raising=False)
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            info = ctx.info
            assert info["sweep_engine"] == 1 and info["tile_r_global"] == int(rg)
            for k in range(C):
                ctx.select(k)
                ctx.factor(0, "matern15_isotropic", [1.0, 0.05 + 0.01 * k, 0.0])
                ctx.set_field(fields[k])
                ctx.set_mu(None, 0.1 * k)
            ctx.sweep_chains(3, [0.1 * k for k in range(C)], [0.1] * C, [-0.4] * C, [31 + k for k in range(C)],
                             [0] * C)
            ctx.sweep_chains(2, [0.1 * k for k in range(C)], [0.0] * C, [-0.5] * C, [41 + k for k in range(C)],
                             [3] * C)
            res = []
            for k in range(C):
                ctx.select(k)
                res.append(ctx.get_field())
            out.append(res)
    for k in range(C):
        np.testing.assert_array_equal(out[1][k], out[0][k], err_msg=f"chain {k}")


@pytest.mark.parametrize("n,m,C", [(20000, 10, 1), (60000, 15, 3), (40000, 20, 4)])
def test_tile_engine_r_in_global_wave_local_equals_lds_bitwise(P, engine, monkeypatch, n, m, C):
    """Wave-local batches (tiles.hip tile_phase_wl) with r in global memory
    (the route n = 1e7 takes on one GPU at 3 chains, where the colour engine
    refuses m = 20) == wave-local LDS tiles on the same layout, bitwise, after
    two calls (3 + 2 sweeps)."""
    if engine != "tiles-default":
        pytest.skip("sets the engine itself")
    monkeypatch.setenv("NNGP_TILE_WL", "1")
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + C + 7)
    rng = np.random.default_rng(C + 7)
    fields = [rng.normal(size=n) for _ in range(C)]
    out = []
    for rg in (False, True):
        if rg:
            monkeypatch.setenv("NNGP_TILE_R", "global")
        else:
            monkeypatch.delenv("NNGP_TILE_R", raising=False)
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            info = ctx.info
            assert info["sweep_engine"] == 1 and info["tile_r_global"] == int(rg), info
            assert "wave-local" in info["engine_note"], info["engine_note"]
            for k in range(C):
                ctx.select(k)
                ctx.factor(0, "matern15_isotropic", [1.0, 0.05 + 0.01 * k, 0.0])
                ctx.set_field(fields[k])
                ctx.set_mu(None, 0.1 * k)
            ctx.sweep_chains(3, [0.1 * k for k in range(C)], [0.1] * C, [-0.4] * C, [31 + k for k in range(C)],
                             [0] * C)
            ctx.sweep_chains(2, [0.1 * k for k in range(C)], [0.0] * C, [-0.5] * C, [41 + k for k in range(C)],
                             [3] * C)
            res = []
            for k in range(C):
                ctx.select(k)
                res.append(ctx.get_field())
            out.append(res)
    for k in range(C):
        np.testing.assert_array_equal(out[1][k], out[0][k], err_msg=f"chain {k}")


@pytest.mark.parametrize("n,m,C,rg", [(60000, 15, 3, False), (200000, 15, 3, False), (40000, 20, 4, False),
                                      (60000, 15, 3, True)])
def test_tile_engine_interior_first_wave_local_matches_wave_local(P, engine, monkeypatch, n, m, C, rg):
    """Interior-first wave-local tiles (NNGP_TILE_SPLIT=1, tiles.hip
    tile_phase_wlib: a colour's interior batches overlap the previous
    colour's hand-off) == plain wave-local tiles after two calls (3 + 2
    sweeps) to 1e-11: the same per-row update order, but the split layout
    cuts a slot's cells over other lanes, so its sum rounds differently
    (measured: 7e-15 absolute)."""
    if engine != "tiles-default":
        pytest.skip("sets the engine itself")
    monkeypatch.setenv("NNGP_TILE_WL", "1")
    if rg:
        monkeypatch.setenv("NNGP_TILE_R", "global")
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + C + 11)
    rng = np.random.default_rng(C + 11)
    fields = [rng.normal(size=n) for _ in range(C)]
    out = []
    for split in (False, True):
        if split:
            monkeypatch.setenv("NNGP_TILE_SPLIT", "1")
        else:
            monkeypatch.delenv("NNGP_TILE_SPLIT", raising=False)
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            info = ctx.info
            assert info["sweep_engine"] == 1 and "wave-local" in info["engine_note"], info["engine_note"]
            assert ("interior first" in info["engine_note"]) == split, info["engine_note"]
            for k in range(C):
                ctx.select(k)
                ctx.factor(0, "matern15_isotropic", [1.0, 0.05 + 0.01 * k, 0.0])
                ctx.set_field(fields[k])
                ctx.set_mu(None, 0.1 * k)
            ctx.sweep_chains(3, [0.1 * k for k in range(C)], [0.1] * C, [-0.4] * C, [31 + k for k in range(C)],
                             [0] * C)
            ctx.sweep_chains(2, [0.1 * k for k in range(C)], [0.0] * C, [-0.5] * C, [41 + k for k in range(C)],
                             [3] * C)
            res = []
            for k in range(C):
                ctx.select(k)
                res.append(ctx.get_field())
            out.append(res)
    for k in range(C):
        np.testing.assert_allclose(out[1][k], out[0][k], rtol=1e-11, atol=1e-12, err_msg=f"chain {k}")


def test_beta0_stats_reuses_loglik_pass_and_invalidates(P, O, engine):
    """nngp_beta0_stats answers from the last log-likelihood pass over the
    current factor and field ((B1)'(Bf) = (B1)'(B(f - b0)) + b0 (B1)'(B1)),
    within 1e-12 of a fresh pass; every write of the field or the factor
    (set_field, sweep, accept_field, factor, accept_factor) invalidates it."""
    if engine != "tiles-default":
        pytest.skip("engine independent")
    n, m = 5000, 10
    locs, NN, col, lm, y = make_problem(P, n, m, seed=3)
    rng = np.random.default_rng(8)
    cp0, cp1 = [1.0, 0.1, 0.0], [1.0, 0.15, 0.0]

    with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
        ctx.factor(0, "exponential_isotropic", cp0)
        ctx.set_field(rng.normal(size=n))
        ctx.set_mu(None, 0.3)
        fresh = ctx.beta0_stats()                     # no pass cached yet: a direct pass
        ctx.loglik(0, 0.3, 0.1)
        cached = ctx.beta0_stats()
        np.testing.assert_allclose(cached, fresh, rtol=1e-12)
        ctx.factor(1, "exponential_isotropic", cp1)
        ctx.loglik(1, 0.3, 0.0)
        ctx.accept_factor()                           # the proposal's pass becomes the current one
        after_accept = ctx.beta0_stats()
        ctx.set_field(ctx.get_field())                # same values, new generation: a fresh pass
        np.testing.assert_allclose(after_accept, ctx.beta0_stats(), rtol=1e-12)
        ctx.loglik(0, 0.3, 0.0)
        ctx.sweep(1, 0.3, 0.0, -0.5, 5, 0)            # the field changes
        swept = ctx.beta0_stats()
        ctx.set_field(ctx.get_field())
        np.testing.assert_allclose(swept, ctx.beta0_stats(), rtol=1e-12)
        assert abs(swept[1] - after_accept[1]) > 1e-9 * abs(after_accept[1])
        # the oracle's 1'B'B1 and 1'B'Bf on the final state
        L, f = ctx.get_linv(0), ctx.get_field()
        B1, Bf = O.linv_mult(L, np.ones(n), NN), O.linv_mult(L, f, NN)
        np.testing.assert_allclose(swept, [B1 @ B1, B1 @ Bf], rtol=1e-10)


@pytest.mark.parametrize("n,m,C", [(60000, 15, 3), (20000, 10, 4)])
def test_tile_engine_interior_first_split_matches_oracle(P, O, engine, monkeypatch, n, m, C):
    """Interior-first tile layouts (NNGP_TILE_SPLIT=1: per colour the slots
    that need no hand-off of the previous colour first, kernels.hip
    tile_phase_ib): every chain after a call of 3 sweeps against the
    oracle's local-form sweep with the same normals (rtol 1e-8: rows take the
    updates of colours c and c-1 in either order)."""
    if engine != "tiles-default":
        pytest.skip("sets the layout itself")
    monkeypatch.setenv("NNGP_TILE_SPLIT", "1")
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + 1)
    rng = np.random.default_rng(2)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0s, lss, lnvs, seeds = [0.1 * k for k in range(C)], [0.1] * C, [-0.4] * C, [51 + k for k in range(C)]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        assert ctx.info["sweep_engine"] == 1
        Ls = []
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "matern15_isotropic", [1.0, 0.05 + 0.01 * k, 0.0])
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0s[k])
            Ls.append(ctx.get_linv(0))
        ctx.sweep_chains(3, b0s, lss, lnvs, seeds, [0] * C)
        got = []
        for k in range(C):
            ctx.select(k)
            got.append(ctx.get_field())
    for k in range(C):
        z = O.sweep_normals(seeds[k], 0, 3, n)
        ref = O.sweep("local", fields[k], Ls[k], NN, col, O.precision_diag(Ls[k], NN), np.ones(n, np.int32), y,
                      np.full(n, b0s[k]), lm, b0s[k], lss[k], lnvs[k], z)
        np.testing.assert_allclose(got[k], ref, rtol=1e-8, atol=1e-9, err_msg=f"chain {k}")


@pytest.mark.parametrize("n,m,C", [(20000, 10, 2), (60000, 15, 3), (3000, 5, 4), (40000, 20, 3), (1_000_000, 15, 3)])
def test_tile_engine_chain_split_equals_joint_bitwise(P, engine, monkeypatch, n, m, C):
    """Chain-split tile launches (NNGP_TILE_CHAINS=split: one workgroup per
    (chain, tile), the chains' workgroups of a tile sharing its CU) run each
    chain's arithmetic in the order of the joint 256-thread tiles (one
    workgroup per tile running every chain) cut into the same 2048-cell
    batches: every chain's field bitwise equal after two calls (3 + 2
    sweeps)."""
    if engine != "tiles-default":
        pytest.skip("sets the engine itself")
    monkeypatch.setenv("NNGP_TILE_NT", "256")
    monkeypatch.setenv("NNGP_TILE_BATCH_CELLS", "2048")
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + C)
    rng = np.random.default_rng(C)
    fields = [rng.normal(size=n) for _ in range(C)]
    out = []
    for mode in ("joint", "split"):
        monkeypatch.setenv("NNGP_TILE_CHAINS", mode)
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            info = ctx.info
            assert info["sweep_engine"] == 1 and info["tile_chain_split"] == int(mode == "split"), info["engine_note"]
            for k in range(C):
                ctx.select(k)
                ctx.factor(0, "matern15_isotropic", [1.0, 0.05 + 0.01 * k, 0.0])
                ctx.set_field(fields[k])
                ctx.set_mu(None, 0.1 * k)
            ctx.sweep_chains(3, [0.1 * k for k in range(C)], [0.1] * C, [-0.4] * C, [31 + k for k in range(C)],
                             [0] * C)
            ctx.sweep_chains(2, [0.1 * k for k in range(C)], [0.0] * C, [-0.5] * C, [41 + k for k in range(C)],
                             [3] * C)
            res = []
            for k in range(C):
                ctx.select(k)
                res.append(ctx.get_field())
            out.append(res)
    for k in range(C):
        np.testing.assert_array_equal(out[1][k], out[0][k], err_msg=f"chain {k}")
