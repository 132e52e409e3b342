"""Pin the CPU oracle: reference golden values (Vignette.md, regenerated toy
inputs), published known-answer vectors, and mathematical identities."""
import numpy as np
import pytest
import scipy.special as sps


def test_r_rng_reproduces_vignette_inputs(printed, toy):
    # Vignette.rmd:26-48 regenerated -> Vignette.md:136-142, 180-186
    np.testing.assert_allclose(toy["locs"][:6], printed["observed_locs_head"], atol=5e-5)
    Xc = toy["X"] - toy["X"].mean(0)
    np.testing.assert_allclose(Xc[:6], printed["X_head"], atol=5e-6, rtol=1e-6)


def test_ordering_prefix_and_locs_head(printed, toy):
    h = np.array(printed["hctam_scol_1_100"]) - 1
    np.testing.assert_allclose(toy["locs"][h[:6]], printed["locs_head"], atol=5e-6)
    # locs_match[o] = position of observation o in the ordering (for o <= 100
    # whose position is <= 100 the two printed maps agree)
    lm = np.array(printed["locs_match_100"])
    pos = {obs: q + 1 for q, obs in enumerate(printed["hctam_scol_1_100"])}
    for o in range(100):
        if (o + 1) in pos:
            assert pos[o + 1] == lm[o]


def _prefix_nn(O, printed, toy, m=5):
    h = np.array(printed["hctam_scol_1_100"]) - 1
    return O.find_ordered_nn(toy["locs"][h], m)


def test_oracle_nnarray_matches_vignette(O, printed, toy):
    NN = _prefix_nn(O, printed, toy)
    head = np.array([[O.NA if v is None else v for v in r] for r in printed["NNarray_head"]])
    np.testing.assert_array_equal(NN[:6], head)


def test_oracle_moral_graph_matches_vignette(O, printed, toy):
    NN = _prefix_nn(O, printed, toy)
    cp, ri = O.moral_graph(NN)
    M = np.zeros((100, 100), int)
    for j in range(100):
        M[ri[cp[j]:cp[j + 1]], j] = 1
    blk = np.array(printed["moral_block_30"])
    assert blk.sum() == 342
    np.testing.assert_array_equal(M[:30, :30], blk)


def test_oracle_coloring_first_30_from_printed_block(O, printed, toy):
    """Colours of nodes 1..30 depend only on their neighbours j < i, which
    all lie in the printed 30x30 block: run Coloring.R's algorithm on it."""
    blk = np.array(printed["moral_block_30"])
    cols = np.zeros(30, int)
    inc = np.zeros((31, blk.sum(0).max()), int)
    for i in range(30):
        cols[i] = np.argmax(inc[i] == 0) + 1
        inc[np.nonzero(blk[:, i])[0], cols[i] - 1] = 1
    col = O.greedy_coloring(_prefix_nn(O, printed, toy))
    np.testing.assert_array_equal(col[:30], cols)


def test_philox_known_answers(O):
    # Random123 philox4x32_10 KAT vectors
    kat = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ]
    for ctr, key, out in kat:
        np.testing.assert_array_equal(O.philox4x32_10(ctr, key), np.array(out, np.uint32))


def test_oracle_normals_are_standard(O):
    z = O.normals(1, 0, 200_000)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    from scipy.stats import kstest
    assert kstest(z, "norm").pvalue > 1e-3


def test_oracle_normals_independent_and_local(O):
    """One Philox call per location (counter = location, sweep): neighbouring
    locations and consecutive sweeps are uncorrelated, also in their squares;
    a location's normal does not depend on n."""
    z = O.normals(7, 3, 400_000)
    a, b = z[0::2], z[1::2]
    assert abs(np.corrcoef(a, b)[0, 1]) < 0.01
    assert abs(np.corrcoef(a * a, b * b)[0, 1]) < 0.01
    z4 = O.normals(7, 4, 400_000)
    assert abs(np.corrcoef(z, z4)[0, 1]) < 0.01
    np.testing.assert_array_equal(O.normals(7, 3, 11), z[:11])


def test_oracle_qnorm_known_values(O):
    """AS241 inversion against scipy's ndtri (published to ~1e-16)."""
    from scipy.special import ndtri
    p = np.concatenate([np.linspace(1e-12, 1 - 1e-12, 2001), [2.0 ** -54, 1e-300 + 2.0 ** -53, 0.5, 0.025, 0.975]])
    got = np.array([O.qnorm(x) for x in p])
    np.testing.assert_allclose(got, ndtri(p), rtol=1e-14, atol=1e-15)


@pytest.mark.parametrize("nu", [0.3, 0.5, 0.77, 1.0, 1.5, 2.2, 3.7])
def test_oracle_bessel_k(O, nu):
    for x in [1e-6, 1e-3, 0.1, 0.9, 2.0, 5.0, 30.0, 200.0]:
        assert O.bessel_k(nu, x) == pytest.approx(sps.kv(nu, x), rel=1e-11)


def test_matern_special_cases(O):
    rng = np.random.default_rng(0)
    locs = rng.uniform(size=(30, 2))
    C_half = O.covmat("matern_isotropic", [1.0, 0.2, 0.5, 0.0], locs)
    C_exp = O.covmat("exponential_isotropic", [1.0, 0.2, 0.0], locs)
    np.testing.assert_allclose(C_half, C_exp, rtol=1e-11)
    C15 = O.covmat("matern_isotropic", [1.0, 0.2, 1.5, 0.0], locs)
    C15e = O.covmat("matern15_isotropic", [1.0, 0.2, 0.0], locs)
    np.testing.assert_allclose(C15, C15e, rtol=1e-10)


def _problem(O, n=150, m=6, seed=0, covfun="exponential_isotropic", cp=(1.0, 0.15, 0.0)):
    rng = np.random.default_rng(seed)
    locs = rng.uniform(size=(n, 2))
    locs = locs[O.order_maxmin_exact(locs) - 1]
    NN = O.find_ordered_nn(locs, m)
    Linv = O.vecchia_linv(covfun, list(cp), locs, NN)
    return locs, NN, Linv


def test_vecchia_rows_are_dense_inverse_cholesky_rows(O):
    """KAT (i): B[i, .] is the last row of the inverse Cholesky factor of the
    local covariance, i.e. [1, -kriging weights] / sqrt(conditional var)."""
    locs, NN, Linv = _problem(O)
    for i in [0, 1, 5, 6, 40, 149]:
        idx = NN[i][NN[i] != O.NA] - 1
        C = O.covmat("exponential_isotropic", [1.0, 0.15, 0.0], locs[idx])
        if len(idx) > 1:
            w = np.linalg.solve(C[1:, 1:], C[1:, 0])
            cv = C[0, 0] - C[1:, 0] @ w
            expect = np.concatenate([[1.0], -w]) / np.sqrt(cv)
        else:
            expect = np.array([1.0 / np.sqrt(C[0, 0])])
        np.testing.assert_allclose(Linv[i, :len(idx)], expect, rtol=1e-10, atol=1e-12)


def test_loglik_is_dense_mvn_density(O):
    """KAT (ii): LL = log N(z; 0, s2 (B'B)^-1) + n/2 log(2 pi)."""
    locs, NN, Linv = _problem(O, n=120)
    B = O.dense_B(Linv, NN)
    Q = B.T @ B
    z = np.random.default_rng(1).normal(size=120)
    ls = 0.4
    cov = np.exp(ls) * np.linalg.inv(Q)
    sign, logdet = np.linalg.slogdet(cov)
    dense = -0.5 * logdet - 0.5 * z @ np.linalg.solve(cov, z)
    assert O.loglik(Linv, z, NN, ls) == pytest.approx(dense, rel=1e-9)


def test_masked_and_local_sweeps_agree(O):
    """KAT (iv): reference masked form == local form."""
    locs, NN, Linv = _problem(O, n=400, m=8)
    n = 400
    col = O.greedy_coloring(NN)
    D = O.precision_diag(Linv, NN)
    rng = np.random.default_rng(2)
    lm = np.concatenate([np.arange(1, n + 1), rng.integers(1, n + 1, 50)]).astype(np.int32)
    y = rng.normal(size=len(lm))
    mu = 0.3 + 0.1 * rng.normal(size=len(lm))
    opl = np.bincount(lm - 1, minlength=n).astype(np.int32)
    f0 = rng.normal(size=n)
    z = rng.normal(size=(3, n))
    a = O.sweep("masked", f0, Linv, NN, col, D, opl, y, mu, lm, 0.3, 0.2, -0.1, z)
    b = O.sweep("local", f0, Linv, NN, col, D, opl, y, mu, lm, 0.3, 0.2, -0.1, z)
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-13)


def test_chromatic_conditional_is_dense_gaussian_conditional(O):
    """KAT (iii): one colour update == exact conditional of the Vecchia prior x
    Gaussian likelihood given the other locations."""
    locs, NN, Linv = _problem(O, n=200, m=5)
    n = 200
    col = O.greedy_coloring(NN)
    D = O.precision_diag(Linv, NN)
    B = O.dense_B(Linv, NN)
    ls, lnv, b0 = 0.25, -0.5, 0.7
    rng = np.random.default_rng(3)
    lm = np.arange(1, n + 1, dtype=np.int32)
    y = rng.normal(size=n)
    mu = np.full(n, b0)
    f0 = rng.normal(size=n) + b0
    # only colour 1 moves: zero noise for the other colours is impossible to
    # isolate in the sweep, so compare the first colour of a single sweep
    z = rng.normal(size=(1, n))
    out = O.sweep("masked", f0, Linv, NN, col, D, np.ones(n, np.int32), y, mu, lm, b0, ls, lnv, z)
    Q = B.T @ B / np.exp(ls) + np.eye(n) / np.exp(lnv)
    w = f0 - b0
    bvec = (y - mu) / np.exp(lnv)
    for i in np.nonzero(col == 1)[0][:20]:
        cond_mean = (bvec[i] - (Q[i] @ w - Q[i, i] * w[i])) / Q[i, i]
        expect = b0 + cond_mean + z[0, i] / np.sqrt(Q[i, i])
        assert out[i] == pytest.approx(expect, rel=1e-10, abs=1e-12)


def test_coloring_is_proper_and_first_fit(O):
    locs, NN, _ = _problem(O, n=500, m=7)
    col = O.greedy_coloring(NN)
    cp, ri = O.moral_graph(NN)
    for i in range(500):
        nb = ri[cp[i]:cp[i + 1]]
        nb = nb[nb != i]
        assert np.all(col[nb] != col[i])
        earlier = set(col[nb[nb < i]])
        assert all(c in earlier for c in range(1, col[i]))  # first fit: smaller colours are blocked


def test_triangular_solve_inverts_linv_mult(O):
    locs, NN, Linv = _problem(O, n=300, m=9)
    x = np.random.default_rng(5).normal(size=300)
    np.testing.assert_allclose(O.tri_solve(Linv, NN, O.linv_mult(Linv, x, NN)), x, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("form", ["masked", "local"])
def test_threaded_oracle_sweeps_bitwise_equal_serial(O, form):
    """The OpenMP sweeps of the CPU baseline (one chain on all host cores)
    give exactly the serial restatement's field."""
    rng = np.random.default_rng(4)
    n, m = 3000, 8
    locs = rng.uniform(size=(n, 2))
    locs = locs[O.order_maxmin_exact(locs) - 1]
    NN = O.find_ordered_nn(locs, m)
    col = O.greedy_coloring(NN)
    Lo = O.vecchia_linv("exponential_isotropic", [1.0, 0.1, 0.0], locs, NN)
    D = O.precision_diag(Lo, NN)
    y = rng.normal(size=n)
    lm = np.arange(1, n + 1, dtype=np.int32)
    f0 = rng.normal(size=n)
    z = rng.normal(size=(2, n))
    args = (Lo, NN, col, D, np.ones(n, np.int32), y, np.full(n, 0.2), lm, 0.2, 0.1, -0.3, z)
    ref = O.sweep(form, f0, *args)
    for th in (2, 5):
        np.testing.assert_array_equal(O.sweep(form, f0, *args, threads=th), ref)
