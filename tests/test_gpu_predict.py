"""Posterior prediction (Scripts/mcmc_nngp_predict.R:1-60):
mcmc_nngp_predict_field on the device (factor on the stacked locations, B11 w
by the device SpMV, the device triangular solve) against the oracle's
restatement of predict.R with the same normals for the new locations."""
import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu


def _z_new(L, n_pred, burn_in, seed):
    chains = list(L["records"].values())
    stored = np.asarray(chains[0]["saved_field"])
    n_s = int((stored > burn_in * stored.max()).sum())
    rng = np.random.default_rng(seed)
    return [rng.normal(size=(n_s, n_pred)) for _ in chains]


def _check(P, O, L, pred, m, burn_in=0.5, rtol=1e-9):
    z = _z_new(L, len(pred), burn_in, 99)
    got = P.mcmc_nngp_predict_field(L, pred, burn_in=burn_in, m=m, z_new=z, device=0)
    ref = O.predict_field(L, pred, z, burn_in=burn_in, m=m)
    assert len(got["predicted_field_samples"]) == len(ref)
    for g, r in zip(got["predicted_field_samples"], ref):
        assert g.shape == r.shape
        scale = np.abs(r).max()
        np.testing.assert_allclose(g, r, rtol=rtol, atol=rtol * scale)
    allsamp = np.vstack(ref)  # summary over all chains' samples (predict.R:57-58)
    np.testing.assert_allclose(got["predicted_field_summary"][:, 0], allsamp.mean(0), rtol=1e-8, atol=1e-8 * scale)
    return got, ref


def test_predict_field_vignette_run_matches_oracle(P, O, toy):
    """Vignette toy (n = 2000, m = 5, exponential, X_locs), 2 chains, a short
    run with field_thinning = .5; 300 new locations predicted with m = 5.
    Saved samples whose shape repeats reuse the factor (predict.R:23,32)."""
    L = P.mcmc_nngp_initialize(toy["locs"], toy["observed_field"], X_locs=toy["X"],
                               stationary_covfun="exponential_isotropic", m=5, n_chains=2, seed=3)
    L = P.mcmc_nngp_run(L, n_cycles=1, n_iterations_update=30, n_chromatic=3, field_thinning=0.5,
                        Gelman_Rubin_Brooks_stop=(1.0, 1.0), verbose=False)
    rng = np.random.default_rng(5)
    lo, hi = L["locs"].min(0), L["locs"].max(0)
    pred = lo + (hi - lo) * rng.uniform(size=(300, L["locs"].shape[1]))
    chains = list(L["records"].values())
    stored = chains[0]["saved_field"]
    stored = stored[stored > 0.5 * stored.max()].astype(int)
    sh = np.asarray(chains[0]["params"]["shape"])[stored - 1].ravel()
    assert len(np.unique(sh)) < len(sh), "want repeated shapes (factor reuse) in the saved samples"
    _check(P, O, L, pred, m=5)
    for c in L["_contexts"]:
        c.close()


def _synthetic_list(n, m, shapes, log_scales, beta0s, fields, covfun="exponential_isotropic", seed=0):
    """The parts of an mcmc_nngp_list predict.R reads: locs, the covariance
    model and per-chain records (iterations 1..len(shapes), every one saved)."""
    k = len(shapes)
    rec = {"saved_field": np.arange(1, k + 1, dtype=np.float64),
           "params": {"shape": np.asarray(shapes, np.float64).reshape(k, -1),
                      "log_scale": np.asarray(log_scales, np.float64).reshape(k, 1),
                      "beta_0": np.asarray(beta0s, np.float64).reshape(k, 1),
                      "field": np.asarray(fields, np.float64)}}
    return rec


def test_predict_field_1e5_matches_oracle(P, O):
    """n = 1e5 observed locations (configs[1] size, m = 10), 5,000 new ones;
    two chains whose saved shapes are [a, a, b, a] (the 4th reuses b's factor:
    predict.R recomputes only at !duplicated(shape), a reference quirk kept)."""
    n, m = 100_000, 10
    locs, NN, col, lm, y = make_problem(P, n, m, seed=12)
    rng = np.random.default_rng(1)
    a, b = np.log(0.1), np.log(0.05)
    recs = {}
    for ch in range(2):
        fields = 1.0 + rng.normal(size=(4, n))
        recs[f"chain_{ch + 1}"] = _synthetic_list(n, m, [a, a, b, a], [0.1 * ch, -0.2, 0.3, 0.0],
                                                  [1.0, 1.1, 0.9, 1.0], fields)
    L = {"locs": locs, "records": recs,
         "space_time_model": {"covfun": {"stationary_covfun": "exponential_isotropic",
                                         "shape_params": ["log_range"]}}}
    pred = rng.uniform(size=(5000, 2))
    _check(P, O, L, pred, m=m, burn_in=0.0)


def test_predict_field_matern_smoothness_transform(P, O):
    """matern_isotropic: predict.R:37 maps qlogis_smoothness with 1.5 * plogis
    (not the MCMC's .5 + .5 * plogis); one chain, shapes (range, smoothness)."""
    n, m = 3000, 8
    locs, *_ = make_problem(P, n, m, seed=4)
    rng = np.random.default_rng(2)
    shapes = [[np.log(0.1), 0.3], [np.log(0.1), 0.3], [np.log(0.08), -0.5]]
    L = {"locs": locs,
         "records": {"chain_1": _synthetic_list(n, m, shapes, [0.0, 0.1, -0.1], [0.5, 0.5, 0.4],
                                                rng.normal(size=(3, n)))},
         "space_time_model": {"covfun": {"stationary_covfun": "matern_isotropic",
                                         "shape_params": ["log_range", "qlogis_smoothness"]}}}
    pred = rng.uniform(size=(400, 2))
    _check(P, O, L, pred, m=m, burn_in=0.0, rtol=1e-8)
