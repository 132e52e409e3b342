"""Full Gibbs iterations of mcmc_nngp_update_Gaussian on the device vs the CPU
oracle of the same iteration (same seeds, same Philox stream), and the
vignette workflow's posterior summaries vs the values printed in the
reference's Vignette.md (statistical parity)."""
import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu


def _compare(res, ref, it, has_X):
    rec = res["records"]
    np.testing.assert_allclose(rec["beta_0"][:, 0], ref["records"]["beta_0"], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(rec["log_scale"][:, 0], ref["records"]["log_scale"], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(rec["log_noise_variance"][:, 0], ref["records"]["log_noise_variance"],
                               rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(rec["shape"], np.array(ref["records"]["shape"]), rtol=1e-7, atol=1e-9)
    if has_X:
        np.testing.assert_allclose(rec["beta"], np.array(ref["records"]["beta"]), rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(res["state"]["params"]["field"], ref["params"]["field"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(res["acceptance"]["covariance_acceptance_ancillary"], ref["acceptance"]["ancillary"])
    np.testing.assert_array_equal(res["acceptance"]["covariance_acceptance_sufficient"], ref["acceptance"]["sufficient"])


@pytest.mark.usefixtures("engine")
def test_update_iterations_match_oracle_no_X(P, O):
    import mcmc_oracle as MO
    from nngp_amd.update_gaussian import _philox_key, _run_chain

    n, m = 500, 6
    locs, NN, col, lm, y = make_problem(P, n, m, seed=31, dup_frac=0.1)
    y = y + 2.0
    va = {"n_locs": n, "n_obs": len(lm), "locs_match": lm, "NNarray": NN, "coloring": col,
          "obs_per_loc": np.bincount(lm - 1, minlength=n).astype(np.int32),
          "hctam_scol_1": np.arange(1, n + 1, dtype=np.int32)}
    stm = {"covfun": {"stationary_covfun": "exponential_isotropic", "shape_params": ["log_range"]}}
    rng = np.random.default_rng(0)
    state = {"params": {"beta_0": 2.0, "beta": None, "log_scale": 0.0, "shape": np.array([np.log(0.1)]),
                        "log_noise_variance": np.log(0.5), "field": 2.0 + rng.normal(size=n)},
             "transition_kernels": {"covariance_params_sufficient": {"logvar": -2.0},
                                    "covariance_params_ancillary": {"logvar": -2.0},
                                    "log_noise_variance": {"logvar": -1.0}}}
    X = {"X": None, "locs": np.zeros(0, np.int64)}
    iters, nc = 30, 3
    with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
        res = _run_chain(0, state, ctx, X, y, stm, va, iters, 1.0, True, nc, 0, 1)
    ref = MO.run_chain(0, state, locs, NN, col, X, y, stm, va, iters, 1.0, nc, 0, _philox_key(0, 1, 1))
    _compare(res, ref, iters, False)


@pytest.mark.usefixtures("engine")
def test_update_iterations_match_oracle_vignette_X_locs(P, O, toy):
    """Vignette toy (n = 2000, m = 5, X_locs with 2 columns => interweaving)."""
    import mcmc_oracle as MO
    from nngp_amd.update_gaussian import _philox_key, _run_chain

    L = P.mcmc_nngp_initialize(toy["locs"], toy["observed_field"], X_locs=toy["X"],
                               stationary_covfun="exponential_isotropic", m=5, n_chains=1, seed=1)
    st = L["states"]["chain_1"]
    va = L["vecchia_approx"]
    iters, nc = 30, 5
    res = _run_chain(0, st, L["_contexts"][0], L["X"], L["observed_field"], L["space_time_model"], va,
                     iters, 1.0, True, nc, 0, 1)
    ref = MO.run_chain(0, st, L["locs"], va["NNarray"], va["coloring"], L["X"], L["observed_field"],
                       L["space_time_model"], va, iters, 1.0, nc, 0, _philox_key(0, 1, 1))
    _compare(res, ref, iters, True)
    for c in L["_contexts"]:
        c.close()


@pytest.mark.usefixtures("engine")
def test_lockstep_batched_chains_equal_sequential_chains(P, toy):
    """mcmc_nngp_update_Gaussian drives the 3 chains of one context in
    lockstep with batched sweeps; every record equals the chains run one
    after another (each sweep alone) on an identical 3-chain context."""
    import copy

    from nngp_amd.context import make_chain_views
    from nngp_amd.update_gaussian import _run_chain, mcmc_nngp_update_Gaussian

    L = P.mcmc_nngp_initialize(toy["locs"], toy["observed_field"], X_locs=toy["X"],
                               stationary_covfun="exponential_isotropic", m=5, n_chains=3, seed=2)
    va = L["vecchia_approx"]
    assert len({id(v.ctx) for v in L["_contexts"]}) == 1  # one 3-chain context
    states0 = copy.deepcopy(L["states"])
    out = mcmc_nngp_update_Gaussian(L["locs"], L["X"], L["observed_field"], L["space_time_model"], va,
                                    L["states"], 20, field_thinning=0.1, n_chromatic=3,
                                    contexts=L["_contexts"], seed=1)
    views = make_chain_views(L["locs"], va["NNarray"], va["coloring"], va["locs_match"], L["observed_field"], 3)
    y = np.asarray(L["observed_field"], np.float64)
    for i, (nm, st) in enumerate(states0.items()):
        ref = _run_chain(i, st, views[i], L["X"], y, L["space_time_model"], va, 20, 0.1, True, 3, 0, 1)
        for key in ("beta_0", "log_scale", "log_noise_variance", "shape", "beta", "field"):
            np.testing.assert_array_equal(out[nm]["records"][key], ref["records"][key], err_msg=f"{nm} {key}")
    views[0].ctx.close()
    L["_contexts"][0].close()


def _dump_vignette(est, printed):
    import json
    from pathlib import Path

    out = Path(__file__).resolve().parent.parent / "gpurun_out"
    if out.is_dir():
        g = est["covariance_params"]["GpGp_covparams"]
        fe = est["fixed_effects"]
        (out / "vignette_estimates.json").write_text(json.dumps({
            "ours": {"GpGp_covparams": dict(zip(g["names"], g["summary"].tolist())),
                     "fixed_effects": dict(zip(fe["names"], fe["summary"][:, :5].tolist()))},
            "reference_printed": {"GpGp_covparams": printed["GpGp_covparams"],
                                  "fixed_effects": printed["fixed_effects"]}}, indent=1))


def test_vignette_posterior_summaries(P, printed, toy):
    """Statistical parity: the vignette's workflow (3 chains, exponential
    covariance, m = 5, X_locs) on the regenerated toy data; posterior means
    within 0.6 posterior sd of Vignette.md:998-1027 (orderings and RNG streams
    differ from the reference run, so only the posterior is comparable)."""
    L = P.mcmc_nngp_initialize(toy["locs"], toy["observed_field"], X_locs=toy["X"],
                               stationary_covfun="exponential_isotropic", m=5, n_chains=3, seed=1)
    L = P.mcmc_nngp_run(L, n_cycles=5, n_iterations_update=200, n_chromatic=5, burn_in=0.5,
                        field_thinning=0.01, Gelman_Rubin_Brooks_stop=(1.0, 1.0), verbose=False)
    L = P.mcmc_nngp_run(L, n_cycles=8, n_iterations_update=100, burn_in=0.5, field_thinning=0.2,
                        Gelman_Rubin_Brooks_stop=(1.0, 1.0), verbose=False)
    est = P.mcmc_nngp_estimate(L, burn_in=0.5)
    _dump_vignette(est, printed)
    g = dict(zip(est["covariance_params"]["GpGp_covparams"]["names"],
                 est["covariance_params"]["GpGp_covparams"]["summary"]))
    ref = printed["GpGp_covparams"]
    for ours, theirs in [("scale", "scale"), ("noise_variance", "noise_variance"), ("range", "range")]:
        mean, sd = g[ours][0], ref[theirs][4]
        assert abs(mean - ref[theirs][0]) < 0.6 * sd + 0.6 * g[ours][4], (ours, mean, ref[theirs])
    fe = dict(zip(est["fixed_effects"]["names"], est["fixed_effects"]["summary"]))
    for ours, theirs in [("V1", "X$Xslope"), ("V2", "X$Xwhite_noise")]:
        mean, sd = fe[ours][0], printed["fixed_effects"][theirs][4]
        assert abs(mean - printed["fixed_effects"][theirs][0]) < 0.6 * sd + 0.6 * fe[ours][4], (ours, mean)
    for c in L["_contexts"]:
        c.close()


def test_device_records_of_the_field(P):
    """On-device records (records$field, update_Gaussian.R:305-311): rows hold
    the field at record time in location order; reserve(0) frees; rows
    outside the reservation are refused."""
    locs, NN, col, lm, y = make_problem(P, 900, 6, seed=12)
    rng = np.random.default_rng(0)
    fields = [rng.normal(size=900) for _ in range(3)]
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=2) as ctx:
        ctx.select(1)
        ctx.records_reserve(3)
        for r, f in enumerate(fields):
            ctx.set_field(f)
            ctx.record_field(r)
        np.testing.assert_array_equal(ctx.get_records(0, 3), np.stack(fields))
        np.testing.assert_array_equal(ctx.get_records(1, 1)[0], fields[1])
        with pytest.raises(P.NNGPError):
            ctx.record_field(3)
        with pytest.raises(P.NNGPError):
            ctx.select(0).record_field(0)  # chain 0 has no reservation
        ctx.select(1).records_reserve(0)
        with pytest.raises(P.NNGPError):
            ctx.get_records(0, 1)


def test_records_streamed_into_host_arrays(P):
    """nngp_records_stream: the rows recorded for two chains land in their
    bound host arrays (bitwise the device records); a row of 1.5e6 doubles
    spans several staging chunks; get_records on the bound array only waits;
    a reserve ends the binding."""
    n = 1_500_000
    rng = np.random.default_rng(3)
    locs = rng.uniform(size=(n, 2))
    NN = P.find_ordered_nn(locs, 3)
    col = P.naive_greedy_coloring(NN)
    with P.ChainContext(locs, NN, col, np.arange(1, n + 1, dtype=np.int32), rng.normal(size=n), device=0,
                        n_chains=2) as ctx:
        hosts, fields = {}, {k: [rng.normal(size=n) for _ in range(3)] for k in (0, 1)}
        for k in (0, 1):
            ctx.select(k).records_reserve(3)
            hosts[k] = np.full((3, n), np.nan)
            ctx.records_stream(hosts[k])
        for r in range(3):
            for k in (0, 1):
                ctx.select(k).set_field(fields[k][r])
                ctx.record_field(r)
        with pytest.raises(P.NNGPError):
            ctx.select(0).records_stream(np.zeros((2, n)))  # not the reserved rows: the binding stays
        assert ctx._rec_host[0] is hosts[0]
        for k in (0, 1):
            out = ctx.select(k).get_records(0, 3, out=hosts[k])
            assert out is hosts[k]
            assert k not in ctx._rec_host  # get_records on the bound array ends the binding
            np.testing.assert_array_equal(hosts[k], np.stack(fields[k]))
            np.testing.assert_array_equal(ctx.get_records(0, 3), np.stack(fields[k]))  # device path
        ctx.select(0).set_field(fields[1][0])  # after the binding: rows stay on the device
        ctx.record_field(0)
        np.testing.assert_array_equal(ctx.get_records(0, 1)[0], fields[1][0])
        np.testing.assert_array_equal(hosts[0][0], fields[0][0])
        ctx.records_stream(hosts[0])
        ctx.records_reserve(3)  # a reserve ends the binding too
        assert 0 not in ctx._rec_host
        ctx.set_field(fields[1][1])
        ctx.record_field(0)
        ctx.get_records(1, 1)
        np.testing.assert_array_equal(hosts[0][0], fields[0][0])


def test_records_bound_after_rows_were_recorded(P):
    """Rows recorded before nngp_records_stream (and rows never recorded)
    are not streamed: get_records on the bound array copies them from the
    device, so the array holds exactly what the device path returns."""
    n = 5000
    rng = np.random.default_rng(5)
    locs = rng.uniform(size=(n, 2))
    NN = P.find_ordered_nn(locs, 4)
    col = P.naive_greedy_coloring(NN)
    with P.ChainContext(locs, NN, col, np.arange(1, n + 1, dtype=np.int32), rng.normal(size=n), device=0) as ctx:
        f = [rng.normal(size=n) for _ in range(4)]
        ctx.records_reserve(4)
        ctx.set_field(f[0])
        ctx.record_field(0)  # before the binding
        host = np.full((4, n), np.nan)
        ctx.records_stream(host)
        for r in (1, 3):  # row 2 never recorded
            ctx.set_field(f[r])
            ctx.record_field(r)
        ctx.get_records(0, 4, out=host)
        dev = ctx.get_records(0, 4)
        np.testing.assert_array_equal(host, dev)
        np.testing.assert_array_equal(host[[0, 1, 3]], np.stack([f[0], f[1], f[3]]))


def test_update_records_streamed_equal_end_of_call_copy(P, toy, monkeypatch):
    """The MCMC update's field records streamed while the chains run equal the
    end-of-call copy (NNGP_RECORDS_STREAM=0) bit for bit."""
    from nngp_amd.update_gaussian import mcmc_nngp_update_Gaussian

    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("NNGP_RECORDS_STREAM", mode)
        L = P.mcmc_nngp_initialize(toy["locs"], toy["observed_field"], X_locs=toy["X"],
                                   stationary_covfun="exponential_isotropic", m=5, n_chains=2, seed=3)
        outs.append(mcmc_nngp_update_Gaussian(L["locs"], L["X"], L["observed_field"], L["space_time_model"],
                                              L["vecchia_approx"], L["states"], 8, field_thinning=0.5,
                                              n_chromatic=2, contexts=L["_contexts"], seed=1))
        for c in L["_contexts"]:
            c.close()
    for name in outs[0]:
        np.testing.assert_array_equal(outs[0][name]["records"]["field"], outs[1][name]["records"]["field"])
        np.testing.assert_array_equal(outs[0][name]["state"]["params"]["field"], outs[1][name]["state"]["params"]["field"])


def test_update_records_field_thinning(P, toy):
    """records$field rows with field_thinning = 0.5: iterations 2, 4, ...; the
    last row is the final state's field."""
    from nngp_amd.update_gaussian import mcmc_nngp_update_Gaussian

    L = P.mcmc_nngp_initialize(toy["locs"], toy["observed_field"], X_locs=toy["X"],
                               stationary_covfun="exponential_isotropic", m=5, n_chains=1, seed=3)
    out = mcmc_nngp_update_Gaussian(L["locs"], L["X"], L["observed_field"], L["space_time_model"],
                                    L["vecchia_approx"], L["states"], 6, field_thinning=0.5, n_chromatic=2,
                                    contexts=L["_contexts"], seed=1)
    rec = out["chain_1"]["records"]["field"]
    assert rec.shape == (3, L["vecchia_approx"]["n_locs"])
    np.testing.assert_array_equal(rec[-1], out["chain_1"]["state"]["params"]["field"])
    assert np.all(np.abs(rec).sum(axis=1) > 0)
    for c in L["_contexts"]:
        c.close()


def test_loglik_pair_equals_two_loglik_calls_bitwise(P, O):
    """nngp_loglik_pair_chains (the sufficient MH step's proposal and current
    log-likelihoods, update_Gaussian.R:184-186, in one pass over the rows) ==
    nngp_loglik_chains(1, ...) and nngp_loglik_chains(0, ...), bitwise, for
    every chain of a 4-chain context; the oracle's log-likelihood to 1e-10."""
    n, m, C = 20_000, 10, 4
    locs, NN, col, lm, y = make_problem(P, n, m, seed=44)
    rng = np.random.default_rng(45)
    b0, lsp, lsc = rng.normal(size=C), rng.normal(size=C) * 0.1, rng.normal(size=C) * 0.1
    res = []
    for pair in (True, False):
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            Ls = []
            for k in range(C):
                ctx.select(k)
                ctx.factor(0, "exponential_isotropic", [1.0, 0.08 + 0.01 * k, 0.0])
                ctx.factor(1, "exponential_isotropic", [1.1, 0.07 + 0.01 * k, 0.0])
                ctx.set_field(np.random.default_rng(k).normal(size=n))
                Ls.append((ctx.get_linv(1), ctx.get_linv(0), ctx.get_field()))
            if pair:
                res.append(ctx.loglik_pair_chains((1 << C) - 1, b0, lsp, lsc))
            else:
                res.append((ctx.loglik_chains(1, (1 << C) - 1, b0, lsp), ctx.loglik_chains(0, (1 << C) - 1, b0, lsc)))
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])
    for k in range(C):
        L1, L0, f = Ls[k]
        for ll, L, ls in ((res[0][0][k], L1, lsp[k]), (res[0][1][k], L0, lsc[k])):
            llo = O.loglik(L, f - b0[k], NN, ls)
            assert abs(ll - llo) <= 1e-10 * abs(llo)


def test_mh_step_calls_equal_separate_calls_bitwise(P):
    """nngp_ancillary_step_chains / nngp_sufficient_step_chains (a proposal's
    factor and its MH step behind one host sync, update_Gaussian.R:123-131 and
    :179-186) == the separate calls they replace, bitwise, chain by chain; a
    chain whose proposal factor is not positive definite (two coinciding
    points, no nugget) reports NNGP_ERR_CHOL and NaN results without
    disturbing the other chains, and a later step of that chain is exact."""
    from nngp_amd._lib import NNGP_ERR_CHOL

    n, m, C = 6000, 10, 3
    locs, NN, col, lm, y = make_problem(P, n, m, seed=46)
    locs = locs.copy()
    k0 = 500
    locs[k0] = locs[NN[k0, 1] - 1]  # row k0 coincides with its first neighbour
    rng = np.random.default_rng(47)
    b0, dls, lnv = rng.normal(size=C) * 0.1, rng.normal(size=C) * 0.1, rng.normal(size=C) * 0.1 - 1.0
    lsp, lsc = rng.normal(size=C) * 0.1, rng.normal(size=C) * 0.1
    cur = [[1.0, 0.08 + 0.01 * k, 0.1] for k in range(C)]
    prop = np.array([[1.1, 0.07 + 0.01 * k, 0.0 if k == 1 else 0.05] for k in range(C)])  # chain 1 fails
    mask = (1 << C) - 1

    def setup(ctx):
        for k in range(C):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", cur[k])
            ctx.set_field(np.random.default_rng(k).normal(size=n))
            ctx.set_mu(None, b0[k])

    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        setup(ctx)
        st_a, ratio = ctx.ancillary_step_chains(mask, "exponential_isotropic", prop, b0, dls, lnv)
        props = []
        for k in range(C):
            ctx.select(k)
            if st_a[k] == 0:
                ctx.accept_field()
            props.append(ctx.get_field())
        st_s, lp, lc = ctx.sufficient_step_chains(mask, "exponential_isotropic", prop, b0, lsp, lsc)
        st_s2, lp2, lc2 = ctx.sufficient_step_chains(2, "exponential_isotropic", prop * [1, 1, 0] + [0, 0, 0.05], b0,
                                                     lsp, lsc)
    with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
        setup(ctx)
        st = ctx.factor_chains(1, mask, "exponential_isotropic", prop)
        ok = (1 << 0) | (1 << 2)
        ctx.ancillary_propose_chains(ok, b0, dls)
        ratio_ref = ctx.field_response_ratio_chains(ok, b0, lnv)
        props_ref = []
        for k in range(C):
            ctx.select(k)
            if st[k] == 0:
                ctx.accept_field()
            props_ref.append(ctx.get_field())
        st2 = ctx.factor_chains(1, mask, "exponential_isotropic", prop)
        lp_ref, lc_ref = ctx.loglik_pair_chains(ok, b0, lsp, lsc)
        ctx.factor_chains(1, 2, "exponential_isotropic", prop * [1, 1, 0] + [0, 0, 0.05])
        lp2_ref, lc2_ref = ctx.loglik_pair_chains(2, b0, lsp, lsc)
    assert list(st) == list(st_a) == list(st2) == list(st_s) == [0, NNGP_ERR_CHOL, 0], (st, st_a, st_s)
    assert np.isnan(ratio[1]) and np.isnan(lp[1]) and np.isnan(lc[1])
    for k in (0, 2):
        assert ratio[k] == ratio_ref[k] and lp[k] == lp_ref[k] and lc[k] == lc_ref[k], k
        np.testing.assert_array_equal(props[k], props_ref[k])
    np.testing.assert_array_equal(props[1], props_ref[1])  # the failed chain kept its field
    assert st_s2[1] == 0 and lp2[1] == lp2_ref[1] and lc2[1] == lc2_ref[1]


@pytest.mark.parametrize("m,covfun", [(5, "exponential_isotropic"), (10, "matern15_isotropic"),
                                      (15, "matern15_isotropic"), (20, "exponential_isotropic"),
                                      (15, "matern_isotropic")])
def test_factor_jobs_launch_equals_chain_by_chain(P, m, covfun, monkeypatch):
    """factor_chains of several chains in one scaled-coordinate and one factor
    launch (launch_factor_jobs) gives every chain's Linv and failure flag
    bitwise as the chain-by-chain launches (NNGP_FACTOR_JOBS=0), including a
    chain whose proposal is not positive definite and a chain not in the mask."""
    from nngp_amd._lib import NNGP_ERR_CHOL

    n, C = 3000, 4
    locs, NN, col, lm, y = make_problem(P, n, m, seed=21)
    if covfun == "matern_isotropic":
        cps = [[1.0, 0.05, 1.2, 0.0], [1.3, 0.04, 1.2, 0.1], [0.8, 0.07, 1.2, 0.0], [1.0, 0.05, 1.2, 0.0]]
    else:
        cps = [[1.0, 0.05, 0.0], [1.3, 0.04, 0.1], [0.8, 0.07, 0.0], [1.0, 0.05, 0.0]]
    bad = list(cps[2])
    bad[-1] = -2.0  # nugget -2: diagonal 1 + nugget < 0, not positive definite
    outs = []
    for mode in ("1", "0"):
        monkeypatch.setenv("NNGP_FACTOR_JOBS", mode)
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            st = ctx.factor_chains(1, 0b1011, covfun, np.array(cps))
            linv = [ctx.select(k).get_linv(1) for k in (0, 1, 3)]
            st2 = ctx.factor_chains(1, 0b0110, covfun, np.array([cps[0], cps[1], bad, cps[3]]))
            linv.append(ctx.select(1).get_linv(1))
            outs.append((list(st), list(st2), linv))
    assert outs[0][0] == outs[1][0] == [0, 0, 0, 0]
    assert outs[0][1] == outs[1][1] and outs[0][1][2] == NNGP_ERR_CHOL and outs[0][1][1] == 0
    for a, b in zip(outs[0][2], outs[1][2]):
        np.testing.assert_array_equal(a, b)
