"""mcmc_nngp_estimate -- host mirror of Scripts/mcmc_nngp_estimate.R:1-96
(posterior summaries; out of the kernel scope, kept for statistical parity)."""
from __future__ import annotations

import numpy as np

SUMMARY_COLS = ["mean", "q0.025", "median", "q0.975", "sd"]


def _quantile7(x, q):
    return np.quantile(x, q, axis=0)  # numpy 'linear' == R type 7


def get_summary(samples):
    """estimate.R:1-6: mean, q0.025, median, q0.975, sd per column."""
    s = np.atleast_2d(np.asarray(samples, np.float64))
    if s.shape[0] == 1 and s.ndim == 2 and s.shape[1] > 1 and np.asarray(samples).ndim == 1:
        s = s.T
    return np.column_stack([s.mean(0), _quantile7(s, 0.025), _quantile7(s, 0.5), _quantile7(s, 0.975),
                            s.std(0, ddof=1)])


def _plogis(x):
    return 1 / (1 + np.exp(-x))


def mcmc_nngp_estimate(mcmc_nngp_list, burn_in=0.5):
    L = mcmc_nngp_list
    recs = L["records"]
    first = next(iter(recs.values()))
    it = int(first["iterations"][-1, 0])
    lo = int(burn_in * it) - 1
    res = {"covariance_params": {}}
    sp = L["space_time_model"]["covfun"]["shape_params"]
    names = ["log_scale", "log_noise_variance"] + list(sp)
    samples = np.vstack([np.column_stack([c["params"]["log_scale"], c["params"]["log_noise_variance"],
                                          c["params"]["shape"]])[lo:it] for c in recs.values()])
    res["covariance_params"]["sampled_covparams"] = {"names": names, "summary": get_summary(samples)}
    g = samples.copy()
    gnames = []
    for j, nm in enumerate(names):
        if nm.startswith("log_"):
            g[:, j] = np.exp(g[:, j])
            gnames.append(nm[4:])
        elif nm.startswith("qlogis_"):
            g[:, j] = 1.5 * _plogis(g[:, j])
            gnames.append(nm[7:])
        else:
            gnames.append(nm)
    res["covariance_params"]["GpGp_covparams"] = {"names": gnames, "summary": get_summary(g)}
    inla = g.copy()
    inames = list(gnames)
    covfun = L["space_time_model"]["covfun"]["stationary_covfun"]
    keep = np.ones(len(inames), bool)
    if "exponential" in covfun:
        for j, nm in enumerate(inames):
            if "range" in nm:
                inla[:, j] *= 2
    if "matern" in covfun and covfun != "matern15_isotropic":
        sm = [j for j, nm in enumerate(inames) if "smoothness" in nm][0]
        for j, nm in enumerate(inames):
            if "range" in nm:
                inla[:, j] *= np.sqrt(8 * inla[:, sm])
        keep[sm] = False
    for j, nm in enumerate(inames):
        if "noise" in nm:
            inla[:, j] = 1 / inla[:, j]
            inames[j] = "precision_of_Gaussian_obs"
        elif "scale" in nm:
            inla[:, j] = np.sqrt(inla[:, j])
            inames[j] = "sd_for_spatial"
    res["covariance_params"]["INLA_covparams"] = {"names": [n for n, k in zip(inames, keep) if k],
                                                  "summary": get_summary(inla[:, keep])}
    # fixed effects (estimate.R:76-87)
    fx = []
    for c in recs.values():
        b = [c["params"]["beta_0"]]
        if "beta" in c["params"]:
            b.append(c["params"]["beta"])
        out = np.column_stack(b)[lo:it].copy()
        if out.shape[1] > 1:
            out[:, 0] = out[:, 0] - out[:, 1:] @ L["X"]["X_mean"]
        fx.append(out)
    fx = np.vstack(fx)
    fe = get_summary(fx)
    zero_out = (np.sign(fe[:, 1]) * np.sign(fe[:, 3])) > 0
    res["fixed_effects"] = {"names": ["beta_0"] + list(L["X"].get("names", [])),
                            "summary": np.column_stack([fe, zero_out])}
    # field (estimate.R:89-96): centered field samples after burn-in
    fs = []
    saved = first["saved_field"]
    sel = saved > it * burn_in
    for c in recs.values():
        f = c["params"]["field"][sel]
        b0 = c["params"]["beta_0"][saved[sel].astype(int) - 1, 0]
        fs.append(f - b0[:, None])
    res["field"] = get_summary(np.vstack(fs))
    return res
