"""CPU ORACLE of one chain of mcmc_nngp_update_Gaussian -- test infrastructure.

Restates Scripts/mcmc_nngp_update_Gaussian.R:27-316 with the C oracle's
kernels (vecchia_Linv, Linv_mult, triangular solve, masked chromatic sweep)
and dense numpy algebra, consuming a numpy Generator in the reference's draw
order (which the product's host mirror also follows), so that a device run
and this oracle run from the same state and seed can be compared
iteration-by-iteration.  The chromatic sweep uses the same Philox stream as
the device (key, counter) -- see oracle.or_normal.
"""
from __future__ import annotations

import numpy as np
from scipy.stats import norm

import oracle as O


def _plogis(x):
    return 1.0 / (1.0 + np.exp(-x))


def _covparms(sp, shape):
    out = [1.0]
    for nm, v in zip(sp, np.atleast_1d(shape)):
        out.append(float(np.exp(v)) if nm.startswith("log") else float(0.5 + 0.5 * _plogis(v)))
    return out + [0.0]


def run_chain(i, state, locs, NN, coloring, X, y, space_time_model, va, n_iterations_update,
              field_thinning, n_chromatic, iter_start, key):
    rng = np.random.default_rng(int(iter_start) + i + 1)
    covfun = space_time_model["covfun"]["stationary_covfun"]
    sp = space_time_model["covfun"]["shape_params"]
    p = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in state["params"].items()}
    tk = {k: dict(v) for k, v in state["transition_kernels"].items()}
    n = va["n_locs"]
    n_obs = va["n_obs"]
    lm = va["locs_match"]
    opl = va["obs_per_loc"].astype(np.int32)
    var_y = float(np.var(y, ddof=1))
    has_X = X.get("X") is not None
    has_locs = has_X and len(X["locs"]) > 0
    n_shape = len(sp)
    recs = {"beta_0": [], "log_scale": [], "log_noise_variance": [], "shape": [], "field": [], "beta": []}
    acc_a = np.zeros(n_iterations_update)
    acc_s = np.zeros(n_iterations_update)
    L = O.vecchia_linv(covfun, _covparms(sp, p["shape"]), locs, NN)
    D = O.precision_diag(L, NN)
    field = np.array(p["field"], np.float64)

    def Bmul(Lm, x):
        return O.linv_mult(Lm, x, NN)

    def interweave(Lm):
        Xl = X["X"][va["hctam_scol_1"] - 1][:, X["locs"]]
        M = np.column_stack([np.ones(n), Xl])
        SX = np.column_stack([Bmul(Lm, M[:, k]) for k in range(M.shape[1])])
        cov = np.linalg.inv(SX.T @ SX)
        return {"Xl": Xl, "SX": SX, "covmat": cov, "chol": np.linalg.cholesky(cov).T}

    iw = interweave(L) if has_locs else None
    mu = (p["beta_0"] + X["X"] @ p["beta"]) if has_X else np.full(n_obs, p["beta_0"])
    adapt = 0 <= iter_start <= 2000
    for it in range(1, n_iterations_update + 1):
        # ancillary
        innov = rng.normal(0.0, np.exp(0.5 * tk["covariance_params_ancillary"]["logvar"]), n_shape + 1)
        new_ls = p["log_scale"] + innov[0]
        new_shape = p["shape"] + innov[1:]
        Ln = O.vecchia_linv(covfun, _covparms(sp, new_shape), locs, NN)
        new_field = p["beta_0"] + np.exp(0.5 * (new_ls - p["log_scale"])) * O.tri_solve(
            Ln, NN, Bmul(L, field - p["beta_0"]))
        sd = np.exp(0.5 * p["log_noise_variance"])
        ratio = np.sum(norm.logpdf(y, new_field[lm - 1] + mu - p["beta_0"], sd)
                       - norm.logpdf(y, field[lm - 1] + mu - p["beta_0"], sd))
        if ratio > np.log(rng.uniform()):
            p["shape"], p["log_scale"], field = new_shape, new_ls, new_field
            L, D = Ln, O.precision_diag(Ln, NN)
            acc_a[it - 1] = 1
            if has_locs:
                iw = interweave(L)
        if adapt and it % 25 == 0:
            a = acc_a[it - 25:it].mean()
            if a < 0.05:
                tk["covariance_params_ancillary"]["logvar"] -= rng.normal(0.4, 0.05)
            if a > 0.15:
                tk["covariance_params_ancillary"]["logvar"] += rng.normal(0.4, 0.05)
        # sufficient
        innov = rng.normal(0.0, np.exp(0.5 * tk["covariance_params_sufficient"]["logvar"]), n_shape + 1)
        new_ls = p["log_scale"] + innov[0]
        if np.exp(new_ls) < var_y:
            new_shape = p["shape"] + innov[1:]
            Ln = O.vecchia_linv(covfun, _covparms(sp, new_shape), locs, NN)
            gp = (O.loglik(Ln, field - p["beta_0"], NN, new_ls)
                  - O.loglik(L, field - p["beta_0"], NN, p["log_scale"]))
            if gp > np.log(rng.uniform()):
                p["shape"], p["log_scale"] = new_shape, new_ls
                L, D = Ln, O.precision_diag(Ln, NN)
                acc_s[it - 1] = 1
                if has_locs:
                    iw = interweave(L)
        if adapt and it % 25 == 0:
            a = acc_s[it - 25:it].mean()
            if a < 0.05:
                tk["covariance_params_sufficient"]["logvar"] -= rng.normal(0.2, 0.05)
            if a > 0.15:
                tk["covariance_params_sufficient"]["logvar"] += rng.normal(0.2, 0.05)
        # field mean
        if (not has_locs) or (not has_X):
            u1 = Bmul(L, np.ones(n))
            uf = Bmul(L, field)
            bc = np.exp(p["log_scale"]) / (u1 @ u1)
            bm = np.exp(-p["log_scale"]) * (uf @ u1) * bc
            p["beta_0"] = float(bm + np.sqrt(bc) * rng.normal())
        if has_X:
            X1 = np.column_stack([np.ones(n_obs), X["X"]])
            resid = y - field[lm - 1] + p["beta_0"]
            bm = (resid @ X1) @ X["solve_1XT1X"]
            innov = bm + np.exp(0.5 * p["log_noise_variance"]) * (X["chol_solve_1XT1X"].T @ rng.normal(size=X1.shape[1]))
            field = field - p["beta_0"] + innov[0]
            p["beta_0"] = float(innov[0])
            p["beta"] = innov[1:].copy()
            if has_locs:
                lc = X["locs"]
                other = field + iw["Xl"] @ p["beta"][lc]
                bm = iw["covmat"] @ (Bmul(L, other) @ iw["SX"])
                innov = bm + np.exp(0.5 * p["log_scale"]) * (iw["chol"].T @ rng.normal(size=len(lc) + 1))
                p["beta_0"] = float(innov[0])
                p["beta"][lc] = innov[1:]
                field = other - iw["Xl"] @ p["beta"][lc]
        mu = (p["beta_0"] + X["X"] @ p["beta"]) if has_X else np.full(n_obs, p["beta_0"])
        # chromatic sweeps with the device's Philox stream
        z = O.sweep_normals(key, (int(iter_start) + it - 1) * n_chromatic, n_chromatic, n)
        field = O.sweep("masked", field, L, NN, coloring, D, opl, y, mu, lm, p["beta_0"], p["log_scale"],
                        p["log_noise_variance"], z)
        # noise variance
        ssr = float(np.sum((y - field[lm - 1] - mu + p["beta_0"]) ** 2))
        for _ in range(10):
            innov = rng.normal(0.0, 0.01)
            if np.exp(p["log_noise_variance"] + innov) < var_y:
                lnv = p["log_noise_variance"]
                if -0.5 * n_obs * innov - 0.5 * ssr * (np.exp(-lnv - innov) - np.exp(-lnv)) > np.log(rng.uniform()):
                    p["log_noise_variance"] = lnv + innov
        recs["beta_0"].append(p["beta_0"])
        recs["log_scale"].append(p["log_scale"])
        recs["log_noise_variance"].append(p["log_noise_variance"])
        recs["shape"].append(np.array(p["shape"]))
        if has_X:
            recs["beta"].append(p["beta"].copy())
        if round(it * field_thinning) == it * field_thinning:
            recs["field"].append(field.copy())
    p["field"] = field
    return {"params": p, "transition_kernels": tk, "records": recs,
            "acceptance": {"ancillary": acc_a, "sufficient": acc_s}}
