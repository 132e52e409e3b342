"""mcmc_nngp_initialize -- host mirror of Scripts/mcmc_nngp_initialize.R:1-240.

Same arguments and the same returned structure (a dict standing for the R
list).  The array work (ordering, NNarray, colouring, the initial Vecchia
field draw) runs through the C ABI; the regression set-up is host numpy.
Random draws use numpy's PCG64 seeded with ``seed`` (R's Mersenne-Twister
stream is not reproduced: parity is statistical for the MCMC).
"""
from __future__ import annotations

import time

import numpy as np

from .context import make_chain_views
from .graph import find_ordered_nn, naive_greedy_coloring, order_maxmin, sparse_chol_indices
from .model import covparms, shape_params_of


def _lonlat_xyz(locs):
    lon, lat = np.radians(locs[:, 0]), np.radians(locs[:, 1])
    return np.column_stack([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)])


def _reorder(locs, reordering, stationary_covfun, rng):
    kind = reordering[0] if isinstance(reordering, (list, tuple)) else reordering
    lonlat = "sphere" in stationary_covfun
    geo = _lonlat_xyz(locs) if lonlat else locs
    if kind == "maxmin":
        return order_maxmin(geo) - 1
    if kind == "random":
        return rng.permutation(len(locs))
    if kind == "coord":
        return np.argsort(locs[:, int(reordering[1]) - 1], kind="stable")
    if kind == "dist_to_point":
        p = np.asarray(reordering[1], np.float64)
        p = _lonlat_xyz(p[None, :])[0] if lonlat else p
        return np.argsort(((geo - p) ** 2).sum(1), kind="stable")
    if kind == "middleout":
        return np.argsort(((geo - geo.mean(0)) ** 2).sum(1), kind="stable")
    raise ValueError(f"unknown reordering {reordering!r}")


def _model_matrix(df):
    """model.matrix(~., df)[, -1] with treatment contrasts (numeric columns kept,
    factors expanded dropping their first level)."""
    import pandas as pd

    if isinstance(df, np.ndarray):
        df = pd.DataFrame(df, columns=[f"V{k + 1}" for k in range(df.shape[1])])
    cols, names = [], []
    for c in df.columns:
        s = df[c]
        if s.dtype.kind in "if" or s.dtype.kind == "b":
            cols.append(np.asarray(s, np.float64))
            names.append(str(c))
        else:
            # a pandas Categorical keeps its level order (R's `levels`
            # attribute); other columns become factors with sorted levels
            cat = s.array if isinstance(s.dtype, pd.CategoricalDtype) else pd.Categorical(s)
            for lev in cat.categories[1:]:
                cols.append((cat == lev).astype(np.float64))
                names.append(f"{c}{lev}")
    return np.column_stack(cols) if cols else np.zeros((len(df), 0)), names


def _ncol(x):
    if x is None:
        return 0
    return x.shape[1]


def mcmc_nngp_initialize(observed_locs, observed_field, X_obs=None, X_locs=None, m: int = 10,
                         reordering="maxmin", stationary_covfun: str = "exponential_isotropic",
                         response_model: str = "Gaussian", n_chains: int = 3, seed: int = 1,
                         devices=None, build_adjacency: bool | None = None):
    t_begin = time.time()
    rng = np.random.default_rng(seed)
    observed_locs = np.asarray(observed_locs, np.float64)
    if observed_locs.ndim == 1:
        observed_locs = observed_locs[:, None]
    observed_field = np.asarray(observed_field, np.float64)
    n_obs = len(observed_field)

    # ---- dedup + reordering (initialize.R:26-36)
    _, first = np.unique(observed_locs, axis=0, return_index=True)
    locs = observed_locs[np.sort(first)]
    perm = _reorder(locs, reordering, stationary_covfun, rng)
    locs = np.ascontiguousarray(locs[perm])
    n = locs.shape[0]

    space_time_model = {"response_model": response_model,
                        "covfun": {"stationary_covfun": stationary_covfun,
                                   "shape_params": shape_params_of(stationary_covfun, locs.shape[1])}}

    # ---- Vecchia approximation (initialize.R:80-110)
    va = {"n_locs": n, "n_obs": n_obs}
    key = {tuple(r): i + 1 for i, r in enumerate(locs)}
    locs_match = np.array([key[tuple(r)] for r in observed_locs], np.int32)
    va["locs_match"] = locs_match
    order = np.argsort(locs_match, kind="stable")
    counts = np.bincount(locs_match, minlength=n + 1)[1:]
    splits = np.split(order + 1, np.cumsum(counts)[:-1])
    va["hctam_scol"] = splits
    va["hctam_scol_1"] = np.array([s[0] for s in splits], np.int32)
    va["obs_per_loc"] = counts.astype(np.int32)
    NNarray = find_ordered_nn(locs, m)  # Euclidean on raw coordinates (reference quirk)
    va["NNarray"] = NNarray
    non_na, row_idx, col_idx = sparse_chol_indices(NNarray)
    va["NNarray_non_NA"] = non_na
    va["sparse_chol_column_idx"] = col_idx
    va["sparse_chol_row_idx"] = row_idx
    if build_adjacency is None:
        build_adjacency = n <= 200_000
    if build_adjacency:
        import scipy.sparse as sp

        B = sp.csc_matrix((np.ones(len(row_idx)), (row_idx - 1, col_idx - 1)), shape=(n, n))
        M = (B.T @ B).tocsc()
        M.data[:] = 1.0
        va["MRF_adjacency_mat"] = M
    va["coloring"] = naive_greedy_coloring(NNarray)

    # ---- regressors (initialize.R:116-137)
    X = {"arg": {"X_locs": X_locs, "X_obs": X_obs}, "X": None, "locs": np.zeros(0, np.int64)}
    parts, names = [], []
    for part in (X_locs, X_obs):
        if part is not None:
            mm, nm = _model_matrix(part)
            parts.append(mm)
            names += nm
    if parts:
        XX = np.column_stack(parts)
        X["names"] = names
        X["locs"] = np.arange(_ncol(np.asarray(X_locs) if X_locs is not None else None))  # seq(ncol(X_locs)), 0-based
        X["X_mean"] = XX.mean(0)
        XX = XX - X["X_mean"]
        X["X"] = XX
        X["solve_XTX"] = np.linalg.inv(XX.T @ XX)
        X["chol_solve_XTX"] = np.linalg.cholesky(X["solve_XTX"]).T  # R chol(): upper
        X1 = np.column_stack([np.ones(n_obs), XX])
        X["solve_1XT1X"] = np.linalg.inv(X1.T @ X1)
        X["chol_solve_1XT1X"] = np.linalg.cholesky(X["solve_1XT1X"]).T

    # ---- chain states (initialize.R:143-209)
    sp_names = space_time_model["covfun"]["shape_params"]
    d100 = locs[: min(100, n)]
    diam = np.sqrt(((d100[:, None, :] - d100[None, :, :]) ** 2).sum(-1)).max() if len(d100) > 1 else 1.0

    def log_range_start(cols=None):
        sub = d100 if cols is None else d100[:, cols]
        dm = np.sqrt(((sub[:, None, :] - sub[None, :, :]) ** 2).sum(-1)).max() if len(sub) > 1 else diam
        return float(rng.choice(np.log(max(dm, 1e-300)) - np.log(np.arange(20, 201))))

    Xd = X["X"]
    design = np.column_stack([np.ones(n_obs)] + ([Xd] if Xd is not None else []))
    coef, *_ = np.linalg.lstsq(design, observed_field, rcond=None)
    resid = observed_field - design @ coef
    p = design.shape[1]
    sigma2 = resid @ resid / max(n_obs - p, 1)
    vcov = sigma2 * np.linalg.inv(design.T @ design)
    var_resid = np.var(resid, ddof=1)

    if devices is None:
        devices = [-1]
    contexts = make_chain_views(locs, NNarray, va["coloring"], locs_match, observed_field, n_chains, devices)
    states = {}
    for i in range(n_chains):
        st = {"params": {}, "transition_kernels": {}}
        f = stationary_covfun
        if f in ("exponential_isotropic", "exponential_sphere", "matern15_isotropic"):
            shape = [log_range_start()]
        elif f == "exponential_scaledim":
            shape = [log_range_start([k]) for k in range(locs.shape[1])]
        elif f == "exponential_spacetime":
            shape = [log_range_start(list(range(locs.shape[1] - 1))), log_range_start([locs.shape[1] - 1])]
        elif f in ("matern_isotropic", "matern_sphere"):
            shape = [log_range_start(), float(rng.normal())]
        elif f == "matern_scaledim":
            shape = [log_range_start([k]) for k in range(locs.shape[1])] + [float(rng.normal())]
        else:  # matern_spacetime
            shape = [log_range_start(list(range(locs.shape[1] - 1))), log_range_start([locs.shape[1] - 1]),
                     float(rng.normal())]
        st["params"]["shape"] = np.array(shape)
        st["transition_kernels"] = {"covariance_params_sufficient": {"logvar": -2.0},
                                    "covariance_params_ancillary": {"logvar": -2.0},
                                    "log_noise_variance": {"logvar": -1.0}}
        perturb = np.linalg.cholesky(vcov) @ rng.normal(size=p)
        st["params"]["beta_0"] = float(coef[0] + perturb[0])
        st["params"]["beta"] = (coef[1:] + perturb[1:]) if Xd is not None else None
        st["params"]["log_scale"] = float(np.log(rng.beta(10, 10) * var_resid))
        st["params"]["log_noise_variance"] = float(np.log(rng.beta(10, 10) * var_resid))
        ctx = contexts[i]
        ctx.factor(0, stationary_covfun, covparms(sp_names, st["params"]["shape"], 0.4, 0.7))
        w = ctx.tri_solve(0, rng.normal(size=n))
        st["params"]["field"] = st["params"]["beta_0"] + np.sqrt(np.exp(st["params"]["log_scale"])) * w
        states[f"chain_{i + 1}"] = st

    records = {f"chain_{i + 1}": {"iterations": np.array([[0.0, time.time() - t_begin]]), "params": {}}
               for i in range(n_chains)}
    print(f"Setup done, {time.time() - t_begin} s elapsed")
    return {"locs": locs, "X": X, "observed_field": observed_field, "observed_locs": observed_locs,
            "space_time_model": space_time_model, "vecchia_approx": va, "states": states,
            "records": records, "diagnostics": {"Gelman_Rubin_Brooks": [], "ESS": []},
            "t_begin": t_begin, "seed": seed, "_contexts": contexts}
