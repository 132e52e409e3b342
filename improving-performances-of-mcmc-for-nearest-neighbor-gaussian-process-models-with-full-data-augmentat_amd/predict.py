"""mcmc_nngp_predict_field / mcmc_nngp_predict_fixed_effects -- host mirror of
Scripts/mcmc_nngp_predict.R:1-104 ("next").

Per saved sample the field is predicted with the device factor build on the
stacked locations and the device sparse triangular solve
(predict.R:39-53): sd * B^{-1} c(B11 (w/sd), z).
"""
from __future__ import annotations

import numpy as np

from .context import ChainContext
from .estimate import get_summary
from .graph import find_ordered_nn, naive_greedy_coloring
from .model import covparms


def mcmc_nngp_predict_field(mcmc_nngp_list, predicted_locs, burn_in=0.5, n_cores=1, m=10, seed=1,
                            device=-1, z_new=None):
    """predict.R:1-60.  ``z_new`` (optional) replaces the rnorm draws of the
    new locations (predict.R:50): z_new[k][i] = the normals of chain k's i-th
    prediction; by default they come from numpy's generator seeded ``seed``."""
    L = mcmc_nngp_list
    locs = L["locs"]
    predicted_locs = np.asarray(predicted_locs, np.float64)
    allloc = np.vstack([locs, predicted_locs])
    NN = find_ordered_nn(allloc, m)
    N, n = allloc.shape[0], locs.shape[0]
    ctx = ChainContext(allloc, NN, naive_greedy_coloring(NN), np.arange(1, N + 1, dtype=np.int32),
                       np.zeros(N), device=device)
    covfun = L["space_time_model"]["covfun"]["stationary_covfun"]
    sp = L["space_time_model"]["covfun"]["shape_params"]
    first = next(iter(L["records"].values()))
    stored = first["saved_field"]
    stored = stored[stored > burn_in * stored.max()].astype(int)
    rng = np.random.default_rng(seed)
    out = []
    for kc, chain in enumerate(L["records"].values()):
        shapes = chain["params"]["shape"][stored - 1]
        _, first_idx = np.unique(shapes, axis=0, return_index=True)
        need = np.zeros(len(stored), bool)
        need[first_idx] = True  # !duplicated(shape[stored_idx, ])
        samples = np.zeros((len(stored), predicted_locs.shape[0]))
        for k, i_chain in enumerate(stored):
            i_field = int(np.nonzero(chain["saved_field"] == i_chain)[0][0]) if "saved_field" in chain \
                else int(np.nonzero(first["saved_field"] == i_chain)[0][0])
            if need[k] or k == 0:
                ctx.factor(0, covfun, covparms(sp, chain["params"]["shape"][i_chain - 1], 0.0, 1.5))
            sd = np.exp(0.5 * chain["params"]["log_scale"][i_chain - 1, 0])
            w = chain["params"]["field"][i_field] - chain["params"]["beta_0"][i_chain - 1, 0]
            u = ctx.spmv(0, np.concatenate([w, np.zeros(N - n)]))[:n]
            z = rng.normal(size=N - n) if z_new is None else np.asarray(z_new[kc][k], np.float64)
            x = ctx.tri_solve(0, np.concatenate([u / sd, z]))
            samples[k] = sd * x[n:]
        out.append(samples)
    ctx.close()
    allsamp = np.vstack(out)
    return {"predicted_locs": predicted_locs, "predicted_field_samples": out,
            "predicted_field_summary": get_summary(allsamp)}


def mcmc_nngp_predict_fixed_effects(mcmc_nngp_list, X_predicted, burn_in=0.5, n_cores=1,
                                    match_field_thinning=True, add_intercept=False):
    from .initialize import _model_matrix

    L = mcmc_nngp_list
    first = next(iter(L["records"].values()))
    stored = first["saved_field"] if match_field_thinning else np.arange(1, int(first["iterations"][-1, 0]) + 1)
    stored = stored[stored > burn_in * stored.max()].astype(int)
    mm, names = _model_matrix(X_predicted)
    mm = np.column_stack([np.ones(len(mm)), mm])
    names = ["beta_0"] + names
    if not add_intercept:
        mm, names = mm[:, 1:], names[1:]
    allnames = ["beta_0"] + list(L["X"].get("names", []))
    subset = [allnames.index(nm) for nm in names]
    out = []
    for kc, chain in enumerate(L["records"].values()):
        bm = np.column_stack([chain["params"]["beta_0"]] + ([chain["params"]["beta"]] if "beta" in chain["params"] else []))
        bm = bm[stored - 1].copy()
        if bm.shape[1] > 1:
            bm[:, 0] = bm[:, 0] - bm[:, 1:] @ L["X"]["X_mean"]
        out.append(bm[:, subset] @ mm.T)
    return {"X_predicted": X_predicted, "predicted_fixed_effects_samples": out,
            "predicted_fixed_effects_summary": get_summary(np.vstack(out))}
