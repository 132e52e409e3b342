"""Convergence diagnostics used by the run loop's stop rule
(Scripts/mcmc_nngp_diagnose.R:1-24 Gelman_Rubin_Brooks, :107-118 ESS).

Out of the hot-path scope; restated here only so that
``mcmc_nngp_run``'s early-stop logic (run.R:38-46) behaves like the
reference.  ESS uses an AR(p)-spectral estimate at frequency 0 in the spirit
of coda::effectiveSize (coda is not available: not parity-checked).
"""
from __future__ import annotations

import numpy as np


def _samples(records, burn_in, n=None):
    out = []
    for chain in records.values():
        p = chain["params"]
        nn = n if n is not None else p["beta_0"].shape[0]
        start = max(int(burn_in * nn) - 1, 0)
        cols, names = [], []
        for k, v in p.items():
            if k == "field":
                continue
            v = np.asarray(v)
            v = v[:, None] if v.ndim == 1 else v
            cols.append(v[start:nn])
            names += [k] if v.shape[1] == 1 else [f"{k}{j + 1}" for j in range(v.shape[1])]
        out.append(np.column_stack(cols))
    return out, names


def Gelman_Rubin_Brooks(records, burn_in=0.5, n=None):
    samples, names = _samples(records, burn_in, n)
    n = n if n is not None else next(iter(records.values()))["params"]["beta_0"].shape[0]
    m = len(samples)
    W = sum(np.atleast_2d(np.cov(s, rowvar=False)) for s in samples) / m
    means = np.array([s.mean(0) for s in samples])
    Bv = np.atleast_2d(np.cov(means, rowvar=False))
    try:
        ev = np.linalg.svd(np.linalg.solve(W, Bv), compute_uv=False)[0]
    except np.linalg.LinAlgError:
        ev = np.inf
    mpsrf = (n - 1) / n + (m + 1) / m * ev
    ind = ((m + 1) / m) * ((n - 1) / n) * (np.diag(Bv) / np.diag(W)) + (n + 1) / n
    return {"R_hat": np.concatenate([[mpsrf], ind]), "names": ["Multivariate"] + names,
            "within_variance": W}


def _ess_1d(x, max_order=None):
    x = np.asarray(x, np.float64)
    n = len(x)
    if n < 4 or np.var(x) == 0:
        return float(n)
    x = x - x.mean()
    max_order = max_order or min(n - 1, int(10 * np.log10(n)))
    acf = np.array([x[: n - k] @ x[k:] / n for k in range(max_order + 1)])
    best = (np.inf, 0, acf[0])
    # Levinson-Durbin, AIC order selection (as stats::ar.yw)
    phi = np.zeros(0)
    v = acf[0]
    aic0 = n * np.log(v)
    best = (aic0, phi.copy(), v)
    for k in range(1, max_order + 1):
        kk = (acf[k] - (phi @ acf[1:k][::-1] if k > 1 else 0.0)) / v
        phi = np.concatenate([phi - kk * phi[::-1], [kk]])
        v = v * (1 - kk * kk)
        if v <= 0:
            break
        aic = n * np.log(v) + 2 * k
        if aic < best[0]:
            best = (aic, phi.copy(), v)
    _, phi, v = best
    spec0 = v / (1 - phi.sum()) ** 2
    return float(n * acf[0] / spec0) if spec0 > 0 else float(n)


def ESS(records, burn_in=0.5):
    samples, names = _samples(records, burn_in)
    E = np.array([[_ess_1d(s[:, j]) for j in range(s.shape[1])] for s in samples])
    return np.vstack([E, E.sum(0)]), names
