"""Covariance-model metadata of the reference (Scripts/mcmc_nngp_initialize.R:62-69)
and the shape-parameter transforms used by the MCMC
(Scripts/mcmc_nngp_update_Gaussian.R:67-71,118-122,174-178)."""
from __future__ import annotations

import numpy as np


def shape_params_of(stationary_covfun: str, d: int):
    """initialize.R:62-69 (+ the GpGp-named matern15_isotropic extension)."""
    f = stationary_covfun
    if f in ("exponential_isotropic", "exponential_sphere", "matern15_isotropic"):
        return ["log_range"]
    if f == "exponential_scaledim":
        return [f"log_range_{k + 1}" for k in range(d)]
    if f == "exponential_spacetime":
        return ["log_range_1", "log_range_2"]
    if f in ("matern_isotropic", "matern_sphere"):
        return ["log_range", "qlogis_smoothness"]
    if f == "matern_scaledim":
        return [f"log_range_{k + 1}" for k in range(d)] + ["qlogis_smoothness"]
    if f == "matern_spacetime":
        return ["log_range_1", "log_range_2", "qlogis_smoothness"]
    raise ValueError(f"unknown stationary_covfun {stationary_covfun!r}")


def plogis(x):
    return 1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))


def transform_shape(shape_params, shape, smooth_lo=0.5, smooth_span=0.5):
    """exp() for log_* parameters, lo + span * plogis() for qlogis_* ones.
    MCMC: (.5, .5) (update_Gaussian.R:70); init: (.4, .7) (initialize.R:199);
    estimate/predict: (0, 1.5) (estimate.R:38, predict.R:37)."""
    out = []
    for name, v in zip(shape_params, np.atleast_1d(shape)):
        if name.startswith("log"):
            out.append(float(np.exp(v)))
        elif name.startswith("qlogis"):
            out.append(float(smooth_lo + smooth_span * plogis(v)))
    return out


def covparms(shape_params, shape, smooth_lo=0.5, smooth_span=0.5):
    """c(1, shape, 0): unit variance, zero nugget (update_Gaussian.R:72)."""
    return np.array([1.0] + transform_shape(shape_params, shape, smooth_lo, smooth_span) + [0.0])
