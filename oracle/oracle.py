"""CPU ORACLE -- test infrastructure only.

ctypes front-end to ``oracle/liboracle.so`` (plain-C restatement of the
reference, see nngp_oracle.c for the file:line map) plus numpy restatements
of the scalar MCMC blocks of ``Scripts/mcmc_nngp_update_Gaussian.R``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  The product never does.
"""
from __future__ import annotations

import ctypes as C
import functools
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
NA = -(2 ** 31)

COVFUN_IDS = {
    "exponential_isotropic": 0, "exponential_sphere": 1,
    "exponential_scaledim": 2, "exponential_spacetime": 3,
    "matern_isotropic": 4, "matern_sphere": 5, "matern_scaledim": 6,
    "matern_spacetime": 7, "matern15_isotropic": 8,
}

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        up = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        L.or_philox4x32_10.argtypes = [up, up, up]
        L.or_normal.restype = C.c_double
        L.or_normal.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        L.or_normals.argtypes = [C.c_uint64, C.c_uint64, C.c_int, dp]
        L.or_qnorm.restype = C.c_double
        L.or_qnorm.argtypes = [C.c_double]
        L.or_bessel_k.restype = C.c_double
        L.or_bessel_k.argtypes = [C.c_double, C.c_double]
        L.or_ncovparms.restype = C.c_int
        L.or_covmat.argtypes = [C.c_int, dp, dp, C.c_int, C.c_int, C.c_int, dp]
        L.or_vecchia_linv.restype = C.c_int
        L.or_vecchia_linv.argtypes = [C.c_int, dp, dp, C.c_int, C.c_int, ip, C.c_int, dp]
        L.or_linv_mult.argtypes = [dp, dp, ip, C.c_int, C.c_int, dp]
        L.or_loglik.restype = C.c_double
        L.or_loglik.argtypes = [dp, dp, ip, C.c_int, C.c_int, C.c_double]
        L.or_precision_diag.argtypes = [dp, ip, C.c_int, C.c_int, dp]
        L.or_residuals_sum.argtypes = [dp, dp, ip, C.c_int, C.c_int, dp]
        sweep_args = [C.c_int, dp, ip, C.c_int, C.c_int, ip, dp, ip, dp, dp, ip,
                      C.c_int, C.c_double, C.c_double, C.c_double, dp, dp]
        L.or_sweep_masked.argtypes = sweep_args
        L.or_sweep_local.argtypes = sweep_args
        L.or_sweep_masked_mt.argtypes = [C.c_int] + sweep_args
        L.or_sweep_local_mt.argtypes = [C.c_int] + sweep_args
        L.or_find_ordered_nn.argtypes = [dp, C.c_int, C.c_int, C.c_int, ip]
        L.or_greedy_coloring.restype = C.c_int
        L.or_greedy_coloring.argtypes = [ip, C.c_int, C.c_int, ip]
        L.or_moral_graph.restype = C.c_int
        L.or_moral_graph.argtypes = [ip, C.c_int, C.c_int, C.POINTER(C.POINTER(C.c_int)),
                                     C.POINTER(C.POINTER(C.c_int))]
        L.or_free.argtypes = [C.c_void_p]
        L.or_tri_solve.argtypes = [dp, ip, C.c_int, C.c_int, dp, dp]
        L.or_order_maxmin_exact.argtypes = [dp, C.c_int, C.c_int, ip]
        _lib = L
    return _lib


def _f(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _colmajor(a, dtype):
    """R matrices are column-major: pass A.T contiguous (= Fortran order)."""
    return np.ascontiguousarray(np.asarray(a, dtype=dtype).T)


# ---------------------------------------------------------------- RNG
def philox4x32_10(ctr, key):
    out = np.zeros(4, np.uint32)
    lib().or_philox4x32_10(np.asarray(ctr, np.uint32), np.asarray(key, np.uint32), out)
    return out


def normals(seed: int, sweep: int, n: int) -> np.ndarray:
    z = np.zeros(n)
    lib().or_normals(seed, sweep, n, z)
    return z


def qnorm(p: float) -> float:
    return lib().or_qnorm(float(p))


def sweep_normals(seed: int, counter_base: int, n_sweeps: int, n: int) -> np.ndarray:
    return np.stack([normals(seed, counter_base + s, n) for s in range(n_sweeps)])


# ---------------------------------------------------------------- graph
def find_ordered_nn(locs: np.ndarray, m: int) -> np.ndarray:
    """GpGp::find_ordered_nn restated (exact). locs n x d. Returns n x (m+1)
    int32, 1-based, NA = INT_MIN (R's NA_integer_)."""
    n, d = locs.shape
    NN = np.zeros((m + 1) * n, np.int32)
    lib().or_find_ordered_nn(_colmajor(locs, np.float64), n, d, m, NN)
    return NN.reshape(m + 1, n).T.copy()


def moral_graph(NNarray: np.ndarray):
    """pattern(crossprod(B)) as CSC (colptr, rowidx) 0-based."""
    n, b = NNarray.shape
    cp = C.POINTER(C.c_int)()
    ri = C.POINTER(C.c_int)()
    nz = lib().or_moral_graph(_colmajor(NNarray, np.int32), n, b, C.byref(cp), C.byref(ri))
    colptr = np.ctypeslib.as_array(cp, shape=(n + 1,)).copy()
    rowidx = np.ctypeslib.as_array(ri, shape=(nz,)).copy()
    lib().or_free(C.cast(cp, C.c_void_p))
    lib().or_free(C.cast(ri, C.c_void_p))
    return colptr, rowidx


def greedy_coloring(NNarray: np.ndarray) -> np.ndarray:
    n, b = NNarray.shape
    cols = np.zeros(n, np.int32)
    K = lib().or_greedy_coloring(_colmajor(NNarray, np.int32), n, b, cols)
    assert K > 0
    return cols


def order_maxmin_exact(locs: np.ndarray) -> np.ndarray:
    n, d = locs.shape
    o = np.zeros(n, np.int32)
    lib().or_order_maxmin_exact(_colmajor(locs, np.float64), n, d, o)
    return o


# ---------------------------------------------------------------- kernels
def covmat(covfun: str, covparms, locs) -> np.ndarray:
    locs = np.asarray(locs, np.float64)
    n, d = locs.shape
    Cm = np.zeros(n * n)
    lib().or_covmat(COVFUN_IDS[covfun], _f(covparms), _colmajor(locs, np.float64), n, d, n, Cm)
    return Cm.reshape(n, n)


def vecchia_linv(covfun: str, covparms, locs, NNarray) -> np.ndarray:
    locs = np.asarray(locs, np.float64)
    n, d = locs.shape
    b = NNarray.shape[1]
    out = np.zeros(n * b)
    fail = lib().or_vecchia_linv(COVFUN_IDS[covfun], _f(covparms), _colmajor(locs, np.float64),
                                 n, d, _colmajor(NNarray, np.int32), b, out)
    if fail:
        raise np.linalg.LinAlgError(f"local covariance not positive definite at row {fail}")
    return out.reshape(b, n).T.copy()


def linv_mult(Linv, z, NNarray) -> np.ndarray:
    n, b = NNarray.shape
    u = np.zeros(n)
    lib().or_linv_mult(_colmajor(Linv, np.float64), _f(z), _colmajor(NNarray, np.int32), n, b, u)
    return u


def loglik(Linv, z, NNarray, log_scale) -> float:
    n, b = NNarray.shape
    return lib().or_loglik(_colmajor(Linv, np.float64), _f(z), _colmajor(NNarray, np.int32), n, b,
                           float(log_scale))


def precision_diag(Linv, NNarray) -> np.ndarray:
    n, b = NNarray.shape
    D = np.zeros(n)
    lib().or_precision_diag(_colmajor(Linv, np.float64), _colmajor(NNarray, np.int32), n, b, D)
    return D


def residuals_sum(y, mu, locs_match, n) -> np.ndarray:
    R = np.zeros(n)
    lib().or_residuals_sum(_f(y), _f(mu), _i(locs_match), len(y), n, R)
    return R


def tri_solve(Linv, NNarray, u) -> np.ndarray:
    n, b = NNarray.shape
    x = np.zeros(n)
    lib().or_tri_solve(_colmajor(Linv, np.float64), _colmajor(NNarray, np.int32), n, b, _f(u), x)
    return x


def sweep(form: str, field, Linv, NNarray, coloring, D, obs_per_loc, y, mu, locs_match,
          beta0, log_scale, log_noise_var, z, threads: int = 1) -> np.ndarray:
    """n_sweeps = z.shape[0] chromatic sweeps; returns the new field.
    threads > 1: the OpenMP forms (bitwise equal to the serial ones)."""
    n, b = NNarray.shape
    z = np.atleast_2d(np.asarray(z, np.float64))
    out = _f(field).copy()
    if threads > 1:
        fn = lib().or_sweep_masked_mt if form == "masked" else lib().or_sweep_local_mt
        fn = functools.partial(fn, int(threads))
    else:
        fn = lib().or_sweep_masked if form == "masked" else lib().or_sweep_local
    fn(z.shape[0], _colmajor(Linv, np.float64), _colmajor(NNarray, np.int32), n, b, _i(coloring),
       _f(D), _i(obs_per_loc), _f(y), _f(mu), _i(locs_match), len(y), float(beta0),
       float(log_scale), float(log_noise_var), np.ascontiguousarray(z), out)
    return out


def bessel_k(nu, x) -> float:
    return lib().or_bessel_k(float(nu), float(x))


# ---------------------------------------------------------------- dense KATs (numpy)
def dense_B(Linv, NNarray) -> np.ndarray:
    n, b = NNarray.shape
    B = np.zeros((n, n))
    for i in range(n):
        for j in range(b):
            if NNarray[i, j] != NA:
                B[i, NNarray[i, j] - 1] = Linv[i, j]
    return B


# ---------------------------------------------------------------- posterior prediction
def _plogis(x):
    return 1.0 / (1.0 + np.exp(-x))


def predict_covparms(shape_params, shape) -> np.ndarray:
    """c(1, shape, 0) with predict.R:34-38's transforms: exp() for log_*,
    1.5 * plogis() for qlogis_* (not the MCMC's .5 + .5 * plogis)."""
    out = [1.0]
    for name, v in zip(shape_params, np.atleast_1d(shape)):
        if name[:3] == "log":
            out.append(float(np.exp(v)))
        elif name[:6] == "qlogis":
            out.append(float(1.5 * _plogis(v)))
    return np.array(out + [0.0])


def predict_field(mcmc_nngp_list, predicted_locs, z_new, burn_in=0.5, m=10):
    """Restatement of Scripts/mcmc_nngp_predict.R:1-60 (mcmc_nngp_predict_field).

    z_new[k] is an (n_samples, n_pred) array of the normals chain k draws for
    the new locations (predict.R:50, rnorm), so the device path can be fed the
    same values.  Returns the per-chain (n_samples, n_pred) sample arrays."""
    L = mcmc_nngp_list
    locs = np.asarray(L["locs"], np.float64)
    pred = np.asarray(predicted_locs, np.float64)
    allloc = np.vstack([locs, pred])                                   # :4
    NN = find_ordered_nn(allloc, m)                                    # :5
    n, N = locs.shape[0], allloc.shape[0]
    covfun = L["space_time_model"]["covfun"]["stationary_covfun"]
    sp = L["space_time_model"]["covfun"]["shape_params"]
    chains = list(L["records"].values())
    stored = np.asarray(chains[0]["saved_field"])                      # :13
    stored = stored[stored > burn_in * stored.max()].astype(int)       # :14
    out = []
    for k, chain in enumerate(chains):                                 # :16-18
        samples = np.zeros((len(stored), pred.shape[0]))               # :21
        shapes = np.asarray(chain["params"]["shape"])[stored - 1]
        shapes = shapes.reshape(len(stored), -1)
        seen = set()
        Linv = None
        for ip, i_chain in enumerate(stored):                          # :25-28
            i_field = int(np.nonzero(np.asarray(chain["saved_field"]) == i_chain)[0][0])  # :30
            key = tuple(shapes[ip])
            if key not in seen:                                        # :23,32 !duplicated
                seen.add(key)
                cp = predict_covparms(sp, shapes[ip])
                Linv = vecchia_linv(covfun, cp, allloc, NN)            # :39
            sd = np.exp(0.5 * float(np.asarray(chain["params"]["log_scale"])[i_chain - 1].ravel()[0]))  # :43
            b0 = float(np.asarray(chain["params"]["beta_0"])[i_chain - 1].ravel()[0])
            w = np.asarray(chain["params"]["field"])[i_field] - b0
            # B[1:n, 1:n] w: rows < n of the stacked factor reference columns < n only
            u = linv_mult(Linv, np.concatenate([w, np.zeros(N - n)]), NN)[:n]   # :49
            x = tri_solve(Linv, NN, np.concatenate([u / sd, np.asarray(z_new[k][ip], np.float64)]))  # :46-52
            samples[ip] = sd * x[n:]                                   # :44,53
        out.append(samples)
    return out
