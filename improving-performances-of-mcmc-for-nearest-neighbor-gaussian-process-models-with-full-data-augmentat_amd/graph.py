"""Init-time graph preparation (host C++ behind the C ABI).

Mirrors the GpGp/Coloring.R entry points the reference calls during
``mcmc_nngp_initialize`` (Scripts/mcmc_nngp_initialize.R:29,93,97-110):

* :func:`order_maxmin`     -- GpGp::order_maxmin (exact max-min here; GpGp's is
                              an RNG-jittered approximation, so orderings are
                              an *input*, not a parity item -- SURVEY §0.1-4)
* :func:`find_ordered_nn`  -- GpGp::find_ordered_nn (exact, ties -> smaller index)
* :func:`naive_greedy_coloring` -- Scripts/Coloring.R:2-20 on the moral graph
* :func:`sparse_chol_indices`  -- the NNarray_non_NA / row / column index
                              vectors of initialize.R:97-101
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import NA_INTEGER, check, colmajor, i32, lib


def order_maxmin(locs) -> np.ndarray:
    """1-based max-min permutation of the rows of ``locs`` (n x d)."""
    locs = np.asarray(locs, np.float64)
    n, d = locs.shape
    out = np.zeros(n, np.int32)
    check(lib.nngp_order_maxmin(colmajor(locs, np.float64), n, d, out))
    return out


def find_ordered_nn(locs, m: int) -> np.ndarray:
    """n x (m+1) int32 NNarray (1-based, NA = INT_MIN like R's NA_integer_)."""
    locs = np.asarray(locs, np.float64)
    n, d = locs.shape
    m = int(min(m, n - 1))
    buf = np.zeros((m + 1) * n, np.int32)
    check(lib.nngp_find_ordered_nn(colmajor(locs, np.float64), n, d, m, buf))
    return buf.reshape(m + 1, n).T.copy()


def naive_greedy_coloring(NNarray) -> np.ndarray:
    """Greedy first-fit colouring of pattern(B^T B) in index order (1-based)."""
    NNarray = np.asarray(NNarray, np.int32)
    n, b = NNarray.shape
    cols = np.zeros(n, np.int32)
    K = C.c_int(0)
    check(lib.nngp_greedy_coloring(colmajor(NNarray, np.int32), n, b, cols, C.byref(K)))
    return cols


def sparse_chol_indices(NNarray):
    """(NNarray_non_NA, sparse_chol_row_idx, sparse_chol_column_idx) as in
    initialize.R:97-101 (column-major vectorisation, 1-based)."""
    non_na = NNarray != NA_INTEGER
    rows = np.broadcast_to(np.arange(1, NNarray.shape[0] + 1)[:, None], NNarray.shape)
    col_idx = NNarray.T[non_na.T]
    row_idx = rows.T[non_na.T]
    return non_na, i32(row_idx), i32(col_idx)
