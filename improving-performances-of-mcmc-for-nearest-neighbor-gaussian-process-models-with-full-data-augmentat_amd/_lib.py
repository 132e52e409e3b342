"""ctypes binding of ``libnngp.so`` (the C ABI declared in include/nngp.h).

This is the Python twin of the R ``.Call`` shim described in INTEGRATION.md:
it only marshals R-convention arrays (column-major, 1-based, NA = INT_MIN)
into the C ABI and turns non-zero statuses into exceptions.  There is no
fallback: if the shared library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
# built in-tree at <repo>/lib/libnngp.so (a short path: the loaded library shows
# up in full in /proc/<pid>/maps and in the driver's native-library record)
LIB_PATH = Path(os.environ.get("NNGP_LIB", PKG_DIR.parent / "lib" / "libnngp.so"))
NA_INTEGER = -(2 ** 31)
# nngp_status (include/nngp.h)
NNGP_OK, NNGP_ERR_ARG, NNGP_ERR_HIP, NNGP_ERR_CHOL, NNGP_ERR_STATE, NNGP_ERR_NOMEM, NNGP_ERR_NODEV, NNGP_ERR_COMM = range(8)

COVFUNS = {
    "exponential_isotropic": 0, "exponential_sphere": 1, "exponential_scaledim": 2,
    "exponential_spacetime": 3, "matern_isotropic": 4, "matern_sphere": 5,
    "matern_scaledim": 6, "matern_spacetime": 7, "matern15_isotropic": 8,
}

# every symbol declared in include/nngp.h
ABI_SYMBOLS = (
    "nngp_abi_version", "nngp_status_string", "nngp_order_maxmin", "nngp_find_ordered_nn",
    "nngp_greedy_coloring", "nngp_ctx_create", "nngp_ctx_destroy", "nngp_ctx_last_error", "nngp_ctx_engine_note",
    "nngp_set_chain", "nngp_ctx_info", "nngp_factor", "nngp_get_linv", "nngp_set_linv", "nngp_accept_factor",
    "nngp_get_precision_diag", "nngp_set_field", "nngp_get_field", "nngp_set_mu",
    "nngp_loglik", "nngp_sweep", "nngp_sweep_chains", "nngp_ancillary_propose", "nngp_ancillary_propose_chains",
    "nngp_field_response_ratio",
    "nngp_accept_field", "nngp_beta0_stats", "nngp_sum_squared_residuals", "nngp_spmv",
    "nngp_tri_solve", "nngp_tri_rescues", "nngp_sweep_timed", "nngp_device_normals", "nngp_get_sweep_r",
    "nngp_ctx_create_shard", "nngp_shard_unique_id", "nngp_shard_comm_init", "nngp_sweep_chains_group",
    "nngp_records_reserve", "nngp_record_field", "nngp_get_records", "nngp_records_stream",
    "nngp_shard_ipc_handle", "nngp_shard_ipc_open", "nngp_shard_sync",
    "nngp_factor_chains", "nngp_loglik_chains", "nngp_field_response_ratio_chains",
    "nngp_sum_squared_residuals_chains", "nngp_loglik_pair_chains",
    "nngp_ancillary_step_chains", "nngp_sufficient_step_chains",
)
SHARD_ID_BYTES = 128  # NNGP_SHARD_ID_BYTES
IPC_HANDLE_BYTES = 192  # NNGP_IPC_HANDLE_BYTES


class NNGPError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"[nngp status {status}] {message}")
        self.status = status


class Info(C.Structure):
    _fields_ = [("n", C.c_int), ("b", C.c_int), ("d", C.c_int), ("n_obs", C.c_int),
                ("n_colors", C.c_int), ("n_levels", C.c_int), ("nnz", C.c_longlong),
                ("n_entries", C.c_longlong), ("max_collen", C.c_int), ("device", C.c_int),
                ("n_chains", C.c_int), ("lanes_per_chain", C.c_int), ("n_chunks", C.c_int),
                ("sweep_engine", C.c_int), ("n_tiles", C.c_int), ("tile_rows_max", C.c_int),
                ("n_ghost_cells", C.c_longlong), ("n_ranks", C.c_int), ("rank", C.c_int),
                ("shard_owned", C.c_longlong), ("shard_needed_rows", C.c_longlong),
                ("shard_exchange_slots", C.c_longlong), ("tile_ghost_pass", C.c_int),
                ("tile_ghost_cells_max", C.c_int), ("tile_r_global", C.c_int),
                ("tile_chain_split", C.c_int), ("tile_resident_per_cu", C.c_int),
                ("engine_fallback", C.c_int), ("tile_exchange_wave", C.c_int), ("device_cus", C.c_int),
                ("tile_rows_needed", C.c_int), ("device_lds", C.c_int)]


_dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_vp = C.c_void_p


def _load():
    if not LIB_PATH.exists():
        raise ImportError(
            f"libnngp.so not found at {LIB_PATH}: build it with `python -c \"import __graft_entry__ as g; g.build()\"` "
            "(or `make -C <pkg>/csrc`). There is no CPU fallback.")
    L = C.CDLL(str(LIB_PATH))
    L.nngp_abi_version.restype = C.c_int
    L.nngp_status_string.restype = C.c_char_p
    L.nngp_status_string.argtypes = [C.c_int]
    L.nngp_order_maxmin.argtypes = [_dp, C.c_int, C.c_int, _ip]
    L.nngp_find_ordered_nn.argtypes = [_dp, C.c_int, C.c_int, C.c_int, _ip]
    L.nngp_greedy_coloring.argtypes = [_ip, C.c_int, C.c_int, _ip, C.POINTER(C.c_int)]
    L.nngp_ctx_create.argtypes = [_dp, C.c_int, C.c_int, _ip, C.c_int, _ip, _ip, _dp, C.c_int,
                                  C.c_int, C.c_int, C.POINTER(_vp)]
    L.nngp_set_chain.argtypes = [_vp, C.c_int]
    L.nngp_ctx_destroy.argtypes = [_vp]
    L.nngp_ctx_destroy.restype = None
    L.nngp_ctx_last_error.argtypes = [_vp]
    L.nngp_ctx_last_error.restype = C.c_char_p
    L.nngp_ctx_info.argtypes = [_vp, C.POINTER(Info)]
    L.nngp_ctx_engine_note.argtypes = [_vp]
    L.nngp_ctx_engine_note.restype = C.c_char_p
    L.nngp_factor.argtypes = [_vp, C.c_int, C.c_int, _dp, C.c_int]
    L.nngp_get_linv.argtypes = [_vp, C.c_int, _dp]
    L.nngp_set_linv.argtypes = [_vp, C.c_int, _dp]
    L.nngp_accept_factor.argtypes = [_vp]
    L.nngp_get_precision_diag.argtypes = [_vp, _dp]
    L.nngp_set_field.argtypes = [_vp, _dp]
    L.nngp_get_field.argtypes = [_vp, _dp]
    L.nngp_set_mu.argtypes = [_vp, _vp, C.c_double]
    L.nngp_loglik.argtypes = [_vp, C.c_int, C.c_double, C.c_double, C.POINTER(C.c_double)]
    L.nngp_sweep.argtypes = [_vp, C.c_int, C.c_double, C.c_double, C.c_double, C.c_uint64,
                             C.c_uint64, _vp]
    L.nngp_ancillary_propose.argtypes = [_vp, C.c_double, C.c_double]
    L.nngp_field_response_ratio.argtypes = [_vp, C.c_double, C.c_double, C.POINTER(C.c_double)]
    L.nngp_accept_field.argtypes = [_vp]
    L.nngp_beta0_stats.argtypes = [_vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.nngp_sum_squared_residuals.argtypes = [_vp, C.c_double, C.POINTER(C.c_double)]
    L.nngp_spmv.argtypes = [_vp, C.c_int, _dp, C.c_int, _dp]
    L.nngp_tri_solve.argtypes = [_vp, C.c_int, _dp, _dp]
    L.nngp_tri_rescues.argtypes = [_vp, C.POINTER(C.c_longlong)]
    _up = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
    L.nngp_sweep_chains.argtypes = [_vp, C.c_int, _dp, _dp, _dp, _up, _up]
    L.nngp_ancillary_propose_chains.argtypes = [_vp, C.c_int, _dp, _dp]
    L.nngp_sweep_timed.argtypes = [_vp, C.c_int, _dp, _dp, _dp, _up, _up,
                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.nngp_device_normals.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, _dp]
    L.nngp_get_sweep_r.argtypes = [_vp, _dp]
    L.nngp_ctx_create_shard.argtypes = [_dp, C.c_int, C.c_int, _ip, C.c_int, _ip, _ip, _dp, C.c_int,
                                        C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]
    L.nngp_shard_unique_id.argtypes = [C.c_char_p, C.c_int]
    L.nngp_shard_comm_init.argtypes = [_vp, C.c_char_p, C.c_int]
    L.nngp_sweep_chains_group.argtypes = [C.POINTER(_vp), C.c_int, C.c_int, _dp, _dp, _dp, _up, _up]
    L.nngp_factor_chains.argtypes = [_vp, C.c_int, C.c_int, C.c_int, _dp, C.c_int, _ip]
    L.nngp_loglik_chains.argtypes = [_vp, C.c_int, C.c_int, _dp, _dp, _dp]
    L.nngp_field_response_ratio_chains.argtypes = [_vp, C.c_int, _dp, _dp, _dp]
    L.nngp_sum_squared_residuals_chains.argtypes = [_vp, C.c_int, _dp, _dp]
    L.nngp_loglik_pair_chains.argtypes = [_vp, C.c_int, _dp, _dp, _dp, _dp, _dp]
    L.nngp_ancillary_step_chains.argtypes = [_vp, C.c_int, C.c_int, _dp, C.c_int, _dp, _dp, _dp, _ip, _dp]
    L.nngp_sufficient_step_chains.argtypes = [_vp, C.c_int, C.c_int, _dp, C.c_int, _dp, _dp, _dp, _ip, _dp, _dp]
    L.nngp_shard_ipc_handle.argtypes = [_vp, C.c_char_p, C.c_int]
    L.nngp_shard_ipc_open.argtypes = [_vp, C.c_char_p, C.c_int]
    L.nngp_shard_sync.argtypes = [_vp]
    L.nngp_records_reserve.argtypes = [_vp, C.c_int]
    L.nngp_record_field.argtypes = [_vp, C.c_int]
    L.nngp_get_records.argtypes = [_vp, C.c_int, C.c_int, _dp]
    L.nngp_records_stream.argtypes = [_vp, _vp, C.c_int]
    return L


lib = _load()


def check(status: int, ctx=None) -> None:
    if status != 0:
        msg = lib.nngp_ctx_last_error(ctx)
        msg = msg.decode() if msg else lib.nngp_status_string(status).decode()
        raise NNGPError(status, msg)


def colmajor(a, dtype) -> np.ndarray:
    """R matrix (n x p, numpy row-major) -> contiguous column-major buffer."""
    return np.ascontiguousarray(np.asarray(a, dtype=dtype).T)


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)
