"""Device contexts of MCMC chains (replace the per-chain ``mclapply`` workers
of Scripts/mcmc_nngp_update_Gaussian.R:25-26 -- HIP is not fork-safe, so
chains live in device contexts, possibly on different devices, not in forked
processes).  One context holds up to 4 chains over the same graph; their
sweeps run in the same kernels (``sweep_chains``).  ``ChainView`` exposes
one chain of a context with the single-chain interface.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import COVFUNS, Info, check, colmajor, f64, i32, lib


MAX_CHAINS_PER_CONTEXT = 4


class ChainContext:
    """Device-resident state of 1..4 chains: locations, NNarray, colouring,
    observations (shared); the current/proposal Vecchia factors, the latent
    field and the mean (per chain).  Per-chain methods act on the selected
    chain (``select``; chain 0 by default)."""

    def __init__(self, locs, NNarray, coloring, locs_match, observed_field, device: int = -1,
                 n_chains: int = 1, _shard=None):
        locs = np.asarray(locs, np.float64)
        if locs.ndim == 1:
            locs = locs[:, None]
        NNarray = np.asarray(NNarray, np.int32)
        n, d = locs.shape
        b = NNarray.shape[1]
        self.n, self.d, self.b = n, d, b
        self.n_obs = len(observed_field)
        self.n_chains = int(n_chains)
        h = C.c_void_p()
        args = (colmajor(locs, np.float64), n, d, colmajor(NNarray, np.int32), b, i32(coloring), i32(locs_match),
                f64(observed_field), self.n_obs, self.n_chains, int(device))
        if _shard is None:
            check(lib.nngp_ctx_create(*args, C.byref(h)))
        else:
            check(lib.nngp_ctx_create_shard(*args, int(_shard[0]), int(_shard[1]), C.byref(h)))
        self._h = h
        self._sel = 0
        self._rec_host = {}  # chain -> host array its records stream into (records_stream)

    def select(self, chain: int) -> "ChainContext":
        if chain != self._sel:
            self._chk(lib.nngp_set_chain(self._h, int(chain)))
            self._sel = int(chain)
        return self

    def view(self, chain: int) -> "ChainView":
        return ChainView(self, chain)

    # ------------------------------------------------------------ lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            lib.nngp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, status):
        check(status, self._h)

    @property
    def info(self) -> dict:
        inf = Info()
        self._chk(lib.nngp_ctx_info(self._h, C.byref(inf)))
        d = {k: getattr(inf, k) for k, _ in Info._fields_}
        d["engine_note"] = lib.nngp_ctx_engine_note(self._h).decode()
        return d

    # ------------------------------------------------------------ factor (A4/A5)
    def factor(self, which: int, covfun: str, covparms) -> None:
        cp = f64(covparms)
        self._chk(lib.nngp_factor(self._h, which, COVFUNS[covfun], cp, len(cp)))

    def get_linv(self, which: int = 0) -> np.ndarray:
        out = np.zeros(self.n * self.b)
        self._chk(lib.nngp_get_linv(self._h, which, out))
        return out.reshape(self.b, self.n).T.copy()

    def set_linv(self, which: int, Linv) -> None:
        self._chk(lib.nngp_set_linv(self._h, which, colmajor(Linv, np.float64)))

    def accept_factor(self) -> None:
        self._chk(lib.nngp_accept_factor(self._h))

    def precision_diag(self) -> np.ndarray:
        out = np.zeros(self.n)
        self._chk(lib.nngp_get_precision_diag(self._h, out))
        return out

    # ------------------------------------------------------------ state
    def set_field(self, field) -> None:
        self._chk(lib.nngp_set_field(self._h, f64(field)))

    def get_field(self) -> np.ndarray:
        out = np.zeros(self.n)
        self._chk(lib.nngp_get_field(self._h, out))
        return out

    # ------------------------------------------------------------ records
    def records_reserve(self, n_rows: int) -> None:
        """Device buffer of n_rows recorded fields for the selected chain."""
        self._chk(lib.nngp_records_reserve(self._h, int(n_rows)))
        self._rec_host.pop(self._sel, None)

    def record_field(self, row: int) -> None:
        self._chk(lib.nngp_record_field(self._h, int(row)))

    def records_stream(self, host: np.ndarray | None) -> None:
        """Stream the selected chain's recorded rows into `host` (C-contiguous
        float64, reserved rows x n) while the chain runs; get_records(0, rows,
        out=host) then only waits for them.  None ends the binding.  The
        context keeps a reference to `host` while it is bound."""
        if host is None:
            self._chk(lib.nngp_records_stream(self._h, None, 0))
            self._rec_host.pop(self._sel, None)
            return
        assert host.dtype == np.float64 and host.flags.c_contiguous and host.ndim == 2 and host.shape[1] == self.n
        self._chk(lib.nngp_records_stream(self._h, host.ctypes.data, int(host.shape[0])))
        self._rec_host[self._sel] = host

    def get_records(self, row0: int, n_rows: int, out: np.ndarray | None = None) -> np.ndarray:
        """Rows [row0, row0 + n_rows) of the records; into `out` (C-contiguous
        float64, n_rows x n) when given."""
        if out is None:
            out = np.empty((int(n_rows), self.n))
        assert out.dtype == np.float64 and out.flags.c_contiguous and out.shape == (int(n_rows), self.n)
        host = self._rec_host.get(self._sel)
        bound = host is not None and out.ctypes.data == host.ctypes.data + int(row0) * self.n * 8
        self._chk(lib.nngp_get_records(self._h, int(row0), int(n_rows), out.reshape(-1)))
        if bound:  # get_records on the bound array ends the binding (nngp.h)
            self._rec_host.pop(self._sel, None)
        return out

    def set_mu(self, mu, beta0: float) -> None:
        """mu = None means mu == beta_0 for every observation (no X)."""
        self._mu_keep = None if mu is None else f64(mu)
        ptr = None if mu is None else self._mu_keep.ctypes.data
        self._chk(lib.nngp_set_mu(self._h, ptr, float(beta0)))

    # ------------------------------------------------------------ kernels
    def loglik(self, which: int, beta0: float, log_scale: float) -> float:
        out = C.c_double()
        self._chk(lib.nngp_loglik(self._h, which, float(beta0), float(log_scale), C.byref(out)))
        return out.value

    def sweep(self, n_sweeps: int, beta0: float, log_scale: float, log_noise_variance: float,
              seed: int, counter_base: int, z=None) -> None:
        zp = None
        if z is not None:
            z = np.ascontiguousarray(np.atleast_2d(z), np.float64)
            assert z.shape == (n_sweeps, self.n)
            zp = z.ctypes.data
        self._chk(lib.nngp_sweep(self._h, int(n_sweeps), float(beta0), float(log_scale),
                                 float(log_noise_variance), int(seed) & (2 ** 64 - 1),
                                 int(counter_base) & (2 ** 64 - 1), zp))

    def sweep_chains(self, n_sweeps: int, beta0, log_scale, log_noise_variance, seed, counter_base) -> None:
        """n_sweeps sweeps of every chain (per-chain argument sequences)."""
        a = self._chain_args(beta0, log_scale, log_noise_variance, seed, counter_base)
        self._chk(lib.nngp_sweep_chains(self._h, int(n_sweeps), *a))

    def _chain_args(self, beta0, log_scale, log_noise_variance, seed, counter_base):
        k = self.n_chains
        f = [np.ascontiguousarray(np.broadcast_to(np.asarray(v, np.float64), (k,))) for v in
             (beta0, log_scale, log_noise_variance)]
        u = [np.ascontiguousarray(np.broadcast_to(np.asarray([int(x) & (2 ** 64 - 1) for x in np.atleast_1d(v)],
                                                             np.uint64), (k,))) for v in (seed, counter_base)]
        return (*f, *u)

    def sweep_timed(self, n_sweeps, beta0, log_scale, log_noise_variance, seed, counter_base,
                    per_kernel: bool = False):
        """sweep_chains bracketed by HIP events -> (ms, summed per-colour kernel ms or None)."""
        ms = C.c_double()
        kms = C.c_double()
        a = self._chain_args(beta0, log_scale, log_noise_variance, seed, counter_base)
        self._chk(lib.nngp_sweep_timed(self._h, int(n_sweeps), *a, C.byref(ms),
                                       C.byref(kms) if per_kernel else None))
        return ms.value, (kms.value if per_kernel else None)

    def get_sweep_r(self) -> np.ndarray:
        """r = B (field - beta0) of the selected chain as the last sweep call
        left it (location order): the state a warm tile call starts from."""
        out = np.empty(self.n, np.float64)
        self._chk(lib.nngp_get_sweep_r(self._h, out))
        return out

    def ancillary_propose(self, beta0: float, dlog_scale: float) -> None:
        self._chk(lib.nngp_ancillary_propose(self._h, float(beta0), float(dlog_scale)))

    def ancillary_propose_chains(self, chain_mask: int, beta0, dlog_scale) -> None:
        """ancillary_propose for every chain in chain_mask (bit k = chain k) in
        one triangular-solve schedule; beta0/dlog_scale indexed by chain."""
        k = self.n_chains
        b = np.ascontiguousarray(np.broadcast_to(np.asarray(beta0, np.float64), (k,)))
        d = np.ascontiguousarray(np.broadcast_to(np.asarray(dlog_scale, np.float64), (k,)))
        self._chk(lib.nngp_ancillary_propose_chains(self._h, int(chain_mask), b, d))

    # ---- batched forms: every chain in chain_mask in one call (one host sync);
    # per-chain arrays indexed by chain, entries of other chains ignored
    def _vec(self, v):
        return np.ascontiguousarray(np.broadcast_to(np.asarray(v, np.float64), (self.n_chains,)))

    def factor_chains(self, which: int, chain_mask: int, covfun: str, covparms) -> np.ndarray:
        """-> per-chain status (0 = ok, NNGP_ERR_CHOL = not positive definite);
        covparms: n_chains rows (chains outside the mask: any values)."""
        cps = np.ascontiguousarray(np.asarray(covparms, np.float64).reshape(self.n_chains, -1))
        st = np.zeros(self.n_chains, np.int32)
        self._chk(lib.nngp_factor_chains(self._h, int(which), int(chain_mask), COVFUNS[covfun], cps.reshape(-1),
                                         cps.shape[1], st))
        return st

    def loglik_chains(self, which: int, chain_mask: int, beta0, log_scale) -> np.ndarray:
        out = np.zeros(self.n_chains)
        self._chk(lib.nngp_loglik_chains(self._h, int(which), int(chain_mask), self._vec(beta0), self._vec(log_scale),
                                         out))
        return out

    def loglik_pair_chains(self, chain_mask: int, beta0, log_scale_prop, log_scale_cur):
        """(loglik_chains(1, ...), loglik_chains(0, ...)) in one pass over the rows."""
        lp, lc = np.zeros(self.n_chains), np.zeros(self.n_chains)
        self._chk(lib.nngp_loglik_pair_chains(self._h, int(chain_mask), self._vec(beta0), self._vec(log_scale_prop),
                                              self._vec(log_scale_cur), lp, lc))
        return lp, lc

    def ancillary_step_chains(self, chain_mask: int, covfun: str, covparms, beta0, dlog_scale, log_noise_variance):
        """factor_chains(1, ...) + ancillary_propose_chains +
        field_response_ratio_chains behind one host sync -> (status, ratio);
        a chain whose proposal factor fails: NNGP_ERR_CHOL and ratio NaN."""
        cps = np.ascontiguousarray(np.asarray(covparms, np.float64).reshape(self.n_chains, -1))
        st = np.zeros(self.n_chains, np.int32)
        out = np.zeros(self.n_chains)
        self._chk(lib.nngp_ancillary_step_chains(self._h, int(chain_mask), COVFUNS[covfun], cps.reshape(-1),
                                                 cps.shape[1], self._vec(beta0), self._vec(dlog_scale),
                                                 self._vec(log_noise_variance), st, out))
        return st, out

    def sufficient_step_chains(self, chain_mask: int, covfun: str, covparms, beta0, log_scale_prop, log_scale_cur):
        """factor_chains(1, ...) + loglik_pair_chains behind one host sync ->
        (status, ll_prop, ll_cur); a failed proposal factor: NaN values."""
        cps = np.ascontiguousarray(np.asarray(covparms, np.float64).reshape(self.n_chains, -1))
        st = np.zeros(self.n_chains, np.int32)
        lp, lc = np.zeros(self.n_chains), np.zeros(self.n_chains)
        self._chk(lib.nngp_sufficient_step_chains(self._h, int(chain_mask), COVFUNS[covfun], cps.reshape(-1),
                                                  cps.shape[1], self._vec(beta0), self._vec(log_scale_prop),
                                                  self._vec(log_scale_cur), st, lp, lc))
        return st, lp, lc

    def field_response_ratio_chains(self, chain_mask: int, beta0, log_noise_variance) -> np.ndarray:
        out = np.zeros(self.n_chains)
        self._chk(lib.nngp_field_response_ratio_chains(self._h, int(chain_mask), self._vec(beta0),
                                                       self._vec(log_noise_variance), out))
        return out

    def sum_squared_residuals_chains(self, chain_mask: int, beta0) -> np.ndarray:
        out = np.zeros(self.n_chains)
        self._chk(lib.nngp_sum_squared_residuals_chains(self._h, int(chain_mask), self._vec(beta0), out))
        return out

    def field_response_ratio(self, beta0: float, log_noise_variance: float) -> float:
        out = C.c_double()
        self._chk(lib.nngp_field_response_ratio(self._h, float(beta0), float(log_noise_variance),
                                                C.byref(out)))
        return out.value

    def accept_field(self) -> None:
        self._chk(lib.nngp_accept_field(self._h))

    def beta0_stats(self):
        a, b = C.c_double(), C.c_double()
        self._chk(lib.nngp_beta0_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def sum_squared_residuals(self, beta0: float) -> float:
        out = C.c_double()
        self._chk(lib.nngp_sum_squared_residuals(self._h, float(beta0), C.byref(out)))
        return out.value

    def spmv(self, which: int, X) -> np.ndarray:
        X = np.asarray(X, np.float64)
        vec = X.ndim == 1
        X2 = X[:, None] if vec else X
        out = np.zeros(X2.shape[0] * X2.shape[1])
        self._chk(lib.nngp_spmv(self._h, which, colmajor(X2, np.float64), X2.shape[1], out))
        Y = out.reshape(X2.shape[1], X2.shape[0]).T
        return Y[:, 0].copy() if vec else Y.copy()

    def tri_solve(self, which: int, u) -> np.ndarray:
        out = np.zeros(self.n)
        self._chk(lib.nngp_tri_solve(self._h, which, f64(u), out))
        return out

    def tri_rescues(self) -> int:
        """Sync-free solves of this context that finished in the rescue's
        ticket order (their static order stalled on non-resident waves)."""
        out = C.c_longlong()
        self._chk(lib.nngp_tri_rescues(self._h, C.byref(out)))
        return out.value


class ChainView:
    """One chain of a ChainContext with the single-chain interface (every
    method selects the chain first)."""

    def __init__(self, ctx: ChainContext, chain: int):
        self.ctx, self.chain = ctx, int(chain)
        self.n, self.d, self.b, self.n_obs = ctx.n, ctx.d, ctx.b, ctx.n_obs

    def __getattr__(self, name):
        attr = getattr(self.ctx, name)
        if not callable(attr) or name in ("close", "view", "sweep_chains", "sweep_timed",
                                                     "ancillary_propose_chains", "factor_chains", "loglik_chains",
                                                     "field_response_ratio_chains", "sum_squared_residuals_chains",
                                                     "loglik_pair_chains", "ancillary_step_chains",
                                                     "sufficient_step_chains"):
            return attr

        def bound(*a, **kw):
            self.ctx.select(self.chain)
            return attr(*a, **kw)
        return bound

    @property
    def info(self) -> dict:
        return self.ctx.info

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.ctx.close()


# LDS of a 512-thread tile besides r (slot totals, batch table, hand-off
# values, ...): about 17 KB at configs[4]'s per-GPU share, graph_prep.cpp
# tile_lds_bytes
_TILE_LDS_OTHER = 24 * 1024


def _lds_limited(ctx) -> bool:
    """The context's tiles do not keep r in LDS at its chain count, but would
    at half of it: it runs the colour engine for the LDS (engine_fallback 1,
    the note names the LDS) or tiles with r in global memory (a tile shard
    whose LDS tiles do not fit) -- not when r in global memory was asked for
    (NNGP_TILE_R=global) or half the chains' rows still exceed the LDS."""
    inf = ctx.info
    limited = ((inf["sweep_engine"] == 0 and inf["engine_fallback"] == 1 and "LDS" in inf["engine_note"]) or
               (inf["sweep_engine"] == 1 and "r in global memory" in inf["engine_note"] and
                os.environ.get("NNGP_TILE_R", "") != "global"))
    half = (ctx.n_chains + 1) // 2
    return limited and 0 < inf["tile_rows_needed"] * half * 8 + _TILE_LDS_OTHER <= inf["device_lds"]


def split_groups(open_ctx, group):
    """Contexts for the chains `group`: open_ctx(chains) -> context; one
    context, or -- when its tiles keep r in LDS only at fewer chains (4
    chains at the headline n = 1e6: a tile's 5.2k local rows x 4 x 8 B > 160
    KB; configs[4]'s per-GPU share at 3 chains) -- the two halves of the group
    as separate contexts, recursively, on the LDS tile engine (the launches of
    the contexts of one device are chained on the GPU, capi.hip
    tile_chain_event).  NNGP_SPLIT_CHAINS=0 keeps one context per group.
    -> [(context, chain ids)]."""
    ctx = open_ctx(len(group))
    if len(group) < 2 or os.environ.get("NNGP_SPLIT_CHAINS", "1") == "0" or not _lds_limited(ctx):
        return [(ctx, group)]
    ctx.close()
    h = (len(group) + 1) // 2
    return split_groups(open_ctx, group[:h]) + split_groups(open_ctx, group[h:])


def _open_group(locs, NNarray, coloring, locs_match, observed_field, dev, group):
    return split_groups(lambda k: ChainContext(locs, NNarray, coloring, locs_match, observed_field, device=dev,
                                               n_chains=k), group)


def make_chain_views(locs, NNarray, coloring, locs_match, observed_field, n_chains: int, devices=None):
    """Chains dealt round-robin over `devices`, then packed <= 4 per context
    (split further where the tile engine needs it, _open_group): returns one
    ChainView per chain (chain i -> views[i])."""
    devices = list(devices) if devices else [-1]
    per_dev = {}
    for i in range(n_chains):
        per_dev.setdefault(devices[i % len(devices)], []).append(i)
    views = [None] * n_chains
    for dev, chains in per_dev.items():
        for g in range(0, len(chains), MAX_CHAINS_PER_CONTEXT):
            for ctx, group in _open_group(locs, NNarray, coloring, locs_match, observed_field, dev,
                                          chains[g:g + MAX_CHAINS_PER_CONTEXT]):
                for k, i in enumerate(group):
                    views[i] = ctx.view(k)
    return views


def device_normals(seed: int, sweep: int, n: int, device: int = 0) -> np.ndarray:
    out = np.zeros(n)
    check(lib.nngp_device_normals(device, seed, sweep, n, out))
    return out
