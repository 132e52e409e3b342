"""Sharded chromatic sweep: ONE set of chains swept by several GPUs
(DESIGN.md §6).

Two engines behind the same interface (nngp_ctx_info's sweep_engine):
 - tile shard (default when the tile layout fits): the persistent tile sweep
   with its tiles split over the ranks; the draws other ranks' tiles read are
   written straight into their granule buffers (peer memory over xGMI, HIP
   IPC), one launch per call, then each rank's halo slots into the peers'
   replicas (peer stores + device flags; the full exchange at sync(), which
   every reader of the field calls first -- collective); with an RCCL
   communicator, one broadcast of every rank's slots per call instead;
 - colour shard (NNGP_ENGINE=colors, or when the tiles do not fit): one
   launch per colour and an RCCL all-gather of the colour's values.

The reference sweeps a colour class at a time (Scripts/mcmc_nngp_update_Gaussian.R:261-275);
the locations of one class are conditionally independent, so each rank (one
process per GPU) sweeps its spatial block of every class and, after each
class, the ranks all-gather the class's new values over xGMI (RCCL inside
libnngp.so, on the context's stream -- no per-colour Python).  Every rank
keeps a replica of the latent field, so the rest of the hot path (factor,
log-likelihood, ...) runs unchanged on each rank.  Results are bitwise equal
to a single rank.

    ctx = ShardContext(locs, NNarray, coloring, locs_match, y, n_ranks=W, rank=r, device=local_rank)
    init_shard_comm(ctx, torch.distributed)      # RCCL communicator of the shard
    ctx.factor(0, covfun, covparms); ctx.set_field(f); ctx.set_mu(None, beta0)
    ctx.sweep_chains(10, ...)                    # collective over the W ranks

``sweep_chains_group`` runs all ranks of a shard inside one process (device
copies instead of RCCL): the single-box test path, and a single-process
multi-GPU mode.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import IPC_HANDLE_BYTES, SHARD_ID_BYTES, check, lib
from .context import ChainContext


class ShardContext(ChainContext):
    """Rank ``rank`` of an ``n_ranks``-way sharded context (tile shard, or
    colour shard with NNGP_ENGINE=colors).  Same interface as ChainContext."""

    def __init__(self, locs, NNarray, coloring, locs_match, observed_field, n_ranks: int, rank: int,
                 device: int = -1, n_chains: int = 1):
        super().__init__(locs, NNarray, coloring, locs_match, observed_field, device=device, n_chains=n_chains,
                         _shard=(n_ranks, rank))
        self.n_ranks, self.rank = int(n_ranks), int(rank)

    def comm_init(self, uid: bytes) -> None:
        """Collective over the ranks: the RCCL communicator of the shard."""
        assert len(uid) >= SHARD_ID_BYTES
        self._chk(lib.nngp_shard_comm_init(self._h, bytes(uid), len(uid)))

    @property
    def tile_shard(self) -> bool:
        return self.info["sweep_engine"] == 1

    def ipc_handle(self) -> bytes:
        """Tile shard: the HIP IPC handle of this rank's granule buffer."""
        buf = C.create_string_buffer(IPC_HANDLE_BYTES)
        self._chk(lib.nngp_shard_ipc_handle(self._h, buf, IPC_HANDLE_BYTES))
        return buf.raw

    def ipc_open(self, handles) -> None:
        """Tile shard: map the other ranks' granule buffers (handles in rank order)."""
        assert len(handles) == self.n_ranks and all(len(h) == IPC_HANDLE_BYTES for h in handles)
        self._chk(lib.nngp_shard_ipc_open(self._h, b"".join(handles), IPC_HANDLE_BYTES))


    def sync(self) -> None:
        """Collective over the ranks (tile shard without a communicator): the
        full exchange of the field replicas (nngp_shard_sync); a no-op when
        the replica is up to date."""
        self._chk(lib.nngp_shard_sync(self._h))


# The library refuses to read a stale replica (nngp_shard_sync is explicit);
# in Python every reader of the field syncs first, so on a tile shard without
# a communicator these methods are collective: every rank calls them, in the
# same order relative to its sweeps (SPMD).
def _sync_first(name):
    base = getattr(ChainContext, name)

    def f(self, *a, **kw):
        self.sync()
        return base(self, *a, **kw)

    f.__name__, f.__doc__ = name, (base.__doc__ or "") + " (collective on a tile shard: syncs the replicas first)"
    return f


for _name in ("get_field", "record_field", "loglik", "loglik_chains", "ancillary_propose", "ancillary_propose_chains",
              "accept_field", "beta0_stats", "field_response_ratio", "field_response_ratio_chains",
              "sum_squared_residuals", "sum_squared_residuals_chains", "loglik_pair_chains", "ancillary_step_chains",
              "sufficient_step_chains"):
    setattr(ShardContext, _name, _sync_first(_name))


def shard_unique_id() -> bytes:
    buf = C.create_string_buffer(SHARD_ID_BYTES)
    check(lib.nngp_shard_unique_id(buf, SHARD_ID_BYTES))
    return buf.raw


def broadcast_unique_id(dist) -> bytes:
    """Rank 0's RCCL unique id on every rank of the torch.distributed group
    (any backend; gloo is enough)."""
    obj = [shard_unique_id() if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def _agreed(dist, fn):
    """fn() on every rank, then agreement over the group: if it raised on any
    rank, every rank raises (no rank goes on to a step its peers never reach)."""
    res, err = None, None
    try:
        res = fn()
    except Exception as e:  # noqa: BLE001 -- re-raised below on every rank
        err = f"{type(e).__name__}: {e}"
    errs = [None] * dist.get_world_size()
    dist.all_gather_object(errs, err)
    bad = [(r, e) for r, e in enumerate(errs) if e is not None]
    if bad:
        raise RuntimeError("shard setup failed: " + "; ".join(f"rank {r}: {e}" for r, e in bad))
    return res


def _same_everywhere(dist, value, what: str):
    """The rank-local `value` (a picklable decision every rank makes on its
    own, e.g. the chain groups of context.split_groups) must be the same on
    every rank: ranks that went different ways would wait for peers that
    never come.  Raises on every rank if any differs."""
    vals = [None] * dist.get_world_size()
    dist.all_gather_object(vals, value)
    if any(v != vals[0] for v in vals):
        raise RuntimeError(f"shard setup: ranks disagree on {what}: " +
                           "; ".join(f"rank {r}: {v}" for r, v in enumerate(vals)))
    return value


def init_shard_comm(ctx: ShardContext, dist, rccl: bool = True) -> None:
    """Collective over the torch.distributed group: the RCCL communicator and,
    for a tile shard, the exchange of the IPC handles (every step agreed by
    all ranks before the next).  rccl=False (tile shard only): no
    communicator, w is exchanged by peer copies and device flags -- the form
    that also runs with several ranks on one GPU."""
    if ctx.n_ranks > 1:
        if rccl or not ctx.tile_shard:
            uid = broadcast_unique_id(dist)
            _agreed(dist, lambda: ctx.comm_init(uid))
        if ctx.tile_shard:
            handles = [None] * ctx.n_ranks
            dist.all_gather_object(handles, _agreed(dist, ctx.ipc_handle))
            _agreed(dist, lambda: ctx.ipc_open(handles))


def sweep_chains_group(ctxs, n_sweeps: int, beta0, log_scale, log_noise_variance, seed, counter_base) -> None:
    """n_sweeps sharded sweeps of every chain, all ranks of the shard in this
    process (ctxs[g] = rank g)."""
    G = len(ctxs)
    hs = (C.c_void_p * G)(*[c._h.value for c in ctxs])
    a = ctxs[0]._chain_args(beta0, log_scale, log_noise_variance, seed, counter_base)
    check(lib.nngp_sweep_chains_group(hs, G, int(n_sweeps), *a), ctxs[0]._h)
