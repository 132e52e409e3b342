"""Colour-sharded chromatic sweep: ONE set of chains swept by several GPUs
(DESIGN.md §6).

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

from ._lib import SHARD_ID_BYTES, check, lib
from .context import ChainContext


class ShardContext(ChainContext):
    """Rank ``rank`` of an ``n_ranks``-way colour-sharded context (the
    colour-launch sweep engine).  Same interface as ChainContext."""

    def __init__(self, locs, NNarray, coloring, locs_match, observed_field, n_ranks: int, rank: int,
                 device: int = -1, n_chains: int = 1):
        super().__init__(locs, NNarray, coloring, locs_match, observed_field, device=device, n_chains=n_chains,
                         _shard=(n_ranks, rank))
        self.n_ranks, self.rank = int(n_ranks), int(rank)

    def comm_init(self, uid: bytes) -> None:
        """Collective over the ranks: the RCCL communicator of the shard."""
        assert len(uid) >= SHARD_ID_BYTES
        self._chk(lib.nngp_shard_comm_init(self._h, bytes(uid), len(uid)))


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


def init_shard_comm(ctx: ShardContext, dist) -> None:
    if ctx.n_ranks > 1:
        ctx.comm_init(broadcast_unique_id(dist))


def sweep_chains_group(ctxs, n_sweeps: int, beta0, log_scale, log_noise_variance, seed, counter_base) -> None:
    """n_sweeps sharded sweeps of every chain, all ranks of the shard in this
    process (ctxs[g] = rank g)."""
    G = len(ctxs)
    hs = (C.c_void_p * G)(*[c._h.value for c in ctxs])
    a = ctxs[0]._chain_args(beta0, log_scale, log_noise_variance, seed, counter_base)
    check(lib.nngp_sweep_chains_group(hs, G, int(n_sweeps), *a), ctxs[0]._h)
