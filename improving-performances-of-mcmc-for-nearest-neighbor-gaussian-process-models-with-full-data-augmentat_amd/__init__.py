"""MI355X-native NNGP chromatic-Gibbs hot path (drop-in for the reference's
``mcmc_nngp_*`` surface; see DESIGN.md / INTEGRATION.md).

The array work runs in ``libnngp.so`` (hand-written HIP for gfx950 behind the
C ABI of include/nngp.h); this package is the host-side mirror of the
reference's R functions.
"""
from ._lib import COVFUNS, NNGPError, lib  # noqa: F401  (fails loudly without libnngp.so)
from .graph import find_ordered_nn, naive_greedy_coloring, order_maxmin, sparse_chol_indices  # noqa: F401
from .context import ChainContext  # noqa: F401
from .shard import ShardContext, init_shard_comm, sweep_chains_group  # noqa: F401
from .initialize import mcmc_nngp_initialize  # noqa: F401
from .update_gaussian import mcmc_nngp_update_Gaussian, ll_compressed_sparse_chol  # noqa: F401
from .run import mcmc_nngp_run  # noqa: F401
from .estimate import mcmc_nngp_estimate, get_summary  # noqa: F401
from .predict import mcmc_nngp_predict_field, mcmc_nngp_predict_fixed_effects  # noqa: F401
from .diagnose import Gelman_Rubin_Brooks, ESS  # noqa: F401

__all__ = [
    "mcmc_nngp_initialize", "mcmc_nngp_run", "mcmc_nngp_update_Gaussian",
    "mcmc_nngp_estimate", "mcmc_nngp_predict_field", "mcmc_nngp_predict_fixed_effects",
    "ll_compressed_sparse_chol", "ChainContext", "find_ordered_nn", "naive_greedy_coloring",
    "order_maxmin", "Gelman_Rubin_Brooks", "ESS", "get_summary",
]
