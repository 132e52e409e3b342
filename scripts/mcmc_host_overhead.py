"""Host-side cost of the MCMC driver (update_gaussian.py) without a GPU
(diagnostic): every device call is a no-op fake returning plausible values,
so the time measured is the Python host logic of the reference's per-chain
iteration (MH steps, adaptation, records) and the lockstep batching.
Usage: mcmc_host_overhead.py [iterations] [chains] [n]  (cProfile top 25)"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _pkgload  # noqa: E402

P = _pkgload.load()
from nngp_amd.context import ChainView  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
C = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000


class FakeCtx:
    """The device context's interface with no device behind it."""

    def __init__(self, n, C):
        self.n, self.d, self.b, self.n_obs, self.n_chains = n, 2, 16, n, C
        self.cur = 0
        self.field = np.zeros(n)
        self.rng = np.random.default_rng(0)

    def select(self, k):
        self.cur = k
        return self

    def factor(self, which, covfun, cp):
        pass

    def set_field(self, f):
        pass

    def get_field(self):
        return self.field

    def set_mu(self, mu, b0):
        pass

    def records_reserve(self, k):
        pass

    def record_field(self, row):
        pass

    def records_stream(self, host):  # the rows land behind the stream (no host work here)
        pass

    def get_records(self, row0, k, out=None):
        return out

    def accept_field(self):
        pass

    def accept_factor(self):
        pass

    def beta0_stats(self):
        return 1e6, 1e3

    def factor_chains(self, which, mask, covfun, cps):
        return np.zeros(self.n_chains, np.int32)

    def ancillary_propose_chains(self, mask, b0, dls):
        pass

    def field_response_ratio_chains(self, mask, b0, lnv):
        return self.rng.normal(size=self.n_chains)

    def loglik_chains(self, which, mask, b0, ls):
        return self.rng.normal(size=self.n_chains)

    def loglik_pair_chains(self, mask, b0, lsp, lsc):
        return self.rng.normal(size=self.n_chains), self.rng.normal(size=self.n_chains)

    def ancillary_step_chains(self, mask, covfun, cps, b0, dls, lnv):
        return np.zeros(self.n_chains, np.int32), self.rng.normal(size=self.n_chains)

    def sufficient_step_chains(self, mask, covfun, cps, b0, lsp, lsc):
        return (np.zeros(self.n_chains, np.int32), self.rng.normal(size=self.n_chains),
                self.rng.normal(size=self.n_chains))

    def sum_squared_residuals_chains(self, mask, b0):
        return np.full(self.n_chains, 0.25 * self.n)

    def sweep_chains(self, *a):
        pass


fake = FakeCtx(n, C)
views = [ChainView(fake, k) for k in range(C)]
va = {"NNarray": None, "coloring": None, "locs_match": np.arange(1, n + 1, dtype=np.int32), "n_obs": n, "n_locs": n}
stm = {"response_model": "Gaussian", "covfun": {"stationary_covfun": "matern15_isotropic", "shape_params": ["log_range"]}}
states = {f"chain_{k + 1}": {"params": {"shape": np.array([np.log(0.05)]), "beta_0": 1.0, "beta": None,
                                        "log_scale": 0.0, "log_noise_variance": np.log(0.25),
                                        "field": np.zeros(n)},
                             "transition_kernels": {"covariance_params_sufficient": {"logvar": -4.0},
                                                    "covariance_params_ancillary": {"logvar": -4.0},
                                                    "log_noise_variance": {"logvar": -1.0}}} for k in range(C)}
X = {"X": None, "locs": np.zeros(0, np.int64)}
y = np.random.default_rng(1).normal(size=n)
P.mcmc_nngp_update_Gaussian(None, X, y, stm, va, states, 2, contexts=views)
t = time.perf_counter()
P.mcmc_nngp_update_Gaussian(None, X, y, stm, va, states, iters, contexts=views, iterations=np.array([[2, 0.0]]),
                            field_thinning=float(os.environ.get("THIN", "1")))
el = time.perf_counter() - t
print(f"unprofiled: {el * 1e3 / iters:.3f} ms per iteration")
t = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
P.mcmc_nngp_update_Gaussian(None, X, y, stm, va, states, iters, contexts=views, iterations=np.array([[2, 0.0]]),
                            field_thinning=float(os.environ.get("THIN", "1")))
pr.disable()
el = time.perf_counter() - t
print(f"{iters} iterations x {C} chains: {el * 1e3 / iters:.3f} ms of host time per iteration (profiled)")
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
