"""Device time of the calls one Gibbs iteration of update_Gaussian.R makes,
at the bench workload (diagnostic): factor, loglik, ancillary proposal
(SpMV + triangular solve), beta_0 stats, SSR, n_chromatic sweeps."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, 15, "matern15_isotropic", cp, seed=5, device=0, chains=1)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 1, seed=3)


def t(name, f, reps=5):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    print(f"{name:28s} {1e3 * (time.perf_counter() - t0) / reps:8.3f} ms", flush=True)


t("factor (proposal)", lambda: ctx.factor(1, "matern15_isotropic", [1.0, 0.051, 0.0]))
t("loglik", lambda: ctx.loglik(1, 1.0, 0.0))
t("ancillary_propose", lambda: ctx.ancillary_propose(1.0, 0.01))
t("beta0_stats", lambda: ctx.beta0_stats())
t("sum_squared_residuals", lambda: ctx.sum_squared_residuals(1.0))
t("sweep x10 (1 chain)", lambda: ctx.sweep(10, 1.0, 0.0, np.log(0.25), 7, 0))
ctx.close()

# 3 chains in one context: per-chain calls vs the batched ones
C = 3
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, C, seed=3)
for k in range(C):
    ctx.select(k).factor(1, "matern15_isotropic", [1.0, 0.051, 0.0])


def anc_seq():
    for k in range(C):
        ctx.select(k).ancillary_propose(1.0, 0.01)


t("ancillary x3 per chain", anc_seq)
t("ancillary_propose_chains x3", lambda: ctx.ancillary_propose_chains(7, [1.0] * C, [0.01] * C))
t("sweep_chains x10 (3 chains)", lambda: ctx.sweep_chains(10, [1.0] * C, [0.0] * C, [np.log(0.25)] * C,
                                                          [7, 8, 9], [0] * C))
ctx.close()
