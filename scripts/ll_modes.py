"""Row-statistics (log-likelihood) passes by mode, headline workload, 3 chains:
alternates a pass over a fresh proposal factor (mode 1: the factor's log
determinant summed in the pass) and a pass over the current factor (mode 2:
log determinant cached).  Run under rocprofv3 --kernel-trace; the dispatches
of row_stats_jobs_kernel alternate 1, 2, 1, 2, ...  (diagnostic)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _pkgload  # noqa: E402
import bench  # noqa: E402

P = _pkgload.load()
n, m, C = 1_000_000, 15, 3
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, "matern15_isotropic", cp, seed=1000, device=0, chains=C)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, C, seed=7)
mask = (1 << C) - 1
for rep in range(12):
    cps = np.tile([1.0, 0.05 * (1 + 0.01 * rep), 0.0], (C, 1))
    ctx.factor_chains(1, mask, "matern15_isotropic", cps)
    ctx.loglik_chains(1, mask, [0.1] * C, [0.0] * C)
    ctx.loglik_chains(0, mask, [0.1] * C, [0.0] * C)
print("done")
ctx.close()
