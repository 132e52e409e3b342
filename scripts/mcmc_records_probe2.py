"""cProfile of 40 MCMC iterations (3 chains, n = 1e6) with field_thinning 1:
where the host time goes beyond the GPU timeline."""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import _pkgload
import bench

P = _pkgload.load()
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, 1_000_000, 15, "matern15_isotropic", cp, seed=1000, device=0, chains=3)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 3, seed=7)
wl["field0"] = ctx.get_field()
sync = lambda: torch.cuda.synchronize(0)  # noqa: E731
bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 5, 2, sync)
pr = cProfile.Profile()
pr.enable()
r = bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 40, 2, sync)
pr.disable()
print(r)
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
import re
print("\n".join(re.sub(r"/\S*/", "", ln) for ln in s.getvalue().splitlines()[:45]))
