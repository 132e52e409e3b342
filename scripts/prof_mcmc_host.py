import cProfile, pstats, sys, io
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import numpy as np, torch
import _pkgload, bench
P = _pkgload.load()
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, 1_000_000, 15, "matern15_isotropic", cp, seed=1000, device=0, chains=3)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 3, seed=7)
wl["field0"] = ctx.get_field()
sync = lambda: torch.cuda.synchronize(0)
bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 3, 2, sync)
pr = cProfile.Profile(); pr.enable()
r = bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 20, 2, sync)
pr.disable()
print(r)
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18); print(s.getvalue()[:5000])
