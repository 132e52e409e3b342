"""cProfile of the bench's MCMC-iterations measurement (host-side time of
the lockstep chain driver; diagnostic).  `--no-cprofile`: the same
iterations without the profiler (for rocprofv3 --hip-trace timelines)."""
import cProfile
import pstats
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, 1_000_000, 15, "matern15_isotropic", cp, seed=5, device=0, chains=3)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 3, seed=3)
wl["field0"] = ctx.get_field()
sync = lambda: torch.cuda.synchronize(0)  # noqa: E731
bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 2, 1, sync)
if "--no-cprofile" in sys.argv:
    print(bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 10, 1, sync), flush=True)
    ctx.close()
    sys.exit(0)
pr = cProfile.Profile()
pr.enable()
r = bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 10, 1, sync)
pr.disable()
print(r)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
