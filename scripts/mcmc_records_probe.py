"""Where the MCMC call's time goes beyond the GPU timeline: the same 40
iterations with field_thinning 1 (a record per iteration, the reference's
default) and 0.025 (one record), plus the D2H of one chain's records."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import _pkgload
import bench

P = _pkgload.load()
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, 1_000_000, 15, "matern15_isotropic", cp, seed=1000, device=0, chains=3)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 3, seed=7)
wl["field0"] = ctx.get_field()
sync = lambda: torch.cuda.synchronize(0)  # noqa: E731
orig = P.mcmc_nngp_update_Gaussian
for ft in (1.0, 0.025, 1.0):
    P.mcmc_nngp_update_Gaussian = lambda *a, **k: orig(*a, **{**k, "field_thinning": ft})  # noqa: B023
    r = bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 40, 2, sync)
    print(f"field_thinning {ft}: {r['value']:.1f} it/s, {r['ms_per_iteration']:.2f} ms/it", flush=True)
v = ctx.view(0)
v.records_reserve(40)
for i in range(40):
    v.record_field(i)
sync()
t = time.perf_counter()
out = v.get_records(0, 40)
print(f"get_records 40 x 1e6 (pageable np.zeros): {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
buf = np.empty((40, 1_000_000))
t = time.perf_counter()
buf[:] = out
print(f"host copy of the same: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
v.records_reserve(0)
