"""A/B of the factor kernels (diagnostic): the one-lane-per-row
factor_kernel against the 16-lane-group factor_lanes_kernel
(NNGP_FACTOR_LANES=16) on the MCMC's multi-chain factor call -- 3 jobs (one
per chain, different parameters) in one launch, n = 1e6, m = 15 (argv: n m),
Matern 3/2 -- wall time per synced call, variants interleaved.  Run under
rocprofv3 --kernel-trace --stats for the per-kernel durations."""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 15
cov = "matern15_isotropic"
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, cov, cp, seed=5, device=0, chains=3)
ctx = bench.open_context(P, wl, cov, cp, 0, 3, seed=3)
cps = np.array([[1.3, 0.051, 0.0], [1.1, 0.049, 0.0], [0.9, 0.052, 0.0]])
res = {"one-lane": [], "lanes16": []}
for rep in range(3):
    for name in res:
        if name == "lanes16":
            os.environ["NNGP_FACTOR_LANES"] = "16"
        else:
            os.environ.pop("NNGP_FACTOR_LANES", None)
        for _ in range(3):
            ctx.factor_chains(1, 7, cov, cps)
        t = time.perf_counter()
        for _ in range(10):
            st = ctx.factor_chains(1, 7, cov, cps)
        res[name].append((time.perf_counter() - t) / 10 * 1e3)
        assert (st == 0).all()
        print(f"rep {rep} {name:9s} {res[name][-1]:.3f} ms per 3-job factor call (wall, synced)", flush=True)
os.environ["NNGP_FACTOR_LANES"] = "16"
ctx.factor_chains(1, 7, cov, cps)
a = [ctx.select(k).get_linv(1) for k in range(3)]
os.environ.pop("NNGP_FACTOR_LANES", None)
ctx.factor_chains(1, 7, cov, cps)
b = [ctx.select(k).get_linv(1) for k in range(3)]
print("max |lanes16 - one-lane| / max|one-lane| per chain:",
      [float(np.abs(x - y).max() / np.abs(y).max()) for x, y in zip(a, b)])
print({k: float(np.median(v)) for k, v in res.items()})
ctx.close()
