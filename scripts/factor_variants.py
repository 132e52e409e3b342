"""Factor kernel variants (NNGP_FACTOR_V = 0..3) at the bench workload, for a
kernel trace (diagnostic): 10 factors each, Linv compared with variant 0."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, 1_000_000, 15, "matern15_isotropic", cp, seed=5, device=0, chains=1)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 1, seed=3)
ref = None
for v in range(4):
    os.environ["NNGP_FACTOR_V"] = str(v)
    for _ in range(10):
        ctx.factor(1, "matern15_isotropic", [1.3, 0.051, 0.0])
    L = ctx.get_linv(1)
    if ref is None:
        ref = L
    print(v, "max rel diff vs V0", float(np.max(np.abs(L - ref) / (np.abs(ref) + 1e-300))), flush=True)
ctx.close()
