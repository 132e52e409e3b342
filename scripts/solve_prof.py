"""Ancillary proposal (SpMV + triangular solve) at the bench workload, for a
kernel trace: 3 chains batched, repeated (diagnostic)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
C = 3
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, 15, "matern15_isotropic", cp, seed=5, device=0, chains=1)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, C, seed=3)
for k in range(C):
    ctx.select(k).factor(1, "matern15_isotropic", [1.0, 0.051, 0.0])
for _ in range(10):
    ctx.ancillary_propose_chains(7, [1.0] * C, [0.01] * C)
ctx.close()
