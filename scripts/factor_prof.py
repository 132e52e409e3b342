"""The Vecchia factor at the bench workload, repeated (for kernel traces and
SQ counter passes; diagnostic)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 15
covfun = sys.argv[3] if len(sys.argv) > 3 else "matern15_isotropic"
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, covfun, cp, seed=5, device=0, chains=1)
ctx = bench.open_context(P, wl, covfun, cp, 0, 1, seed=3)
for k in range(10):
    ctx.factor(1, covfun, [1.0, 0.05 + 0.001 * k, 0.0])
ctx.close()
