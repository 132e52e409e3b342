"""Wall time per synced Vecchia factor (diagnostic): n, m from argv (default
1e6, 20), Matern 3/2, one chain, 3 warm-up + 10 timed factors."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import _pkgload  # noqa: E402

P = _pkgload.load()
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, "matern15_isotropic", cp, seed=5, device=0, chains=1)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 1, seed=3)
for _ in range(3):
    ctx.factor(1, "matern15_isotropic", [1.3, 0.051, 0.0])
t = time.perf_counter()
for _ in range(10):
    ctx.factor(1, "matern15_isotropic", [1.3, 0.051, 0.0])
print(f"n={n} m={m}: {(time.perf_counter() - t) / 10 * 1e3:.3f} ms per factor (wall, synced)", flush=True)
ctx.close()
