"""Diagnostic: one/three sweeps of the tile engine vs the oracle, error by colour."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import _pkgload
import oracle as O
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import make_problem

P = _pkgload.load()
n, m = int(sys.argv[1]), int(sys.argv[2])
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 1
locs, NN, col, lm, y = make_problem(P, n, m, seed=0)
cp = [1.0, 0.08, 0.0]
rng = np.random.default_rng(1)
field = rng.normal(size=n)
z = rng.normal(size=(ns, n))
with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
    print("info", {k: v for k, v in ctx.info.items() if k in ("sweep_engine", "n_tiles", "tile_rows_max", "n_ghost_cells", "n_colors")})
    ctx.factor(0, "exponential_isotropic", cp)
    ctx.set_field(field)
    ctx.set_mu(None, 0.4)
    ctx.sweep(ns, 0.4, 0.3, -0.2, 1, 0, z=z)
    got = ctx.get_field()
    Lo = ctx.get_linv(0)
    Dd = ctx.precision_diag() if hasattr(ctx, "precision_diag") else None
D = O.precision_diag(Lo, NN)
if Dd is not None:
    print("D maxdiff", np.abs(Dd - D).max())
ref = O.sweep("local", field, Lo, NN, col, D, np.ones(n, np.int32), y, np.full(n, 0.4), lm, 0.4, 0.3, -0.2, z)
err = np.abs(got - ref)
print("max err", err.max())
for c in range(1, col.max() + 1):
    e = err[col == c]
    print(f"colour {c}: n={len(e)} bad={(e > 1e-9).sum()} max={e.max():.3e}")
