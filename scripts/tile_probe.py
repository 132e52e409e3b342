"""Tile engine phase times (NNGP_PROBE=9 build path): per tile, microseconds
spent in own batches / prefetch / ghost hand-off, over one call of
n_chromatic sweeps at the bench workload.  Usage: tile_probe.py [n] [m] [chains]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ["NNGP_PROBE"] = "9"
out = "/tmp/tile_probe.bin"
os.environ["NNGP_DBG_OUT"] = out
import _pkgload  # noqa: E402
import bench  # noqa: E402

P = _pkgload.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 15
C = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, "matern15_isotropic", cp, seed=1000, device=0, chains=C)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, C, seed=7)
info = ctx.info
print({k: info[k] for k in ("sweep_engine", "n_tiles", "tile_rows_max", "n_ghost_cells", "n_colors")})
args = ([wl["beta0"]] * C, [wl["log_scale"]] * C, [wl["log_noise_variance"]] * C, [77 + k for k in range(C)])
for rep in range(3):
    t = time.perf_counter()
    ctx.sweep_chains(10, *args, [rep * 10] * C)
    el = time.perf_counter() - t
    d = np.fromfile(out, dtype=np.uint64).reshape(-1, 8).astype(np.float64) / 100.0  # 100 MHz -> us
    names = ["items", "products", "totals", "draw", "scatter", "prefetch", "ghost", "init"]
    print(f"call {rep}: {el*1e3:.3f} ms wall; per tile us mean(max): " +
          " ".join(f"{nm} {d[:, k].mean():.0f}({d[:, k].max():.0f})" for k, nm in enumerate(names)))
ctx.close()
