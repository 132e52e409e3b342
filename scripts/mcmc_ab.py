"""Interleaved A/B of the bench's MCMC-iterations measurement (3 chains,
n = 1e6, m = 15, 40 iterations per update call as in bench.py) over values
of one environment variable read per update call (diagnostic).
Usage: mcmc_ab.py VAR v1 v2 [rounds]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402  (before libnngp, as in bench.py)

import bench  # noqa: E402
import _pkgload  # noqa: E402

var, vals = sys.argv[1], sys.argv[2:4]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
P = _pkgload.load()
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, 1_000_000, 15, "matern15_isotropic", cp, seed=5, device=0, chains=3)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, 3, seed=3)
wl["field0"] = ctx.get_field()
sync = lambda: torch.cuda.synchronize(0)  # noqa: E731
res = {v: [] for v in vals}
for r in range(rounds):
    for v in vals:
        os.environ[var] = v
        out = bench.mcmc_iterations(P, wl, "matern15_isotropic", cp, ctx, 40, 2, sync)
        res[v].append(out["ms_per_iteration"])
        print(f"round {r} {var}={v}: {out['ms_per_iteration']:.3f} ms/it ({out['value']:.1f} it/s)", flush=True)
for v in vals:
    print(f"{var}={v}: best {min(res[v]):.3f} ms/it, all {[round(x, 3) for x in res[v]]}")
