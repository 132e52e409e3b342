"""Chain groups on one GPU (diagnostic bench line): the chains of a
workload in ONE context (whatever engine it gets) against the groups that
context.make_chain_views opens when that context's tiles exceed the LDS
(context._open_group: halves, each on the tile engine).  configs[4]'s
per-GPU share is `chain_groups_bench.py 1250000 20 3`: one 3-chain context
runs the colour engine (its tiles need ~168 KB of LDS), the split runs a
2-chain and a 1-chain tile context one after the other.  A step = one sweep
of every chain (calls of n_chromatic = 10 sweeps, warm as in bench.py);
value = chain-sweeps/s.  Prints one JSON line per arm.
Usage: chain_groups_bench.py [n] [m] [chains] [steps]"""
import json
import os
import sys
import time

import numpy as np
import torch  # before libnngp: the process's HIP runtime is torch's (as in bench.py)

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _pkgload  # noqa: E402
import bench  # noqa: E402

P = _pkgload.load()
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_250_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 20
C = int(sys.argv[3]) if len(sys.argv) > 3 else 3
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 60
nc = 10
covfun, cp = "matern15_isotropic", [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, covfun, cp, seed=1000, device=0, chains=C)
seeds = [77 + k for k in range(C)]
b0, ls, lnv = wl["beta0"], wl["log_scale"], wl["log_noise_variance"]


def prepare(ctx, first):
    rng = np.random.default_rng(7 + first)
    for k in range(ctx.n_chains):
        ctx.select(k)
        ctx.factor(0, covfun, cp)
        ctx.set_field(b0 + wl["w"] + 0.1 * rng.normal(size=len(wl["y"])))
        ctx.set_mu(None, b0)
    ctx.select(0)


def run_groups(groups, label):
    """groups: [(ctx, [chain ids])]; every step sweeps each group in turn."""
    def run(nsw, base):
        done = 0
        while done < nsw:
            s = min(nc, nsw - done)
            for ctx, ids in groups:
                k = len(ids)
                ctx.sweep_chains(s, [b0] * k, [ls] * k, [lnv] * k, [seeds[i] for i in ids], [base + done] * k)
            done += s
        return base + done

    for _ in range(8):  # prime every call shape (graph capture) before the timed region
        run(nc, 1 << 40)
    el, _ = bench.timed_region(run, steps, 10, None, lambda: torch.cuda.synchronize(0))
    engines = [("tiles" if ctx.info["sweep_engine"] == 1 else "colours") + f" x{len(ids)}" for ctx, ids in groups]
    print(json.dumps({"arm": label, "value": steps * C / el, "unit": "chain-sweeps/s", "ms_per_step": el * 1e3 / steps,
                      "n": n, "m": m, "chains": C, "contexts": engines}), flush=True)


torch.cuda.init()
t = time.time()
one = P.ChainContext(wl["locs"], wl["NN"], wl["col"], wl["lm"], wl["y"], device=0, n_chains=C)
print(f"# one {C}-chain context: {one.info['engine_note']} ({time.time() - t:.1f} s)", flush=True)
prepare(one, 0)
run_groups([(one, list(range(C)))], "one context")
one.close()
groups = P.context._open_group(wl["locs"], wl["NN"], wl["col"], wl["lm"], wl["y"], 0, list(range(C)))
for ctx, ids in groups:
    prepare(ctx, ids[0])
run_groups(groups, "split groups")
for ctx, _ in groups:
    ctx.close()
