"""A/B of context-creation environment variants of the sweep on one workload
(diagnostic; the workload is built once).  Each variant: a context with the
variant's environment, its call shapes captured, then `steps` sweeps of every
chain in calls of 10 (warm) and the sweep kernel's launch time (HIP events,
median of 5).  Variants run interleaved, `reps` rounds.
Usage: ab_env.py CHAINS STEPS REPS 'NAME:VAR=V,VAR=V' ['NAME:...' ...]
(env NNGP_AB_N / NNGP_AB_M: workload size, default 1e6 / 15)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import _pkgload  # noqa: E402
import bench  # noqa: E402

P = _pkgload.load()
C, steps, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
variants = []
for spec in sys.argv[4:]:
    name, _, kv = spec.partition(":")
    env = dict(x.split("=", 1) for x in kv.split(",") if x)
    variants.append((name, env))
n = int(float(os.environ.get("NNGP_AB_N", "1e6")))
m = int(os.environ.get("NNGP_AB_M", "15"))
cp = [1.0, 0.05, 0.0]
t = time.time()
wl = bench.make_workload(P, n, m, "matern15_isotropic", cp, seed=1000, device=0, chains=C)
print(f"workload n={n} m={m} {time.time() - t:.1f}s", flush=True)
b0, ls, lnv = wl["beta0"], wl["log_scale"], wl["log_noise_variance"]
seeds = [77 + k for k in range(C)]
res = {name: [] for name, _ in variants}
for rep in range(reps):
    for name, env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, C, seed=7)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        args = ([b0] * C, [ls] * C, [lnv] * C, seeds)
        for _ in range(3):
            ctx.sweep_chains(10, *args, [0] * C)
        ctx.get_field()
        t0 = time.perf_counter()
        for i in range(steps // 10):
            ctx.sweep_chains(10, *args, [10 * i] * C)
        ctx.get_field()
        el = time.perf_counter() - t0
        kms = []
        for r in range(5):
            _, k = ctx.sweep_timed(10, *args, [r * 10] * C, per_kernel=True)
            kms.append(k)
        out = {"chain_sweeps_s": steps * C / el, "kernel_us": float(np.median(kms)) * 1e3,
               "engine": ctx.info["sweep_engine"]}
        ctx.close()
        res[name].append(out)
        print(f"rep {rep} {name:12s} {out['chain_sweeps_s']:9.1f} chain-sweeps/s  kernel {out['kernel_us']:8.1f} us"
              + (f"  [{out['engine']}]" if rep == 0 else ""), flush=True)
summ = {name: {"chain_sweeps_s": [r["chain_sweeps_s"] for r in v], "kernel_us": [r["kernel_us"] for r in v]}
        for name, v in res.items()}
print(json.dumps(summ))
