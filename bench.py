#!/usr/bin/env python
"""Headline benchmark: full-field chromatic Gibbs sweeps/sec at n=1e6, m=15
(synthetic 2-D Matern-3/2 field, fp64), with the sweep kernel's achieved
bandwidth against the MI355X HBM roofline and the CPU oracle's
reference-faithful sweep timed on the host beside it.

Contract: python bench.py --gpus N --steps K --warmup W  (N>1 under
torch.distributed.run; one rank per GPU).  A step = one chromatic sweep (all K
colours, all n latents, update_Gaussian.R:257-275 with n_chromatic = 1) of
each of the --chains chains of the GPU (default 3 = the reference's default
n_chains, initialize.R:9, which it runs concurrently with mclapply).  The
chains of a GPU share one context and sweep in the same kernels
(nngp_sweep_chains).  value = chain-sweeps/s over all GPUs.  The timed region
runs the reference's per-iteration call shape: n_chromatic = 10 sweeps per
call.  Calls back to back with the field, factor and beta_0 unchanged are
"warm" (the call starts from the slot-order w and r = B w the previous call
left; DESIGN.md §3 "Round 3", pinned to cold calls by
tests/test_gpu_warm_calls.py); every call shape the timed region uses is
captured as a hipGraph before it (cold and warm), so no capture lands inside
t0..t1.  The cold rate (r = B w rebuilt every call, what an MCMC iteration
runs since beta_0 is redrawn every iteration) is timed beside it
("cold_calls" in config), and a single-chain context too ("single_chain").
Multi-GPU (N > 1): the tile-sharded sweep of ONE field whose
size grows with N (n = N x 1e6; every GPU keeps the tile geometry of the
n=1e6 headline): weak scaling, value = chain-sweeps/s x n/1e6.  A small
cross-GPU parity check (N-rank shard == one GPU, bitwise) runs first and is
reported.  --multi shard-strong keeps n fixed; --multi replicas runs
independent chains per GPU (the reference's mclapply -> ranks).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(msg, rank=0):
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def make_workload(P, n, m, covfun, cp, seed, device, chains):
    rng = np.random.default_rng(seed)
    t = time.time()
    locs = rng.uniform(size=(n, 2))
    locs = locs[P.order_maxmin(locs) - 1]
    NN = P.find_ordered_nn(locs, m)
    col = P.naive_greedy_coloring(NN)
    t_graph = time.time() - t
    lm = np.arange(1, n + 1, dtype=np.int32)
    beta0, tau2 = 1.0, 0.25
    # truth: w = B^{-1} z (sigma^2 = 1), y = beta0 + w + eps
    ctx = P.ChainContext(locs, NN, col, lm, np.zeros(n), device=device)
    ctx.factor(0, covfun, cp)
    w = ctx.tri_solve(0, rng.normal(size=n))
    y = beta0 + w + np.sqrt(tau2) * rng.normal(size=n)
    ctx.close()
    wl = dict(locs=locs, NN=NN, col=col, lm=lm, y=y, beta0=beta0, log_noise_variance=np.log(tau2),
              log_scale=0.0, t_graph=t_graph, w=w)
    return wl


def replica_seeds(rank, chains):
    """--multi replicas / N = 1: (workload seed, chain seeds) of a rank -- every
    rank sweeps its own field and chains (weak scaling of independent chains)."""
    return 1000 + rank, [77 + 10 * rank + k for k in range(chains)]


def open_context(P, wl, covfun, cp, device, chains, seed):
    rng = np.random.default_rng(seed)
    ctx = P.ChainContext(wl["locs"], wl["NN"], wl["col"], wl["lm"], wl["y"], device=device, n_chains=chains)
    for k in range(chains):
        ctx.select(k)
        ctx.factor(0, covfun, cp)
        ctx.set_field(wl["beta0"] + wl["w"] + 0.1 * rng.normal(size=len(wl["y"])))
        ctx.set_mu(None, wl["beta0"])
    ctx.select(0)
    return ctx


def cpu_baseline(P, wl, covfun, cp, budget_s, chains):
    """The reference's CPU path restated: the masked-form chromatic sweep
    (update_Gaussian.R:257-275, full masked SpMV + column crossprod per colour)
    of the C oracle, one chain per host thread as the reference runs one chain
    per mclapply worker (update_Gaussian.R:25-26), on the same workload; whole
    sweeps until ~budget_s/2.  ctypes releases the GIL, so the threads run in
    parallel without forking this GPU-initialised process.  The single-thread
    local-form oracle is reported beside it."""
    import threading

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O

    n = len(wl["y"])
    t = time.time()
    Lo = O.vecchia_linv(covfun, cp, wl["locs"], wl["NN"])
    D = O.precision_diag(Lo, wl["NN"])
    t_factor = time.time() - t
    opl = np.ones(n, np.int32)
    mu = np.full(n, wl["beta0"])
    z = O.sweep_normals(3, 0, 1, n)

    def run(form, out, k, threads=1):
        field = np.asarray(wl["field0"]).copy()
        done, t0 = 0, time.time()
        while True:
            field = O.sweep(form, field, Lo, wl["NN"], wl["col"], D, opl, wl["y"], mu, wl["lm"], wl["beta0"],
                            wl["log_scale"], wl["log_noise_variance"], z, threads=threads)
            done += 1
            if time.time() - t0 > budget_s / 2 or done >= 20:
                break
        out[k] = (done, time.time() - t0)

    res = [None] * chains
    th = [threading.Thread(target=run, args=("masked", res, k)) for k in range(chains)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    masked = sum(d / el for d, el in res)
    # one chain on all the host cores the process may use (OMP_NUM_THREADS on
    # the GPU box), masked form and the optimised local form
    # the "all cores" leg runs on the CPUs this process may actually use: its
    # affinity set (the GPU box gives a job a share of a larger host, and
    # OMP_NUM_THREADS names that share), not the host's whole os.cpu_count()
    host_cpus = os.cpu_count() or 1
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host_cpus
    omp_env = int(os.environ.get("OMP_NUM_THREADS") or 0)
    omp = max(1, min(affinity, omp_env) if omp_env > 0 else affinity)
    one, locmt, loc = [None], [None], [None]
    run("masked", one, 0, omp)
    run("local", locmt, 0, omp)
    run("local", loc, 0)
    rate = lambda r: r[0][0] / r[0][1]  # noqa: E731
    return {"value": masked, "unit": "sweeps/s", "cores": chains, "kind": "port",
            "sample": (f"oracle C restatement of the reference's masked-form chromatic sweep "
                       f"(update_Gaussian.R:257-275), {chains} chains on {chains} host threads (the reference's "
                       f"mclapply over chains), same n={n} workload, whole sweeps until ~{budget_s / 2:.0f}s each "
                       f"({sum(d for d, _ in res)} sweeps); 1 chain x {omp} OpenMP threads: masked form "
                       f"{rate(one):.3g}, local form {rate(locmt):.3g} sweeps/s; local form 1 thread "
                       f"{rate(loc):.3g} sweeps/s; oracle factor build {t_factor:.1f}s; host os.cpu_count() "
                       f"{host_cpus}, CPUs in this process's affinity set {affinity}, OMP_NUM_THREADS "
                       f"{omp_env or 'unset'}"),
            "host_cpus": host_cpus,
            "affinity_cpus": affinity,
            "one_chain_all_cores": {"value": rate(one), "threads": omp, "form": "masked"},
            "local_form_all_cores": {"value": rate(locmt), "threads": omp, "form": "local"},
            "local_form_value_1_thread": rate(loc)}


def mcmc_iterations(P, wl, covfun, cp, ctx, iters, warmup, sync):
    """Secondary metric: full MCMC iterations of
    update_Gaussian.R:101-313 (ancillary + sufficient covariance MH steps,
    beta_0 Gibbs step, n_chromatic = 10 sweeps, noise-variance MH, records with
    field_thinning = 1) for every chain of ctx, through the package's
    mcmc_nngp_update_Gaussian (chains driven in lockstep).  -> iterations/s of
    the whole chain set and seconds per iteration."""
    n = len(wl["y"])
    C = ctx.n_chains
    va = {"NNarray": wl["NN"], "coloring": wl["col"], "locs_match": wl["lm"], "n_obs": n, "n_locs": n}
    stm = {"response_model": "Gaussian",
           "covfun": {"stationary_covfun": covfun, "shape_params": ["log_range"]}}
    rng = np.random.default_rng(11)
    states = {}
    for k in range(C):
        states[f"chain_{k + 1}"] = {
            "params": {"shape": np.array([np.log(cp[1]) + 0.05 * rng.normal()]), "beta_0": wl["beta0"],
                       "beta": None, "log_scale": wl["log_scale"],
                       "log_noise_variance": wl["log_noise_variance"], "field": wl["field0"].copy()},
            "transition_kernels": {"covariance_params_sufficient": {"logvar": -4.0},
                                   "covariance_params_ancillary": {"logvar": -4.0},
                                   "log_noise_variance": {"logvar": -1.0}}}
    views = [ctx.view(k) for k in range(C)]
    X = {"X": None, "locs": np.zeros(0, np.int64)}

    def run(it, start):
        out = P.mcmc_nngp_update_Gaussian(wl["locs"], X, wl["y"], stm, va, states, it, contexts=views,
                                          iterations=np.array([[start, 0.0]]))
        for name, r in out.items():
            states[name] = r["state"]
        return out  # the caller keeps the records: freeing them is not part of the update call

    run(warmup, 0)
    sync()
    t0 = time.perf_counter()
    kept = run(iters, warmup)
    sync()
    el = time.perf_counter() - t0
    del kept
    return {"metric": "MCMC iterations/s (update_Gaussian.R:101-313, n_chromatic=10, all chains of the GPU)",
            "value": iters / el, "unit": "iterations/s", "chains": C, "iterations": iters,
            "ms_per_iteration": el * 1e3 / iters, "field_thinning": 1.0,
            "iterations_per_update_call": iters}


def pmc_traffic(chains, n, m, kernel):
    """Per-launch HBM bytes of the sweep kernel from the committed rocprofv3
    PMC summary of the same workload (profiles/): the request-size-resolved
    passes (scripts/pmc_sizes.sh: TCC_EA0_RDREQ_{128B,64B,32B}, WRREQ) where
    a round has them, else FETCH_SIZE and WRITE_SIZE calibrated on known-byte
    kernels (scripts/pmc.sh) -- the latest round's, sized first."""
    best, best_key = None, None
    for f in sorted((ROOT / "profiles").glob("r*_pmc_*.json")):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        w = d.get("workload", {})
        if not isinstance(w, dict):
            continue
        if (w.get("chains") == chains and w.get("n") == n and w.get("m") == m and kernel.startswith(d.get("kernel", "?"))
                and d.get("traffic_bytes_per_launch")):
            key = (f.name[:3], "RDREQ" in d.get("method", ""), f.name)
            if best_key is None or key > best_key:
                best, best_key = (d["traffic_bytes_per_launch"], f.name), key
    return best


def timed_region(run, steps, warmup, dist=None, sync=lambda: None):
    """The bench contract's timed region: `warmup` untimed steps, then exactly
    `steps` steps bracketed by barrier + device sync on both sides; returns
    (max over ranks of the elapsed seconds, run's last return value).
    run(n_steps, counter) -> counter."""
    import torch

    ctr = run(warmup, 0)
    sync()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ctr = run(steps, ctr)
    sync()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, ctr


def shard_parity_check(P, args, world, rank, local_rank, dist):
    """Cross-GPU parity at a small size, run by every rank before the sharded
    measurement: the world-rank tile shard (IPC granule puts over xGMI, halo
    stores into the peers' replicas) against this GPU alone with the same
    tiles, bitwise after two calls (2 + 1 sweeps of 2 chains, nothing read in
    between); -> True on every rank iff every rank matched."""
    import torch

    from nngp_amd.shard import ShardContext, _agreed, init_shard_comm

    n, m, C = 20000, 10, 2
    rng = np.random.default_rng(99)
    locs = rng.uniform(size=(n, 2))
    locs = locs[P.order_maxmin(locs) - 1]
    NN = P.find_ordered_nn(locs, m)
    col = P.naive_greedy_coloring(NN)
    lm = np.arange(1, n + 1, dtype=np.int32)
    y = rng.normal(size=n)
    fields = [rng.normal(size=n) for _ in range(C)]
    args_c = ([0.1, 0.2], [0.0, 0.1], [-0.5, -0.3], [5, 6], [0, 0])
    old = os.environ.get("NNGP_TILES")
    os.environ["NNGP_TILES"] = str(16 * world)  # the same tiles on one GPU and over the ranks
    # shard calls always rebuild r = B w in their prologue: the one-GPU side
    # does too (a warm call starts from the carried-over r, last bits apart)
    old_warm = os.environ.get("NNGP_SWEEP_WARM")
    os.environ["NNGP_SWEEP_WARM"] = "0"
    try:
        res = []
        for shard in (False, True):
            # every step that may fail on one rank is agreed before the next
            # collective (a rank never waits for a peer that has given up)
            ctx = _agreed(dist, lambda: (
                ShardContext(locs, NN, col, lm, y, n_ranks=world, rank=rank, device=local_rank, n_chains=C)
                if shard else P.ChainContext(locs, NN, col, lm, y, device=local_rank, n_chains=C)))
            if shard:
                init_shard_comm(ctx, dist, rccl=False)
            for k in range(C):
                ctx.select(k)
                ctx.factor(0, "exponential_isotropic", [1.0, 0.1, 0.0])
                ctx.set_field(fields[k])
                ctx.set_mu(None, args_c[0][k])
            # two calls back to back (nothing read in between: the second
            # starts from the halo-only exchange of the first), then the read
            # (a full exchange first)
            ctx.sweep_chains(2, *args_c)
            ctx.sweep_chains(1, *args_c[:4], [2] * C)
            out = []
            for k in range(C):
                ctx.select(k)
                out.append(ctx.get_field())
            res.append((out, ctx.info))
            ctx.close()
    finally:
        if old is None:
            os.environ.pop("NNGP_TILES", None)
        else:
            os.environ["NNGP_TILES"] = old
        if old_warm is None:
            os.environ.pop("NNGP_SWEEP_WARM", None)
        else:
            os.environ["NNGP_SWEEP_WARM"] = old_warm
    ok = all(np.array_equal(a, b) for a, b in zip(res[0][0], res[1][0])) and res[1][1]["sweep_engine"] == 1
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item()), {"n": n, "m": m, "chains": C, "sweeps": 3, "tiles": 16 * world,
                            "exchange_slots_rank0": res[1][1]["shard_exchange_slots"]}


METRIC = "full-field Gibbs sweeps/sec at n=1e6, m=15; achieved HBM GB/s vs roofline"


def shard_failure_line(args, world, scaling, note, parity=None, pinfo=None):
    """The sharded measurement did not run (or its cross-GPU parity check
    failed): the line says so with a null value -- no other measurement is
    substituted (independent replicas only with --multi replicas)."""
    n = args.n * world if scaling == "weak" else args.n
    return {"metric": METRIC, "value": None, "unit": "sweeps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"sharded chromatic sweep of ONE field n={n} m={args.m} {args.covfun}",
                       "n": n, "m": args.m, "chains": args.chains,
                       "parity_check": {"bitwise_equal_to_one_gpu": parity, **(pinfo or {})},
                       "error": note},
            "roofline": None, "cpu_baseline": None}


def shard_main(P, args, world, rank, local_rank, dist, scaling):
    """The sharded sweep of ONE set of chains over the world GPUs (DESIGN.md
    §6; tile shard by default, colour shard with NNGP_ENGINE=colors).  Every
    rank builds the same workload (same seed).  scaling "weak": n = world x
    --n (every GPU keeps the tiles of an n=--n field: 256 tiles of ~3.9k
    locations at 1e6); "strong": n = --n split over the GPUs.  A step = one
    sweep of every chain; value = chain-sweeps/s x n / 1e6, i.e. sweeps of
    1e6-location fields per second (a sweep of the 8e6-location field counts 8)."""
    import torch

    from nngp_amd.shard import ShardContext, _agreed, _same_everywhere, init_shard_comm

    covfun, cp, C, nc = args.covfun, [1.0, args.range, 0.0], args.chains, args.n_chromatic
    n = args.n * world if scaling == "weak" else args.n
    t_par = time.time()
    parity, pinfo = shard_parity_check(P, args, world, rank, local_rank, dist) if world > 1 else (None, None)
    log(f"cross-GPU parity check ({time.time() - t_par:.1f}s): {parity}", rank)
    if world > 1 and not parity:
        return shard_failure_line(args, world, scaling, "the sharded sweep differs from one GPU on the cross-GPU "
                                  "parity check: not measured", parity, pinfo)
    log(f"shard setup n={n} m={args.m} {covfun} chains={C} world={world} scaling={scaling}", rank)
    agree = (lambda f: _agreed(dist, f)) if world > 1 else (lambda f: f())
    wl = agree(lambda: make_workload(P, n, args.m, covfun, cp, seed=1000, device=local_rank, chains=C))
    # the chains in groups whose tiles keep r in LDS (context.split_groups:
    # configs[4] at 3 chains -> a 2-chain and a 1-chain shard; one group
    # otherwise); every rank makes the same decision (same layout)
    groups = agree(lambda: P.context.split_groups(
        lambda k: ShardContext(wl["locs"], wl["NN"], wl["col"], wl["lm"], wl["y"], n_ranks=world, rank=rank,
                               device=local_rank, n_chains=k), list(range(C))))
    ctx = groups[0][0]
    try:
        if world > 1:  # the groups must match across ranks (their shards pair up rank by rank)
            _same_everywhere(dist, [list(ids) for _, ids in groups], "the chain groups")
        for g, _ in groups:
            init_shard_comm(g, dist, rccl=False)
        rng = np.random.default_rng(7)

        def prep():
            for g, ids in groups:
                for k in range(len(ids)):
                    g.select(k)
                    g.factor(0, covfun, cp)
                    g.set_field(wl["beta0"] + wl["w"] + 0.1 * rng.normal(size=len(wl["y"])))
                    g.set_mu(None, wl["beta0"])
                g.select(0)

        agree(prep)
        info = ctx.info
        b0, ls, lnv = wl["beta0"], wl["log_scale"], wl["log_noise_variance"]
        seeds = [77 + k for k in range(C)]

        def run(nsw, base):
            done = 0
            while done < nsw:
                s = min(nc, nsw - done)
                for g, ids in groups:
                    k = len(ids)
                    g.sweep_chains(s, [b0] * k, [ls] * k, [lnv] * k, [seeds[i] for i in ids], [base + done] * k)
                done += s
            return base + done

        sync = (lambda: torch.cuda.synchronize(local_rank)) if torch.cuda.is_available() else (lambda: None)
        log(f"graph prep {wl['t_graph']:.1f}s colours={info['n_colors']} engine={info['sweep_engine']} "
            f"tiles={info['n_tiles']} owned={info['shard_owned']} exchange_slots={info['shard_exchange_slots']}", rank)
        elapsed, _ = timed_region(run, args.steps, args.warmup, dist, sync)
    finally:
        for g, _ in groups:
            g.close()
    nnz = info["nnz"]
    tiles = info["sweep_engine"] == 1
    bytes_sweep = C * (8 * nnz + 40 * n) + 4 * nnz
    achieved = bytes_sweep * args.steps / elapsed / 1e9 / world  # per GPU, whole sharded call (wall clock)
    how = ("tile shard: the tiles of all GPUs in one persistent launch per GPU and call, cross-GPU hand-offs "
           "as 16-B granules stored into the reader GPU's buffer over xGMI (HIP IPC), each rank's halo slots of w "
           "stored into the peers' replicas after a call (device flags, no RCCL)" if tiles
           else "colour shard: one launch per colour, RCCL all-gather per colour")
    out = {"metric": METRIC,
           "metric_detail": (f"sweeps of 1e6-location fields per second = chain-sweeps/s x n/1e6 of the one "
                             f"n={n} field ({scaling} scaling" +
                             (f": n = {world} x {args.n}" if scaling == "weak" else "") + ")"),
           "value": args.steps * C * (n / 1e6) / elapsed, "unit": "sweeps/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
           "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (U[0,1]^2 locations, exact max-min order, field drawn from the Vecchia prior)",
           "config": {"workload": (f"sharded chromatic sweep of ONE field n={n} m={args.m} {covfun} "
                                   f"range={args.range}, {C} chains swept by all {world} GPUs "
                                   f"(value = chain-sweeps/s x n/1e6)"),
                      "n": n, "m": args.m, "n_colors": info["n_colors"], "nnz": nnz, "chains": C,
                      "chain_sweeps_per_s": args.steps * C / elapsed,
                      "chain_groups": [len(ids) for _, ids in groups],
                      "engine_note_rank0": info["engine_note"],
                      "n_chromatic_per_call": nc, "sweep_engine": "tile shard" if tiles else "colour shard",
                      "n_tiles": info["n_tiles"], "owned_rank0": info["shard_owned"],
                      "needed_rows_rank0": info["shard_needed_rows"],
                      "exchange_slots": info["shard_exchange_slots"],
                      "parity_check": {"bitwise_equal_to_one_gpu": parity, **(pinfo or {})},
                      "parallelism": f"{how}; {world} GPUs"},
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                        "kernel": "whole sharded call per GPU (wall clock)",
                        "algorithmic_bytes_per_sweep": bytes_sweep},
           "cpu_baseline": None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", "--n-locs", dest="n", type=int, default=1_000_000,
                    help="locations per GPU-share (--n-locs: the same, safe under torch.distributed.run)")
    ap.add_argument("--m", "--neighbours", dest="m", type=int, default=15)
    ap.add_argument("--covfun", default="matern15_isotropic")
    ap.add_argument("--range", type=float, default=0.05)
    ap.add_argument("--n-chromatic", type=int, default=10)
    ap.add_argument("--chains", type=int, default=3)
    ap.add_argument("--no-single-chain", action="store_true")
    ap.add_argument("--no-rebuild-calls", action="store_true", help="skip the rebuild-every-call measurement")
    ap.add_argument("--sustained-s", type=float, default=5.0,
                    help="seconds of back-to-back warm calls timed as one region (config.sustained; 0: skip)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--mcmc-iters", type=int, default=200,
                    help="timed MCMC iterations for the secondary metric, one update call (default: the "
                         "reference's n_iterations_update = 200, Scripts/mcmc_nngp_run.R:3; 0: skip)")
    ap.add_argument("--multi", choices=["shard-weak", "shard-strong", "replicas"], default="shard-weak",
                    help="N > 1: the sharded sweep of ONE field over the N GPUs with n = N x --n (shard-weak, "
                         "default) or n = --n (shard-strong), or independent chains per GPU (replicas)")
    ap.add_argument("--shard", action="store_true", help="the sharded sweep even at N = 1 (strong)")
    ap.add_argument("--no-fallback", action="store_true",
                    help="(default; kept for old command lines) a failed sharded sweep prints a null value")
    ap.add_argument("--workload", choices=["headline", "configs4"], default="headline",
                    help="configs4: BASELINE.json configs[4] exactly -- ONE field of n = 1e7, m = 20 (Matern 3/2) "
                         "swept by all N GPUs (the tile shard, strong scaling; at N = 1 the one-GPU engine): "
                         "python -m torch.distributed.run --nproc-per-node 8 bench.py --gpus 8 --workload configs4")
    args = ap.parse_args()
    if args.workload == "configs4":
        args.n, args.m = 10_000_000, 20
        args.multi = "shard-strong"
        args.shard = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("NNGP_BENCH_DEVICE"):  # test hook: every rank on this device
        local_rank = int(os.environ["NNGP_BENCH_DEVICE"])
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    import _pkgload

    P = _pkgload.load()
    covfun = args.covfun
    cp = [1.0, args.range, 0.0]
    note = None
    if args.shard or (world > 1 and args.multi != "replicas"):
        scaling = "weak" if (world > 1 and args.multi == "shard-weak") else "strong"
        try:
            out = shard_main(P, args, world, rank, local_rank, dist, scaling)
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line (null value)
            out = None
            note = f"sharded sweep failed on rank {rank}: {type(e).__name__}: {e}"
            log(note, 0)
        if world > 1:
            import torch as _t

            ok = _t.tensor([0 if out is None else 1], dtype=_t.int32)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if not ok.item():
                out = None
                note = note or "sharded sweep failed on another rank"
        if out is None:
            out = shard_failure_line(args, world, scaling, note)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    log(f"setup n={args.n} m={args.m} {covfun} chains={args.chains} world={world}", rank)
    wseed, seeds = replica_seeds(rank, args.chains)
    wl = make_workload(P, args.n, args.m, covfun, cp, seed=wseed, device=local_rank, chains=args.chains)
    C = args.chains
    nc = args.n_chromatic
    b0, ls, lnv = wl["beta0"], wl["log_scale"], wl["log_noise_variance"]

    def timed(ctx, steps, warmup, cold=False):
        """warmup + steps sweeps of every chain of ctx in calls of n_chromatic.
        cold: beta_0 alternates by 1e-9 between calls (the MCMC call shape
        when no covariance proposal was accepted: beta_0 is redrawn every
        iteration, update_Gaussian.R:219-224), so every call starts from
        w - d and r - d B 1 (capi.hip warm_kinds) -- or, on a context opened
        with NNGP_SWEEP_WARM=0, rebuilds w -> slots and r = B w."""
        k = ctx.n_chains
        calls = [0]

        def call(s, base):
            bb = b0 + (1e-9 if cold and calls[0] % 2 else 0.0)
            calls[0] += 1
            ctx.sweep_chains(s, [bb] * k, [ls] * k, [lnv] * k, seeds[:k], [base] * k)

        def run(nsw, base):
            done = 0
            while done < nsw:
                s = min(nc, nsw - done)
                call(s, base + done)
                done += s
            return base + done

        # capture every call shape of the timed region before it: the first
        # call of a shape (and of its warm form) captures and instantiates a
        # hipGraph (capi.hip graph_for), which must not land inside t0..t1.
        # The second call of a shape is warm (warm mode) or cold (cold mode,
        # beta_0 alternates) -- the form every timed call takes; eight calls
        # per shape so the device has run the timed shape for ~20 ms before
        # t0 whatever --warmup is (measured at the driver's --steps 20:
        # --warmup 5 with two priming calls 12.44-12.47k against 12.66-12.72k
        # at --warmup 20; with four 12.78k against 12.87-12.88k)
        for s in sorted({min(nc, steps)} | ({steps % nc} if steps % nc else set())):
            for _ in range(8):
                call(s, 1 << 40)
        sync = (lambda: torch.cuda.synchronize(local_rank)) if torch.cuda.is_available() else (lambda: None)
        return timed_region(run, steps, warmup, dist, sync)

    single = None
    if not args.no_single_chain:
        ctx1 = open_context(P, wl, covfun, cp, local_rank, 1, seed=5 + rank)
        el1, _ = timed(ctx1, args.steps, args.warmup)
        single = {"value": args.steps * world / el1, "unit": "sweeps/s",
                  "ms_per_step": el1 * 1e3 / args.steps,
                  "n_entries": ctx1.info["n_entries"]}
        ctx1.close()
    ctx = open_context(P, wl, covfun, cp, local_rank, C, seed=7 + rank)
    info = ctx.info
    wl["field0"] = ctx.get_field()
    log(f"graph prep {wl['t_graph']:.1f}s colours={info['n_colors']} nnz={info['nnz']} "
        f"entries={info['n_entries']} engine={info['sweep_engine']} tiles={info['n_tiles']} chunks={info['n_chunks']} "
        f"max_collen={info['max_collen']}", rank)
    elapsed, ctr = timed(ctx, args.steps, args.warmup)
    el_cold, ctr = timed(ctx, args.steps, args.warmup, cold=True)
    cold_calls = {"value": args.steps * C * world / el_cold, "unit": "sweeps/s",
                  "ms_per_step": el_cold * 1e3 / args.steps,
                  "how": ("beta_0 alternates by 1e-9 between calls (an MCMC iteration's beta_0 Gibbs step): "
                          "field and factor unchanged, so every call shifts w by -d and r by -d B 1 instead of "
                          "rebuilding them (NNGP_SWEEP_SHIFT=0: rebuild)")}
    # per-kernel timing with HIP events on the context's own stream: the
    # sweep kernel's launches alone (tile engine: one persistent launch per
    # call of n_chromatic sweeps; colour engine: one launch per colour)
    n, nnz = args.n, info["nnz"]
    engine = info["sweep_engine"]
    # SURVEY §8(d) algorithmic bytes: 12 nnz + 40 n per chain-sweep, the 4-byte
    # row index of an entry shared by the chains of a launch
    bytes_sweep = C * (8 * nnz + 40 * n) + 4 * nnz
    roofline = None
    if not args.no_kernel_timing:
        ksw = nc if engine == 1 else max(4, min(20, args.steps))
        reps = 5 if engine == 1 else 1
        kms_all = []
        try:
            for r in range(reps):
                _, kms = ctx.sweep_timed(ksw, [b0] * C, [ls] * C, [lnv] * C, seeds, [ctr + r * ksw] * C,
                                         per_kernel=True)
                kms_all.append(kms)
            kms = float(np.median(kms_all))
        except Exception as e:  # report, do not hide the throughput line
            log(f"per-kernel timing failed: {e}", rank)
            kms = float("nan")
        launches = 1 if engine == 1 else ksw * info["n_colors"]
        bytes_launch = bytes_sweep * ksw / launches
        achieved = bytes_launch / (kms * 1e-3 / launches) / 1e9
        kname = "sweep_tiles_kernel" if engine == 1 else "sweep_color_kernel"
        tr = pmc_traffic(C, n, args.m, kname)
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS,
                    "traffic": tr[0] / (kms * 1e-3 / launches) / 1e9 if tr else None,
                    "traffic_unit": "GB/s (PMC bytes per launch / measured launch time)",
                    "traffic_bytes_per_launch": tr[0] if tr else None,
                    "traffic_source": f"profiles/{tr[1]}" if tr else None,
                    "kernel": kname, "kernel_avg_us": kms * 1e3 / launches,
                    "algorithmic_bytes_per_sweep": bytes_sweep,
                    "algorithmic_bytes_per_launch": bytes_launch,
                    "sweeps_per_launch": ksw / launches,
                    "launches_per_sweep": launches / ksw}
    sustained = None
    if args.sustained_s > 0:
        # the same warm calls back to back for a few seconds as one timed
        # region: the rate with clocks and caches at steady state, and GPU
        # work long enough for a sampling monitor beside the bench to see
        ssteps = max(nc, int(math.ceil(args.sustained_s / (elapsed / args.steps) / nc)) * nc)
        el_s, ctr = timed(ctx, ssteps, 0)
        sustained = {"value": ssteps * C * world / el_s, "unit": "sweeps/s", "steps": ssteps,
                     "seconds": el_s, "ms_per_step": el_s * 1e3 / ssteps}
    mcmc = None
    if args.mcmc_iters > 0:
        sync = (lambda: torch.cuda.synchronize(local_rank)) if torch.cuda.is_available() else (lambda: None)
        try:
            mcmc = mcmc_iterations(P, wl, covfun, cp, ctx, args.mcmc_iters, 2, sync)
        except Exception as e:  # report, do not hide the throughput line
            log(f"mcmc iterations failed: {e}", rank)
    if not args.no_rebuild_calls and info["sweep_engine"] == 1:
        # the call after an accepted covariance proposal (new factor: r = B w
        # rebuilt): the same calls on a context that rebuilds every call --
        # after the kernel timing and the MCMC iterations (a second 3-chain
        # context on the device left the live kernel timing ~95 us slower
        # afterwards, not the throughput: profiles/r06_rebuild_timing_effect_*)
        os.environ["NNGP_SWEEP_WARM"] = "0"
        try:
            ctxr = open_context(P, wl, covfun, cp, local_rank, C, seed=7 + rank)
        finally:
            os.environ.pop("NNGP_SWEEP_WARM", None)
        el_rb, _ = timed(ctxr, args.steps, args.warmup, cold=True)
        ctxr.close()
        cold_calls["rebuild_calls"] = {"value": args.steps * C * world / el_rb, "unit": "sweeps/s",
                                       "ms_per_step": el_rb * 1e3 / args.steps,
                                       "how": "every call rebuilds w -> slots and r = B w (NNGP_SWEEP_WARM=0 "
                                              "context): the call after an accepted covariance proposal"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log(f"cpu baseline (oracle, {C} threads)...", rank)
        cpu = cpu_baseline(P, wl, covfun, cp, args.cpu_budget, C)
    ctx.close()
    value = args.steps * C * world / elapsed
    out = {"metric": METRIC,
           "value": value, "unit": "sweeps/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (U[0,1]^2 locations, exact max-min order, field drawn from the Vecchia prior)",
           "config": {"workload": (f"chromatic sweep n={n} m={args.m} {covfun} range={args.range}, "
                                   f"{C} chains per GPU swept together (value = chain-sweeps/s)"),
                      "n": n, "m": args.m, "n_colors": info["n_colors"], "nnz": nnz, "chains_per_gpu": C,
                      "n_entries": info["n_entries"], "n_chromatic_per_call": nc,
                      "sweep_engine": "tiles" if info["sweep_engine"] == 1 else "colours",
                      "n_tiles": info["n_tiles"], "tile_rows_max": info["tile_rows_max"],
                      "n_ghost_cells": info["n_ghost_cells"],
                      "call_prologue": ("warm: a call whose field, factor and beta_0 are unchanged since the "
                                        "last call starts from the slot-order w and r = B w that call left "
                                        "(NNGP_SWEEP_WARM=0: rebuild every call)"
                                        if os.environ.get("NNGP_SWEEP_WARM", "1") != "0" and info["sweep_engine"] == 1
                                        else "cold: w -> slots and r = B w rebuilt every call"),
                      "value_is": ("warm-call throughput: consecutive n_chromatic-sweep calls with nothing "
                                   "changed in between; an MCMC iteration redraws beta_0 (cold_calls: w and r "
                                   "shifted) and, after an accepted covariance proposal, rebuilds r = B w "
                                   "(cold_calls.rebuild_calls)"
                                   if os.environ.get("NNGP_SWEEP_WARM", "1") != "0" and info["sweep_engine"] == 1
                                   else "cold-call throughput"),
                      "single_chain": single,
                      "cold_calls": cold_calls,
                      "sustained": sustained,
                      "parallelism": f"chains {C} per GPU x {world} GPUs (independent)"},
           "roofline": roofline, "cpu_baseline": cpu, "secondary": mcmc}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
