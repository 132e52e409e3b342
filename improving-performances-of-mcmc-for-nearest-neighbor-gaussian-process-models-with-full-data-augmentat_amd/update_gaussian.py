"""mcmc_nngp_update_Gaussian -- host mirror of
Scripts/mcmc_nngp_update_Gaussian.R:14-317 (and ll_compressed_sparse_chol,
:8-12).

The scalar Metropolis-Hastings / adaptation logic stays on the
host exactly as in the reference; every O(n) / O(nnz) array operation is a
call into the device context of the chain:

=====================================  =====================================
reference (update_Gaussian.R)          device call (include/nngp.h)
=====================================  =====================================
vecchia_Linv + sparseMatrix :72-73     ctx.factor(0, ...)
precision_diag :74,142,197             (inside nngp_factor / nngp_accept_factor)
vecchia_Linv :123 / :179               ctx.factor(1, ...)
solve(new_B, B %*% (field-b0)) :127    ctx.ancillary_propose
sum(dnorm(.)) - sum(dnorm(.)) :129-131 ctx.field_response_ratio
ll_compressed_sparse_chol :184-186     ctx.loglik(1, .) - ctx.loglik(0, .)
crossprod(B 1), (B f, B 1) :221-222    ctx.beta0_stats
residuals_sum + chromatic loop :257-275 ctx.sweep(n_chromatic, ...)
sum_squared_residuals :281             ctx.sum_squared_residuals
sparse_chol %*% X :79,82,147,241       ctx.spmv
=====================================  =====================================

Chains live in device contexts (up to 4 chains per context, contexts possibly
on distinct devices) instead of forked ``mclapply`` workers: HIP must never
be initialised before a fork.  Each chain's iteration is a generator that
yields at its chromatic sweep; the driver advances all chains in lockstep and
sweeps the chains of one context in the same kernels (``sweep_chains``).
Chains are independent (own RNG streams, own device state), so the lockstep
order gives exactly the results of running the chains one after another.
Seeds: numpy PCG64 seeded with ``iter_start + i`` (the reference's
``set.seed(iter_start + i)``, :34-36); the chromatic sweep's normals come from
the device Philox stream keyed by the same value, so a resumed run is
reproducible.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading

import numpy as np

from ._lib import NNGP_ERR_CHOL, NNGPError
from .context import ChainContext, make_chain_views
from .model import covparms


def ll_compressed_sparse_chol(ctx: ChainContext, which: int, beta0: float, log_scale: float) -> float:
    """Vecchia log-likelihood of field - beta_0 (update_Gaussian.R:8-12)."""
    return ctx.loglik(which, beta0, log_scale)


def _philox_key(iter_start: int, chain: int, seed: int) -> int:
    return ((int(seed) & 0xFFFFFFFF) << 32) ^ ((int(iter_start) + int(chain)) & 0xFFFFFFFF) ^ 0x9E3779B97F4A7C15


def _interweave_prep(ctx, X, va):
    """beta_interweaved_* (update_Gaussian.R:77-83,145-151)."""
    Xl = X["X"][va["hctam_scol_1"] - 1][:, X["locs"]]
    M = np.column_stack([np.ones(va["n_locs"]), Xl])
    SX = ctx.spmv(0, M)
    prec = SX.T @ SX
    cov = np.linalg.inv(prec)
    return {"Xl": Xl, "SX": SX, "covmat": cov, "covmat_chol": np.linalg.cholesky(cov).T}


def _prefault(arr: np.ndarray) -> threading.Thread:
    """Touch the pages of a fresh host array on a helper thread (memset
    through ctypes, which releases the GIL) while the chain runs: the record
    copy at the end of the call then lands in resident pages (measured for a
    40 x 1e6 record block: 18.9 ms into fresh pages, 6.5 ms into touched ones)."""
    def run():
        step = 1 << 26
        base, nb = arr.ctypes.data, arr.nbytes
        for off in range(0, nb, step):
            ctypes.memset(base + off, 0, min(step, nb - off))

    th = threading.Thread(target=run, daemon=True)
    th.start()
    return th


def _proposal_ok(status, on_chol_error):
    """Outcome of a proposal's vecchia_Linv (update_Gaussian.R:123,179).  In
    the reference a local covariance that is not positive definite makes GpGp
    raise an R error, which ends the update call (on_chol_error="error", the
    default); on_chol_error="reject" treats the proposal as rejected instead.
    Any other failure (HIP, memory, a timeout) propagates from the call."""
    if status == 0:
        return True
    if status == NNGP_ERR_CHOL and on_chol_error != "reject":
        raise NNGPError(NNGP_ERR_CHOL, "vecchia factor: a local covariance of the proposal is not positive definite")
    return False


def _chain_program(i, state, ctx, X, observed_field, space_time_model, va, n_iterations_update,
                   field_thinning, ancillary, n_chromatic, iter_start, seed, on_chol_error="error", var_y=None):
    """Chain i's n_iterations_update Gibbs iterations; yields its device
    requests and receives their results, so that the chains of one context
    are served by one batched call per step (one host sync for all of them):
      ("astep", covfun, covparms, beta_0, dlog_scale, lnv)
          -> (status of the proposal factor, dnorm ratio of the ancillary proposal)
      ("sstep", covfun, covparms | None, beta_0, new_ls, ls)
          -> (status, (loglik(1), loglik(0))) | None when covparms is None
      ("sweep", n_sweeps, beta_0, log_scale, lnv, key, counter) -> None
      ("ssr", beta_0)                          -> sum of squared residuals
    Every chain yields every step of an iteration (None = nothing to do), so
    the chains stay in lockstep.  Returns {"state", "records", "acceptance"}."""
    # (runif(1) is rng.random(): the same draw as rng.uniform() bit for bit,
    # without its argument handling -- 0.36 vs 1.5 us a call)
    rng = np.random.default_rng(int(iter_start) + i + 1)
    key = _philox_key(iter_start, i + 1, seed)
    covfun = space_time_model["covfun"]["stationary_covfun"]
    sp_names = space_time_model["covfun"]["shape_params"]
    params = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in state["params"].items()}
    tk = {k: dict(v) for k, v in state["transition_kernels"].items()}
    n_obs = va["n_obs"]
    if var_y is None:
        var_y = float(np.var(observed_field, ddof=1))
    has_X = X.get("X") is not None
    has_locs = has_X and len(X["locs"]) > 0
    n_shape = len(sp_names)

    rec = {"beta_0": np.zeros((n_iterations_update, 1)),
           "log_scale": np.zeros((n_iterations_update, 1)),
           "log_noise_variance": np.zeros((n_iterations_update, 1)),
           "shape": np.zeros((n_iterations_update, n_shape)),
           "field": np.empty((int(round(n_iterations_update * field_thinning)), va["n_locs"]))}
    if has_X:
        rec["beta"] = np.zeros((n_iterations_update, X["X"].shape[1]))
    acc_suf = np.zeros(n_iterations_update)
    acc_anc = np.zeros(n_iterations_update)
    # recorded fields (records$field, :56,311) are kept on the device and
    # streamed into rec["field"] by the library while the chain runs
    # (records_stream; NNGP_RECORDS_STREAM=0: copied at the end of the call,
    # the host pages touched meanwhile); host copies per iteration if HBM is
    # short
    n_rec = rec["field"].shape[0]
    dev_rec = n_rec > 0
    if dev_rec:
        try:
            ctx.records_reserve(n_rec)
        except NNGPError:
            dev_rec = False
    if not dev_rec:
        rec["field"][:] = 0.0
    streamed = False
    if dev_rec and os.environ.get("NNGP_RECORDS_STREAM", "1") != "0":
        try:
            ctx.records_stream(rec["field"])
            streamed = True
        except (AttributeError, NNGPError):
            pass
    touch = _prefault(rec["field"]) if dev_rec and not streamed else None

    # Vecchia factor of the current state (:67-74)
    ctx.factor(0, covfun, covparms(sp_names, params["shape"]))
    ctx.set_field(params["field"])
    iw = _interweave_prep(ctx, X, va) if has_locs else None

    def mu_of():
        if has_X:
            return params["beta_0"] + X["X"] @ params["beta"]
        return None

    ctx.set_mu(mu_of(), params["beta_0"])
    adapt = 0 <= iter_start <= 2000

    for it in range(1, n_iterations_update + 1):
        # ---- ancillary covariance update (:113-157)
        if ancillary:
            innov = rng.normal(0.0, math.exp(0.5 * tk["covariance_params_ancillary"]["logvar"]), n_shape + 1)
            new_ls = params["log_scale"] + innov[0]
            new_shape = params["shape"] + innov[1:]
            # the proposal's factor (:123), its field (:127) and the dnorm ratio
            # (:129-131) behind one host sync
            st, ratio = yield ("astep", covfun, covparms(sp_names, new_shape), params["beta_0"],
                               new_ls - params["log_scale"], params["log_noise_variance"])
            ok = _proposal_ok(st, on_chol_error)
            if ok:
                if ratio > math.log(rng.random()):
                    params["shape"] = new_shape
                    params["log_scale"] = new_ls
                    ctx.accept_field()
                    ctx.accept_factor()
                    acc_anc[it - 1] = 1
                    if has_locs:
                        iw = _interweave_prep(ctx, X, va)
            if adapt and it % 25 == 0:
                a = acc_anc[it - 25:it].mean()
                if a < 0.05:
                    tk["covariance_params_ancillary"]["logvar"] -= rng.normal(0.4, 0.05)
                if a > 0.15:
                    tk["covariance_params_ancillary"]["logvar"] += rng.normal(0.4, 0.05)

        # ---- sufficient covariance update (:165-213)
        innov = rng.normal(0.0, math.exp(0.5 * tk["covariance_params_sufficient"]["logvar"]), n_shape + 1)
        new_ls = params["log_scale"] + innov[0]
        propose = math.exp(new_ls) < var_y
        new_shape = params["shape"] + innov[1:] if propose else None
        # the proposal's factor (:179) and both log-likelihoods (:184-186)
        # behind one host sync; a chain that does not propose still yields, so
        # the chains of one context stay in lockstep
        res = yield ("sstep", covfun, covparms(sp_names, new_shape) if propose else None, params["beta_0"], new_ls,
                     params["log_scale"])
        ok = propose and _proposal_ok(res[0], on_chol_error)
        lls = res[1] if ok else None
        if ok:
            gp_ratio = lls[0] - lls[1]
            if gp_ratio > math.log(rng.random()):
                params["shape"] = new_shape
                params["log_scale"] = new_ls
                ctx.accept_factor()
                acc_suf[it - 1] = 1
                if has_locs:
                    iw = _interweave_prep(ctx, X, va)
        if adapt and it % 25 == 0:
            a = acc_suf[it - 25:it].mean()
            if a < 0.05:
                tk["covariance_params_sufficient"]["logvar"] -= rng.normal(0.2, 0.05)
            if a > 0.15:
                tk["covariance_params_sufficient"]["logvar"] += rng.normal(0.2, 0.05)

        # ---- field mean (:219-247)
        if (not has_locs) or (not has_X):
            oqo, oqf = ctx.beta0_stats()
            beta_covmat = math.exp(params["log_scale"]) / oqo
            beta_mean = math.exp(-params["log_scale"]) * oqf * beta_covmat
            params["beta_0"] = float(beta_mean + math.sqrt(beta_covmat) * rng.normal())
        if has_X:
            field = ctx.get_field()
            X1 = np.column_stack([np.ones(n_obs), X["X"]])
            resid = observed_field - field[va["locs_match"] - 1] + params["beta_0"]
            beta_mean = (resid @ X1) @ X["solve_1XT1X"]
            innov = beta_mean + math.exp(0.5 * params["log_noise_variance"]) * (
                X["chol_solve_1XT1X"].T @ rng.normal(size=X1.shape[1]))
            field = field - params["beta_0"] + innov[0]
            params["beta_0"] = float(innov[0])
            params["beta"] = innov[1:].copy()
            if has_locs:
                locs_cols = X["locs"]
                other = field + iw["Xl"] @ params["beta"][locs_cols]
                Bo = ctx.spmv(0, other)
                bm = iw["covmat"] @ (Bo @ iw["SX"])
                innov = bm + math.exp(0.5 * params["log_scale"]) * (iw["covmat_chol"].T @ rng.normal(size=len(locs_cols) + 1))
                params["beta_0"] = float(innov[0])
                params["beta"][locs_cols] = innov[1:]
                field = other - iw["Xl"] @ params["beta"][locs_cols]
            ctx.set_field(field)
        ctx.set_mu(mu_of(), params["beta_0"])

        # ---- chromatic sampling of the field (:257-275)
        yield ("sweep", n_chromatic, params["beta_0"], params["log_scale"], params["log_noise_variance"],
               key, (int(iter_start) + it - 1) * n_chromatic)

        # ---- noise variance (:281-293)
        ssr = yield ("ssr", params["beta_0"])
        for _ in range(10):
            innov = rng.normal(0.0, 0.01)
            if math.exp(params["log_noise_variance"] + innov) < var_y:
                lnv = params["log_noise_variance"]
                if -0.5 * n_obs * innov - 0.5 * ssr * (math.exp(-lnv - innov) - math.exp(-lnv)) > math.log(rng.random()):
                    params["log_noise_variance"] = lnv + innov

        # ---- records (:305-311)
        if has_X:
            rec["beta"][it - 1] = params["beta"]
        rec["beta_0"][it - 1] = params["beta_0"]
        rec["log_noise_variance"][it - 1] = params["log_noise_variance"]
        rec["log_scale"][it - 1] = params["log_scale"]
        rec["shape"][it - 1] = params["shape"]
        # (R's records$field[0, ] <- ... is a no-op: field_thinning = 0 records nothing)
        if round(it * field_thinning) == it * field_thinning and it * field_thinning >= 1:
            if dev_rec:
                ctx.record_field(int(it * field_thinning) - 1)
            else:
                rec["field"][int(it * field_thinning) - 1] = ctx.get_field()

    if dev_rec:
        if touch is not None:
            touch.join()
        ctx.get_records(0, n_rec, out=rec["field"])
        ctx.records_reserve(0)
    params["field"] = ctx.get_field()
    return {"state": {"params": params, "transition_kernels": tk}, "records": rec,
            "acceptance": {"covariance_acceptance_sufficient": acc_suf,
                           "covariance_acceptance_ancillary": acc_anc}}


def _owner_of(ctx):
    """(ChainContext, chain) serving a chain's batched calls, or (None, None)."""
    owner = getattr(ctx, "ctx", None)
    if owner is not None:
        return owner, ctx.chain
    if getattr(ctx, "n_chains", None) == 1 and hasattr(ctx, "ancillary_step_chains"):
        return ctx, 0
    return None, None


def _serve_step_separately(ctx, req):
    """A step request through the separate calls (contexts without the
    one-sync step entry points)."""
    try:
        ctx.factor(1, req[1], req[2])
        st = 0
    except NNGPError as e:
        if e.status != NNGP_ERR_CHOL:
            raise
        return NNGP_ERR_CHOL, float("nan") if req[0] == "astep" else None
    if req[0] == "astep":
        ctx.ancillary_propose(req[3], req[4])
        return st, ctx.field_response_ratio(req[3], req[5])
    return st, (ctx.loglik(1, req[3], req[4]), ctx.loglik(0, req[3], req[5]))


def _serve_one(ctx, req):
    """One chain's request on its own -> its result."""
    kind = req[0]
    if kind in ("astep", "sstep"):
        if req[2] is None:
            return None
        owner, k = _owner_of(ctx)
        if owner is None:
            return _serve_step_separately(ctx, req)
        cps = np.tile(np.asarray(req[2], np.float64), (owner.n_chains, 1))
        if kind == "astep":
            st, r = owner.ancillary_step_chains(1 << k, req[1], cps, req[3], req[4], req[5])
            return int(st[k]), float(r[k])
        st, lp, lc = owner.sufficient_step_chains(1 << k, req[1], cps, req[3], req[4], req[5])
        return int(st[k]), (float(lp[k]), float(lc[k]))
    if kind == "ssr":
        return ctx.sum_squared_residuals(req[1])
    ctx.sweep(*req[1:])
    return None


def _run_chain(i, state, ctx, X, observed_field, space_time_model, va, n_iterations_update,
               field_thinning, ancillary, n_chromatic, iter_start, seed, on_chol_error="error"):
    """One chain alone (each request served on its own)."""
    prog = _chain_program(i, state, ctx, X, observed_field, space_time_model, va, n_iterations_update,
                          field_thinning, ancillary, n_chromatic, iter_start, seed, on_chol_error)
    try:
        req = next(prog)
        while True:
            req = prog.send(_serve_one(ctx, req))
    except StopIteration as stop:
        return stop.value


def _serve_group(owner, ids, reqs, contexts, out):
    """Serve the same-kind requests of the chains `ids` of one ChainContext
    with one batched call (results into out[i]); False if they cannot be
    batched."""
    if owner is None or owner.n_chains < 2:
        return False
    kinds = {reqs[i][0] for i in ids}
    if len(kinds) != 1:
        return False
    kind = kinds.pop()
    k = owner.n_chains
    live = [i for i in ids if reqs[i][2] is not None] if kind in ("astep", "sstep") else list(ids)
    mask = 0
    for i in live:
        mask |= 1 << contexts[i].chain
    for i in ids:
        out[i] = None
    if kind in ("astep", "sstep"):
        if not live:
            return True
        covfuns = {reqs[i][1] for i in live}
        if len(covfuns) != 1:
            return False
        cps = np.zeros((k, len(reqs[live[0]][2])))
        cols = [np.zeros(k) for _ in range(3)]
        for i in live:
            c = contexts[i].chain
            cps[c] = reqs[i][2]
            for q in range(3):
                cols[q][c] = reqs[i][3 + q]
        if kind == "astep":
            st, r = owner.ancillary_step_chains(mask, covfuns.pop(), cps, *cols)
            for i in live:
                out[i] = (int(st[contexts[i].chain]), float(r[contexts[i].chain]))
        else:
            st, lp, lc = owner.sufficient_step_chains(mask, covfuns.pop(), cps, *cols)
            for i in live:
                c = contexts[i].chain
                out[i] = (int(st[c]), (float(lp[c]), float(lc[c])))
        return True
    if kind == "ssr":
        b0 = np.zeros(k)
        for i in ids:
            b0[contexts[i].chain] = reqs[i][1]
        r = owner.sum_squared_residuals_chains(mask, b0)
        out.update({i: float(r[contexts[i].chain]) for i in ids})
        return True
    if len(ids) != k or len({reqs[i][1] for i in ids}) != 1:
        return False
    order = sorted(ids, key=lambda i: contexts[i].chain)
    cols = list(zip(*[reqs[i][1:] for i in order]))
    owner.sweep_chains(cols[0][0], cols[1], cols[2], cols[3], cols[4], cols[5])
    return True


def _drive(programs, contexts):
    """Advance chain programs in lockstep; the requests of the chains of one
    ChainContext go through one batched call (sweep_chains, the one-sync MH
    steps, sum_squared_residuals_chains)."""
    results = [None] * len(programs)
    reqs = {}
    for i, g in enumerate(programs):
        try:
            reqs[i] = next(g)
        except StopIteration as stop:
            results[i] = stop.value
    while reqs:
        groups = {}
        for i in reqs:
            owner = getattr(contexts[i], "ctx", None)
            groups.setdefault(id(owner) if owner is not None else ("solo", i), []).append(i)
        served = {}
        for ids in groups.values():
            owner = getattr(contexts[ids[0]], "ctx", None)
            if not _serve_group(owner, ids, reqs, contexts, served):
                for i in ids:
                    served[i] = _serve_one(contexts[i], reqs[i])
        nxt = {}
        for i in reqs:
            try:
                nxt[i] = programs[i].send(served.get(i))
            except StopIteration as stop:
                results[i] = stop.value
        reqs = nxt
    return results


def mcmc_nngp_update_Gaussian(locs, X, observed_field, space_time_model, vecchia_approx, states,
                              n_iterations_update, n_cores=None, field_thinning=1.0, ancillary=True,
                              n_chromatic=10, iterations=None, contexts=None, seed=1, devices=None,
                              on_chol_error="error"):
    """Returns one {"state", "records"} per chain (update_Gaussian.R:315).
    on_chol_error: "error" (GpGp's behaviour: a non positive definite local
    covariance of a proposal raises) or "reject" (the proposal is rejected)."""
    if on_chol_error not in ("error", "reject"):
        raise ValueError("on_chol_error must be 'error' or 'reject'")
    iter_start = int(iterations[-1, 0]) if iterations is not None else 0
    names = list(states.keys()) if isinstance(states, dict) else [f"chain_{i + 1}" for i in range(len(states))]
    st_list = list(states.values()) if isinstance(states, dict) else list(states)
    if contexts is None:
        contexts = make_chain_views(locs, vecchia_approx["NNarray"], vecchia_approx["coloring"],
                                    vecchia_approx["locs_match"], observed_field, len(st_list), devices)
    y = np.asarray(observed_field, np.float64)
    var_y = float(np.var(y, ddof=1))  # var(observed_field), :167,286 (once for all chains)
    programs = [_chain_program(i, st, contexts[i], X, y, space_time_model, vecchia_approx,
                               int(n_iterations_update), float(field_thinning), bool(ancillary),
                               int(n_chromatic), iter_start, seed, on_chol_error, var_y)
                for i, st in enumerate(st_list)]
    return dict(zip(names, _drive(programs, contexts)))
