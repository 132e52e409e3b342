"""Warm sweep calls and tile-launch residency (needs an MI355X).

A tile-engine call whose chains' field, current factor and beta_0 are
unchanged since the last call starts from the slot-order w and the r = B w the
last launch wrote back instead of rebuilding them ("warm", capi.hip
warm_call).  These tests pin that path to the cold path (which
tests/test_gpu_parity.py pins to the oracle): per call at the headline
workload, after every trigger that must invalidate it, and for the drift of
the carried-over r over 100 warm sweeps.  Cold contexts are created with
NNGP_SWEEP_WARM=0.

Tolerances: warm vs cold field max|a - b| <= 1e-10 max|b| per chain (the
warm call differs only in the rounding of the carried-over w and r); r drift
max|r - B (field - beta0)| <= 1e-11 max|B (field - beta0)|.  A call whose
field and factor are unchanged but whose beta_0 moved (the MCMC's beta_0
Gibbs step) stays warm: w -= d, r -= d B 1 (capi.hip warm_kinds); pinned the
same way, per call and for the drift over 100 shifted calls.

Last: two contexts swept concurrently from two host threads on one device,
whose tile grids together exceed the CUs -- the per-device tile lock
(capi.hip tile_lock) serialises the persistent launches, so both finish (no
spin timeout) with fields equal to the sequential run bitwise and to the
oracle's sweep (update_Gaussian.R:257-275).
"""
import threading

import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu

COV = "matern15_isotropic"


def _rel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


def _open(P, monkeypatch, prob, C, warm, cps, fields, b0s):
    locs, NN, col, lm, y = prob
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.delenv("NNGP_TILES", raising=False)
    if warm:
        monkeypatch.delenv("NNGP_SWEEP_WARM", raising=False)
    else:
        monkeypatch.setenv("NNGP_SWEEP_WARM", "0")
    ctx = P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C)
    monkeypatch.delenv("NNGP_SWEEP_WARM", raising=False)
    assert ctx.info["sweep_engine"] == 1, ctx.info
    for k in range(C):
        ctx.select(k)
        ctx.factor(0, COV, cps[k])
        ctx.set_field(fields[k])
        ctx.set_mu(None, b0s[k])
    return ctx


def _fields(ctx, C):
    out = []
    for k in range(C):
        ctx.select(k)
        out.append(ctx.get_field())
    return out


def test_warm_calls_equal_cold_calls_headline(P, monkeypatch):
    """The benched call shape: n = 1e6, m = 15, 3 chains, three back-to-back
    10-sweep calls with beta_0 unchanged (calls 2 and 3 warm) against the same
    calls on a context that rebuilds w and r every call."""
    n, m, C = 1_000_000, 15, 3
    prob = make_problem(P, n, m, seed=7)
    cps = [[1.0, 0.05, 0.0], [1.2, 0.04, 0.0], [0.8, 0.06, 0.0]]
    rng = np.random.default_rng(5)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0s, lss, lnvs, seeds = [0.0, 0.1, 0.2], [0.0, 0.2, -0.1], [-0.5, -0.4, -0.6], [11, 12, 13]
    res = {}
    for warm in (True, False):
        ctx = _open(P, monkeypatch, prob, C, warm, cps, fields, b0s)
        try:
            res[warm] = []
            for call in range(3):
                ctx.sweep_chains(10, b0s, lss, lnvs, seeds, [10 * call] * C)
                res[warm].append(_fields(ctx, C))
        finally:
            ctx.close()
    for call in range(3):
        for k in range(C):
            e = _rel(res[True][call][k], res[False][call][k])
            assert e <= 1e-10, (call, k, e)
    # the first call is cold on both: identical bits
    for k in range(C):
        assert np.array_equal(res[True][0][k], res[False][0][k])


@pytest.mark.parametrize("C", [1, 3])
def test_warm_call_r_drift_bounded(P, monkeypatch, C):
    """100 warm sweeps (one cold call, then ten warm 10-sweep calls): the r the
    kernel wrote back against a fresh r = B (field - beta_0)."""
    n, m = 1_000_000, 15
    prob = make_problem(P, n, m, seed=9)
    cps = [[1.0, 0.05, 0.0], [1.1, 0.045, 0.0], [0.9, 0.055, 0.0]][:C]
    rng = np.random.default_rng(6)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0s, lss, lnvs, seeds = [0.3, -0.1, 0.0][:C], [0.0, 0.1, -0.2][:C], [-0.5, -0.3, -0.7][:C], [21, 22, 23][:C]
    ctx = _open(P, monkeypatch, prob, C, True, cps, fields, b0s)
    try:
        for call in range(11):
            ctx.sweep_chains(10, b0s, lss, lnvs, seeds, [10 * call] * C)
        for k in range(C):
            ctx.select(k)
            r = ctx.get_sweep_r()
            fresh = ctx.spmv(0, ctx.get_field() - b0s[k])
            e = _rel(r, fresh)
            assert e <= 1e-11, (k, e)
    finally:
        ctx.close()


def test_beta0_shifted_warm_calls_equal_cold_calls_headline(P, monkeypatch):
    """The MCMC call shape without an accepted covariance proposal: beta_0
    redrawn between calls (the no-X beta_0 Gibbs step, update_Gaussian.R:
    219-224), field and factor unchanged -- the warm context shifts w by -d and
    r by -d B 1 (capi.hip warm_kinds / enqueue_warm_shift) instead of
    rebuilding them.  n = 1e6, m = 15, 3 chains, four 10-sweep calls with
    every chain's beta_0 moving by a different amount, and a fifth where
    chain 1's factor changed (cold) while chains 0 and 2 shift: every call
    against the cold context, <= 1e-10 max|field|."""
    n, m, C = 1_000_000, 15, 3
    prob = make_problem(P, n, m, seed=17)
    cps = [[1.0, 0.05, 0.0], [1.2, 0.04, 0.0], [0.8, 0.06, 0.0]]
    rng = np.random.default_rng(15)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0s, lss, lnvs, seeds = [0.0, 0.1, 0.2], [0.0, 0.2, -0.1], [-0.5, -0.4, -0.6], [11, 12, 13]
    shifts = [[0.0, 0.0, 0.0], [0.31, -0.07, 1e-9], [-0.5, 0.02, 0.0], [0.013, 0.4, -0.25], [0.1, 0.0, -0.1]]
    res = {}
    for warm in (True, False):
        ctx = _open(P, monkeypatch, prob, C, warm, cps, fields, b0s)
        b0 = list(b0s)
        try:
            res[warm] = []
            for call, d in enumerate(shifts):
                b0 = [a + x for a, x in zip(b0, d)]
                if call == 4:  # chain 1: a new current factor -> cold, the others shift
                    ctx.select(1).factor(0, COV, [1.1, 0.045, 0.0])
                ctx.sweep_chains(10, b0, lss, lnvs, seeds, [10 * call] * C)
                res[warm].append(_fields(ctx, C))
        finally:
            ctx.close()
    for call in range(len(shifts)):
        for k in range(C):
            e = _rel(res[True][call][k], res[False][call][k])
            assert e <= 1e-10, (call, k, e)


@pytest.mark.parametrize("C", [1, 3])
def test_beta0_shifted_calls_r_drift_bounded(P, monkeypatch, C):
    """100 one-sweep calls, beta_0 moving before every one (shifted warm
    calls: r -= d B 1 on top of the kernel's incremental r): the r the last
    call left against a fresh r = B (field - beta_0), as the warm-call drift
    bound."""
    n, m = 1_000_000, 15
    prob = make_problem(P, n, m, seed=19)
    cps = [[1.0, 0.05, 0.0], [1.1, 0.045, 0.0], [0.9, 0.055, 0.0]][:C]
    rng = np.random.default_rng(16)
    fields = [rng.normal(size=n) for _ in range(C)]
    b0s, lss, lnvs, seeds = [0.3, -0.1, 0.0][:C], [0.0, 0.1, -0.2][:C], [-0.5, -0.3, -0.7][:C], [21, 22, 23][:C]
    ctx = _open(P, monkeypatch, prob, C, True, cps, fields, b0s)
    b0 = list(b0s)
    try:
        for call in range(101):
            if call:
                b0 = [a + x for a, x in zip(b0, rng.normal(scale=0.05, size=C))]
            ctx.sweep_chains(1, b0, lss, lnvs, seeds, [call] * C)
        for k in range(C):
            ctx.select(k)
            r = ctx.get_sweep_r()
            fresh = ctx.spmv(0, ctx.get_field() - b0[k])
            e = _rel(r, fresh)
            assert e <= 1e-11, (k, e)
    finally:
        ctx.close()


TRIGGERS = ["set_field", "factor", "set_linv", "accept_factor", "beta0", "accept_field", "none"]


@pytest.mark.parametrize("trigger", TRIGGERS)
def test_warm_state_invalidated(P, monkeypatch, trigger):
    """Two calls (the second warm), then a change that invalidates the warm
    state of chain 0 (new field, new current factor through factor / set_linv
    / accept_factor, a new beta_0, an accepted ancillary proposal) or none, then
    a third call: every chain equals the same sequence on a cold context.  A
    warm call that missed the change would start from the old w / r (errors of
    order one)."""
    n, m, C = 60_000, 15, 2
    prob = make_problem(P, n, m, seed=13)
    cps = [[1.0, 0.05, 0.0], [0.9, 0.06, 0.0]]
    rng = np.random.default_rng(8)
    fields = [rng.normal(size=n) for _ in range(C)]
    new_field = rng.normal(size=n)
    b0s, lss, lnvs, seeds = [0.2, -0.1], [0.0, 0.1], [-0.5, -0.3], [31, 32]
    res = {}
    for warm in (True, False):
        ctx = _open(P, monkeypatch, prob, C, warm, cps, fields, b0s)
        b0 = list(b0s)
        try:
            ctx.sweep_chains(10, b0, lss, lnvs, seeds, [0] * C)
            ctx.sweep_chains(10, b0, lss, lnvs, seeds, [10] * C)
            ctx.select(0)
            if trigger == "set_field":
                ctx.set_field(new_field)
            elif trigger == "factor":
                ctx.factor(0, COV, [1.1, 0.045, 0.0])
            elif trigger == "set_linv":
                ctx.set_linv(0, ctx.get_linv(0) * 1.001)
            elif trigger == "accept_factor":
                ctx.factor(1, COV, [1.1, 0.045, 0.0])
                ctx.accept_factor()
            elif trigger == "beta0":
                b0[0] += 0.25
            elif trigger == "accept_field":
                ctx.factor(1, COV, [1.1, 0.045, 0.0])
                ctx.ancillary_propose(b0[0], 0.1)
                ctx.accept_field()
            ctx.sweep_chains(10, b0, lss, lnvs, seeds, [20] * C)
            res[warm] = _fields(ctx, C)
        finally:
            ctx.close()
    for k in range(C):
        e = _rel(res[True][k], res[False][k])
        assert e <= 1e-10, (trigger, k, e)


def test_two_contexts_swept_concurrently_one_device(P, O, monkeypatch):
    """Two 1-chain contexts on device 0 whose tile grids together exceed the
    CUs (each alone fits), swept from two host threads at once: both finish
    (no spin timeout), the first call of each equals the oracle's sweep with
    the device's factor, and every field equals the same calls run one
    context after the other, bitwise."""
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.delenv("NNGP_TILES", raising=False)
    n, m = 400_000, 10
    probs = [make_problem(P, n, m, seed=40 + q) for q in range(2)]
    cps = [[1.0, 0.08, 0.0], [1.3, 0.06, 0.0]]
    fields = [np.random.default_rng(50 + q).normal(size=n) for q in range(2)]
    b0s, lss, lnvs, seeds = [0.1, -0.2], [0.0, 0.2], [-0.6, -0.4], [61, 62]

    def make(q):
        locs, NN, col, lm, y = probs[q]
        ctx = P.ChainContext(locs, NN, col, lm, y, device=0)
        ctx.factor(0, "exponential_isotropic", cps[q])
        ctx.set_field(fields[q])
        ctx.set_mu(None, b0s[q])
        return ctx

    def run(ctx, q, out):
        try:
            got = []
            ctx.sweep_chains(2, [b0s[q]], [lss[q]], [lnvs[q]], [seeds[q]], [0])
            got.append(ctx.get_field())
            for call in range(3):
                ctx.sweep_chains(10, [b0s[q]], [lss[q]], [lnvs[q]], [seeds[q]], [2 + 10 * call])
            got.append(ctx.get_field())
            out[q] = got
        except Exception as e:  # noqa: BLE001 -- re-raised in the main thread
            out[q] = e

    ctxs = [make(0), make(1)]
    try:
        info = ctxs[0].info
        assert info["sweep_engine"] == 1 and ctxs[1].info["sweep_engine"] == 1
        assert info["n_tiles"] + ctxs[1].info["n_tiles"] > info["device_cus"], info
        Ls = [c.get_linv(0) for c in ctxs]
        conc = [None, None]
        th = [threading.Thread(target=run, args=(ctxs[q], q, conc)) for q in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in th), "a sweep thread did not finish"
        for q in range(2):
            if isinstance(conc[q], Exception):
                raise conc[q]
    finally:
        for c in ctxs:
            c.close()
    seq = [None, None]
    for q in range(2):
        c = make(q)
        try:
            run(c, q, seq)
        finally:
            c.close()
        if isinstance(seq[q], Exception):
            raise seq[q]
    for q in range(2):
        for a, b in zip(conc[q], seq[q]):
            assert np.array_equal(a, b), q
        locs, NN, col, lm, y = probs[q]
        z = O.sweep_normals(seeds[q], 0, 2, n)
        ref = O.sweep("local", fields[q], Ls[q], NN, col, O.precision_diag(Ls[q], NN), np.ones(n, np.int32), y,
                      np.full(n, b0s[q]), lm, b0s[q], lss[q], lnvs[q], z)
        np.testing.assert_allclose(conc[q][0], ref, rtol=1e-8, atol=1e-9)


def test_four_chains_split_into_tile_contexts(P, O, monkeypatch):
    """Four chains at the headline size: one 4-chain context's tiles exceed a
    CU's LDS (colour engine), so make_chain_views opens two 2-chain tile
    contexts instead (context.py _open_group); each chain's sweep equals the
    oracle's (update_Gaussian.R:257-275) and a 4-chain colour context."""
    ctxmod = P.context
    n, m = 1_000_000, 15
    locs, NN, col, lm, y = make_problem(P, n, m, seed=21)
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.delenv("NNGP_SPLIT_CHAINS", raising=False)
    views = ctxmod.make_chain_views(locs, NN, col, lm, y, 4, devices=[0])
    owners = [v.ctx for v in views]
    assert owners[0] is owners[1] and owners[2] is owners[3] and owners[0] is not owners[2]
    for o in (owners[0], owners[2]):
        assert o.n_chains == 2 and o.info["sweep_engine"] == 1, o.info
    rng = np.random.default_rng(5)
    cps = [[1.0, 0.05 * (1 + 0.1 * k), 0.0] for k in range(4)]
    fields = [rng.normal(size=n) for _ in range(4)]
    b0s, lss, lnvs = [0.3, -0.2, 0.1, 0.0], [0.1, -0.3, 0.0, 0.2], [-0.5, -0.2, -0.7, -0.4]
    keys = [101 + k for k in range(4)]
    for k, v in enumerate(views):
        v.factor(0, COV, cps[k])
        v.set_field(fields[k])
        v.set_mu(None, b0s[k])
    for o, ks in ((owners[0], [0, 1]), (owners[2], [2, 3])):
        o.sweep_chains(2, [b0s[k] for k in ks], [lss[k] for k in ks], [lnvs[k] for k in ks], [keys[k] for k in ks],
                       [0, 0])
    got = [v.get_field() for v in views]
    for o in {id(o): o for o in owners}.values():
        o.close()
    # the same chains in one 4-chain (colour-engine) context
    monkeypatch.setenv("NNGP_SPLIT_CHAINS", "0")
    one = ctxmod.make_chain_views(locs, NN, col, lm, y, 4, devices=[0])
    assert one[0].ctx is one[3].ctx and one[0].ctx.info["sweep_engine"] == 0
    for k, v in enumerate(one):
        v.factor(0, COV, cps[k])
        v.set_field(fields[k])
        v.set_mu(None, b0s[k])
    one[0].ctx.sweep_chains(2, b0s, lss, lnvs, keys, [0, 0, 0, 0])
    ref = [v.get_field() for v in one]
    one[0].ctx.close()
    for k in range(4):
        assert _rel(got[k], ref[k]) <= 1e-8, (k, _rel(got[k], ref[k]))
