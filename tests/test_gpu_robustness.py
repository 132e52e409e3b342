"""Forward progress and error reporting of the persistent launches (needs an
MI355X).

1. The sync-free triangular solve (update_Gaussian.R:127, the ancillary
   proposal B1^{-1} (B0 w); kernels.hip tri_dag_kernel) must not rest on
   residency or dispatch order: its ticket ("rescue") order is checked
   bitwise against the static order and the oracle, and a solve issued from
   a second host thread while another context's persistent tile sweep holds
   every CU finishes without a timeout and matches the oracle's tri_solve;
   with a grid twice the resident waves the rescue is proven to have run
   (nngp_tri_rescues).
2. A tile timeout is reported by the next host sync however many sweep calls
   were enqueued after it (the sticky timeout word, tiles.hip
   tile_call_bump_kernel): injected after the first of two async calls.

Tolerance: tri solve vs the oracle rtol 1e-9, atol 1e-10 (as
tests/test_gpu_parity.py); ticket order vs static order bitwise (same
products, same reduction order per row).
"""
import threading

import numpy as np
import pytest

from conftest import make_problem

pytestmark = pytest.mark.gpu

COV = "matern15_isotropic"


@pytest.mark.parametrize("n,m,C", [(5000, 5, 1), (120000, 15, 3)])
def test_tri_solve_ticket_order_equals_static_order(P, O, n, m, C, monkeypatch):
    """NNGP_TRI_RESCUE=1: every wave of the sync-free solve takes its groups
    from the ticket counter from the start (the order a rescue switches to):
    bitwise the static order's x, and the oracle's solve."""
    locs, NN, col, lm, y = make_problem(P, n, m, seed=n + 17)
    rng = np.random.default_rng(5)
    us = [rng.normal(size=n) for _ in range(2)]
    res = {}
    for rescue in ("0", "1"):
        monkeypatch.setenv("NNGP_TRI_RESCUE", rescue)
        with P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C) as ctx:
            for k in range(C):
                ctx.select(k).factor(0, COV, [1.0 + 0.1 * k, 0.05, 0.0])
            res[rescue] = [[ctx.select(k).tri_solve(0, u) for k in range(C)] for u in us]
            Ls = [ctx.select(k).get_linv(0) for k in range(C)]
    for a, b in zip(res["0"], res["1"]):
        for x0, x1 in zip(a, b):
            np.testing.assert_array_equal(x0, x1)
    for k in range(C):
        np.testing.assert_allclose(res["1"][0][k], O.tri_solve(Ls[k], NN, us[0]), rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("oversub", [1, 2])
def test_tri_solve_beside_a_persistent_tile_sweep(P, O, monkeypatch, oversub):
    """Thread A sweeps a 3-chain tile context (256 persistent workgroups, one
    per CU: while a launch runs no other wave fits the CUs it holds); thread B
    meanwhile runs sync-free solves on a second context.  Both finish without
    a timeout, every solve equals the oracle's, and the sweep's fields equal
    the same calls run alone, bitwise.  oversub = 2 (NNGP_TRI_OVERSUB): the
    solves' grids are twice what the device holds at once, so their static
    order waits on waves that are not resident (each wave's later groups
    depend on the first groups of waves past the resident set) and only the
    rescue's ticket order can finish them -- asserted through the context's
    rescue count, which proves the rescue path ran, not just that the solve
    happened to get its CUs."""
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.delenv("NNGP_TILES", raising=False)
    monkeypatch.delenv("NNGP_TRI_RESCUE", raising=False)
    monkeypatch.delenv("NNGP_TRI", raising=False)
    monkeypatch.setenv("NNGP_TRI_OVERSUB", str(oversub))
    n, m, C = 400_000, 10, 3
    locs, NN, col, lm, y = make_problem(P, n, m, seed=91)
    fields = [np.random.default_rng(92 + k).normal(size=n) for k in range(C)]
    b0, ls, lnv = [0.1] * C, [0.0] * C, [-0.5] * C
    seeds = [71 + k for k in range(C)]
    n_calls = 12

    def open_sweeper():
        ctx = P.ChainContext(locs, NN, col, lm, y, device=0, n_chains=C)
        for k in range(C):
            ctx.select(k).factor(0, "exponential_isotropic", [1.0, 0.08 + 0.01 * k, 0.0])
            ctx.set_field(fields[k])
            ctx.set_mu(None, b0[k])
        return ctx

    def sweeps(ctx, out):
        try:
            for call in range(n_calls):
                ctx.sweep_chains(10, b0, ls, lnv, seeds, [10 * call] * C)
            out["fields"] = [ctx.select(k).get_field() for k in range(C)]
        except Exception as e:  # noqa: BLE001 -- re-raised in the main thread
            out["err"] = e

    n2, m2 = 150_000, 15
    p2 = make_problem(P, n2, m2, seed=93)
    us = [np.random.default_rng(94 + q).normal(size=n2) for q in range(6)]

    def solves(ctx, out):
        try:
            out["x"] = [ctx.tri_solve(0, u) for u in us]
            out["rescues"] = ctx.tri_rescues()
        except Exception as e:  # noqa: BLE001
            out["err"] = e

    sw = open_sweeper()
    so = P.ChainContext(*p2, device=0, n_chains=1)
    try:
        assert sw.info["sweep_engine"] == 1, sw.info
        so.factor(0, COV, [1.0, 0.05, 0.0])
        L2 = so.get_linv(0)
        a, b = {}, {}
        ta = threading.Thread(target=sweeps, args=(sw, a))
        tb = threading.Thread(target=solves, args=(so, b))
        ta.start()
        tb.start()
        ta.join(timeout=300)
        tb.join(timeout=300)
        assert not ta.is_alive() and not tb.is_alive(), "a thread did not finish"
        for out in (a, b):
            if "err" in out:
                raise out["err"]
    finally:
        sw.close()
        so.close()
    for u, x in zip(us, b["x"]):
        np.testing.assert_allclose(x, O.tri_solve(L2, p2[1], u), rtol=1e-9, atol=1e-10)
    print(f"oversub {oversub}: {b['rescues']} of {len(us)} solves finished in the rescue's ticket order")
    if oversub > 1:
        assert b["rescues"] >= 1, "no solve ran the rescue: the static order finished on its own"
    alone = {}
    sw = open_sweeper()
    try:
        sweeps(sw, alone)
    finally:
        sw.close()
    if "err" in alone:
        raise alone["err"]
    for f0, f1 in zip(a["fields"], alone["fields"]):
        np.testing.assert_array_equal(f0, f1)


def test_tile_timeout_survives_a_later_async_call(P, monkeypatch):
    """A timeout raised by the first of two sweep calls enqueued without a
    host sync (NNGP_TILE_INJECT_TIMEOUT=1: the control words a timed-out
    launch leaves, after call 1) is still reported at the next sync (the
    second call's launch resets only its own timeout word), once: the call
    after the report runs clean."""
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.delenv("NNGP_TILES", raising=False)
    monkeypatch.setenv("NNGP_TILE_INJECT_TIMEOUT", "1")
    n, m = 60_000, 10
    locs, NN, col, lm, y = make_problem(P, n, m, seed=95)
    with P.ChainContext(locs, NN, col, lm, y, device=0) as ctx:
        assert ctx.info["sweep_engine"] == 1, ctx.info
        ctx.factor(0, "exponential_isotropic", [1.0, 0.08, 0.0])
        ctx.set_field(np.zeros(n))
        ctx.set_mu(None, 0.0)
        ctx.sweep_chains(2, [0.0], [0.0], [-0.5], [3], [0])  # async: returns after the launch
        ctx.sweep_chains(2, [0.0], [0.0], [-0.5], [3], [2])
        with pytest.raises(P.NNGPError, match="timed out"):
            ctx.get_field()
        ctx.sweep_chains(2, [0.0], [0.0], [-0.5], [3], [4])
        f = ctx.get_field()
        assert np.isfinite(f).all()
