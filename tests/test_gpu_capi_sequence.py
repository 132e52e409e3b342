"""A C client of include/nngp.h (tests/cpp/capi_sequence.c: the call sequence
of the R drop-in, rpkg/R/mcmc_nngp_update_Gaussian.R) gives exactly what the
same sequence gives through the Python binding: the boundary carries no
hidden state of the binding."""
import math
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
EXE = ROOT / "tests" / "cpp" / "capi_sequence"
pytestmark = pytest.mark.gpu


def _jit(i, k):
    h = (np.uint64(i) * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)
    h ^= (np.uint64(k + 1) * np.uint64(40503)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0x5BD1E995)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    return (h & np.uint64(0xFFFFFF)).astype(np.float64) / float(0x1000000) - 0.5


def test_c_client_equals_python_binding(P):
    n, m = 3000, 10
    assert EXE.exists(), "build() compiles tests/cpp/capi_sequence"
    out = subprocess.run([str(EXE), str(n), str(m)], capture_output=True, text=True, timeout=120, check=True).stdout
    lines = out.strip().splitlines()
    K = int(lines[0].split()[1])
    ll_c = float.fromhex(lines[1].split()[1])
    fields_c = [np.array([float.fromhex(v) for v in ln.split()[2:]]) for ln in lines[2:4]]

    i = np.arange(n)
    side = int(np.ceil(np.sqrt(n)))
    raw = np.column_stack([(i % side + 0.3 * _jit(i, 0)) / side, (i // side + 0.3 * _jit(i, 1)) / side])
    locs = raw[P.order_maxmin(raw) - 1]
    NN = P.find_ordered_nn(locs, m)
    col = P.naive_greedy_coloring(NN)
    assert col.max() == K
    y = np.sin(6 * locs[:, 0]) + np.cos(4 * locs[:, 1]) + 0.3 * _jit(i, 2)
    f = y + 0.1 * _jit(i, 3)
    cps = [[1.0, 0.1, 0.0], [0.8, 0.15, 0.0]]
    b0, ls, lnv = [0.1, -0.2], [0.0, 0.3], [-1.0, -0.7]
    with P.ChainContext(locs, NN, col, np.arange(1, n + 1, dtype=np.int32), y, device=0, n_chains=2) as ctx:
        for k in range(2):
            ctx.select(k)
            ctx.factor(0, "exponential_isotropic", cps[k])
            ctx.set_field(f)
            ctx.set_mu(None, b0[k])
        ctx.select(1)
        ll = ctx.loglik(0, b0[1], ls[1])
        ctx.sweep_chains(3, b0, ls, lnv, [101, 202], [0, 50])
        fields = []
        for k in range(2):
            ctx.select(k)
            fields.append(ctx.get_field())
    assert ll == ll_c
    for k in range(2):
        np.testing.assert_array_equal(fields[k], fields_c[k], err_msg=f"chain {k}")


def test_c_client_r_dropin_lockstep_equals_python_binding(P):
    """The R drop-in's 3-chain lockstep iteration (rpkg/R/mcmc_nngp_update_Gaussian.R:
    ancillary_step_chains -> accept_field / accept_factor ->
    sufficient_step_chains -> (here, in Python: the separate calls they
    replace, factor_chains -> ancillary_propose_chains ->
    field_response_ratio_chains and factor_chains -> loglik_chains x 2) ->
    accept_factor -> beta0_stats / set_mu per chain -> sweep_chains ->
    sum_squared_residuals_chains -> record_field; get_records / get_field at the
    end), 2 iterations with fixed draws and fixed log-uniforms (chain 0 always
    accepts, chain 1 never, chain 2 by the device value), from C and through the
    Python binding: every device result the host sees, every record and every
    field bitwise equal (host math through libm on both sides: math.exp/sin)."""
    n, m = 3000, 10
    assert EXE.exists(), "build() compiles tests/cpp/capi_sequence"
    out = subprocess.run([str(EXE), str(n), str(m), "lockstep"], capture_output=True, text=True, timeout=120,
                         check=True).stdout
    got = {}
    for ln in out.strip().splitlines()[1:]:
        w = ln.split()
        got[tuple(w[:3]) if w[0] in ("beta0_stats", "record") else tuple(w[:2])] = [float.fromhex(v) for v in w[
            (3 if w[0] in ("beta0_stats", "record") else 2):]]

    i = np.arange(n)
    side = int(np.ceil(np.sqrt(n)))
    raw = np.column_stack([(i % side + 0.3 * _jit(i, 0)) / side, (i // side + 0.3 * _jit(i, 1)) / side])
    locs = raw[P.order_maxmin(raw) - 1]
    NN = P.find_ordered_nn(locs, m)
    col = P.naive_greedy_coloring(NN)
    y = np.sin(6 * locs[:, 0]) + np.cos(4 * locs[:, 1]) + 0.3 * _jit(i, 2)
    C, NC, NIT = 3, 2, 2
    ls, shape, b0 = [0.0, 0.2, -0.1], [-2.3, -2.0, -2.6], [0.1, -0.2, 0.0]
    lnv = [-1.0, -0.7, -1.2]
    lu_anc, lu_suf = [-1e300, 1e300, -0.7], [1e300, -1e300, -0.3]
    want = {}
    with P.ChainContext(locs, NN, col, np.arange(1, n + 1, dtype=np.int32), y, device=0, n_chains=C) as ctx:
        for k in range(C):
            ctx.select(k)
            ctx.records_reserve(NIT)
            ctx.factor(0, "exponential_isotropic", [1.0, math.exp(shape[k]), 0.0])
            ctx.set_field(np.array([0.05 * k + math.sin(3.0 * q / n + k) for q in range(n)]))
            ctx.set_mu(None, b0[k])
        for it in range(1, NIT + 1):
            nls = [ls[k] + 0.05 * (k + 1) * (1.0 if it % 2 else -1.0) for k in range(C)]
            nsh = [shape[k] + 0.02 * (k - 1) for k in range(C)]
            st = ctx.factor_chains(1, 7, "exponential_isotropic", [[1.0, math.exp(s), 0.0] for s in nsh])
            ctx.ancillary_propose_chains(7, b0, [nls[k] - ls[k] for k in range(C)])
            v = ctx.field_response_ratio_chains(7, b0, lnv)
            want[("ratio", str(it))] = list(v)
            for k in range(C):
                if st[k] == 0 and v[k] > lu_anc[k]:
                    shape[k], ls[k] = nsh[k], nls[k]
                    ctx.select(k)
                    ctx.accept_field()
                    ctx.accept_factor()
            nls = [ls[k] - 0.03 * (k + 1) for k in range(C)]
            nsh = [shape[k] + 0.01 * (2 - k) for k in range(C)]
            st = ctx.factor_chains(1, 7, "exponential_isotropic", [[1.0, math.exp(s), 0.0] for s in nsh])
            l1 = ctx.loglik_chains(1, 7, b0, nls)
            l0 = ctx.loglik_chains(0, 7, b0, ls)
            want[("l1", str(it))], want[("l0", str(it))] = list(l1), list(l0)
            for k in range(C):
                if st[k] == 0 and l1[k] - l0[k] > lu_suf[k]:
                    shape[k], ls[k] = nsh[k], nls[k]
                    ctx.select(k)
                    ctx.accept_factor()
                ctx.select(k)
                oqo, oqf = ctx.beta0_stats()
                want[("beta0_stats", str(it), str(k))] = [oqo, oqf]
                b0[k] = 0.5 * oqf / oqo + 0.1 * k
                ctx.set_mu(None, b0[k])
            ctx.sweep_chains(NC, b0, ls, lnv, [11, 12, 13], [(it - 1) * NC] * C)
            ssr = ctx.sum_squared_residuals_chains(7, b0)
            want[("ssr", str(it))] = list(ssr)
            lnv = [lnv[k] + (0.01 if ssr[k] > n * math.exp(lnv[k]) else -0.01) for k in range(C)]
            for k in range(C):
                ctx.select(k)
                ctx.record_field(it - 1)
        for k in range(C):
            ctx.select(k)
            rec = ctx.get_records(0, NIT)
            for r in range(NIT):
                want[("record", str(k), str(r))] = list(rec[r])
            want[("field", str(k))] = list(ctx.get_field())
    assert set(got) == set(want), sorted(set(got) ^ set(want))
    for key in want:
        np.testing.assert_array_equal(np.array(got[key]), np.array(want[key]), err_msg=str(key))
