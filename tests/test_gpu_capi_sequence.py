"""A C client of include/nngp.h (tests/cpp/capi_sequence.c: the call sequence
of the R drop-in, rpkg/R/mcmc_nngp_update_Gaussian.R) gives exactly what the
same sequence gives through the Python binding: the boundary carries no
hidden state of the binding."""
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
