"""CPU-side checks of the product library: it loads, exports every symbol
the C ABI header declares, and its host-side graph preparation is bit-exact
against the oracle (no GPU compute is called here)."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def test_header_symbols_exported(P):
    hdr = (ROOT / "include" / "nngp.h").read_text()
    declared = set(re.findall(r"\b(nngp_[a-z0-9_]+)\s*\(", hdr))
    from nngp_amd import _lib

    assert declared == set(_lib.ABI_SYMBOLS)
    lib = C.CDLL(str(_lib.LIB_PATH))
    for s in sorted(declared):
        assert hasattr(lib, s), s
    assert P.lib.nngp_abi_version() == 14


def test_library_has_gfx950_code_object():
    from nngp_amd import _lib

    blob = Path(_lib.LIB_PATH).read_bytes()
    assert b"gfx950" in blob


@pytest.mark.parametrize("n,d,m,seed", [(1, 2, 3, 0), (2, 2, 3, 0), (7, 2, 10, 1), (500, 2, 5, 2),
                                        (3000, 2, 10, 3), (2000, 3, 15, 4), (1500, 1, 4, 5),
                                        (800, 4, 8, 6), (2500, 2, 30, 7)])
def test_graph_prep_bit_exact_vs_oracle(P, O, n, d, m, seed):
    rng = np.random.default_rng(seed)
    locs = rng.uniform(size=(n, d))
    o1 = P.order_maxmin(locs)
    np.testing.assert_array_equal(o1, O.order_maxmin_exact(locs))
    L = locs[o1 - 1]
    a = P.find_ordered_nn(L, m)
    b = O.find_ordered_nn(L, min(m, n - 1))
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(P.naive_greedy_coloring(a), O.greedy_coloring(b))


def test_nn_ties_and_duplicates(P, O):
    # integer grid: many equal distances -> ties broken by the smaller index
    g = np.array([(x, y) for x in range(20) for y in range(20)], np.float64)
    g = g[np.random.default_rng(0).permutation(len(g))]
    for m in [4, 8, 12]:
        np.testing.assert_array_equal(P.find_ordered_nn(g, m), O.find_ordered_nn(g, m))
    dup = np.vstack([g[:50], g[:50]])  # exact duplicates (distance 0)
    np.testing.assert_array_equal(P.find_ordered_nn(dup, 5), O.find_ordered_nn(dup, 5))
    np.testing.assert_array_equal(P.order_maxmin(g), O.order_maxmin_exact(g))


def test_product_nn_on_vignette_prefix(P, printed, toy, O):
    h = np.array(printed["hctam_scol_1_100"]) - 1
    NN = P.find_ordered_nn(toy["locs"][h], 5)
    head = np.array([[O.NA if v is None else v for v in r] for r in printed["NNarray_head"]])
    np.testing.assert_array_equal(NN[:6], head)


def test_vignette_full_toy_graph(P, O, toy):
    """Full 2000-point toy (our exact max-min ordering of the regenerated
    locations): product NN + colouring == oracle."""
    locs = toy["locs"]
    o = P.order_maxmin(locs)
    L = locs[o - 1]
    NN = P.find_ordered_nn(L, 5)
    np.testing.assert_array_equal(NN, O.find_ordered_nn(L, 5))
    col = P.naive_greedy_coloring(NN)
    np.testing.assert_array_equal(col, O.greedy_coloring(NN))
    n = len(L)
    assert (NN != O.NA).sum() == n * 6 - 15  # nnz(B) = n(m+1) - m(m+1)/2


def test_sparse_chol_indices(P):
    NN = np.array([[1, P.find_ordered_nn.__globals__["NA_INTEGER"], -2 ** 31], [2, 1, -2 ** 31], [3, 1, 2]], np.int32)
    non_na, row_idx, col_idx = P.sparse_chol_indices(NN)
    # column-major vectorisation: self column first (initialize.R:97-101)
    np.testing.assert_array_equal(col_idx, [1, 2, 3, 1, 1, 2])
    np.testing.assert_array_equal(row_idx, [1, 2, 3, 2, 3, 3])


def test_ctx_create_without_gpu_fails_loudly(P):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    locs = np.random.default_rng(0).uniform(size=(10, 2))
    NN = P.find_ordered_nn(locs, 3)
    with pytest.raises(P.NNGPError) as e:
        P.ChainContext(locs, NN, P.naive_greedy_coloring(NN), np.arange(1, 11, dtype=np.int32), np.zeros(10))
    assert e.value.status == 6  # NNGP_ERR_NODEV: no silent CPU fallback


def test_shape_transforms():
    import _pkgload

    M = _pkgload.load().model
    sp = M.shape_params_of("matern_isotropic", 2)
    assert sp == ["log_range", "qlogis_smoothness"]
    np.testing.assert_allclose(M.covparms(sp, [np.log(3.0), 0.0]), [1.0, 3.0, 0.75, 0.0])
    np.testing.assert_allclose(M.covparms(sp, [0.0, 0.0], 0.4, 0.7), [1.0, 1.0, 0.75, 0.0])
    assert M.shape_params_of("exponential_scaledim", 3) == ["log_range_1", "log_range_2", "log_range_3"]


def test_gelman_rubin_on_identical_chains(P):
    rng = np.random.default_rng(0)
    recs = {f"chain_{i}": {"params": {"beta_0": rng.normal(size=(400, 1)), "log_scale": rng.normal(size=(400, 1))}}
            for i in range(3)}
    g = P.Gelman_Rubin_Brooks(recs, 0.5)
    assert np.all(g["R_hat"] < 1.05)
    E, _ = P.ESS(recs, 0.5)
    assert np.all(E[:-1] > 100)


@pytest.mark.parametrize("n,m,lw,seed", [(3000, 10, 64, 1), (5000, 15, 32, 2), (8000, 15, 16, 3),
                                         (2000, 30, 16, 4), (4000, 12, 21, 7), (50, 3, 64, 5), (1, 0, 64, 6)])
def test_sweep_layout_invariants(tmp_path, n, m, lw, seed):
    """C++ check of the planner: every nonzero of B exactly once, at the
    address the sweep kernel computes from the colour class table."""
    import subprocess

    csrc = next(ROOT.glob("*_amd")) / "csrc"
    exe = tmp_path / "layout_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(csrc), str(ROOT / "tests/cpp/layout_check.cpp"),
                    str(csrc / "graph_prep.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(n), str(m), str(lw), str(seed)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


@pytest.fixture(scope="module")
def tile_check_exe(tmp_path_factory):
    import subprocess

    csrc = next(ROOT.glob("*_amd")) / "csrc"
    exe = tmp_path_factory.mktemp("tiles") / "tile_sweep_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(csrc), str(ROOT / "tests/cpp/tile_sweep_check.cpp"),
                    str(csrc / "graph_prep.cpp"), "-o", str(exe)], check=True)
    return exe


@pytest.mark.parametrize("n,m,tiles,chains,seed,nt,rmax", [
    (1500, 10, 16, 2, 1, 256, 16), (800, 5, 7, 3, 2, 64, 4), (300, 8, 1, 1, 3, 256, 16),
    (2000, 15, 40, 4, 4, 128, 2), (1200, 12, 256, 1, 5, 256, 16), (5, 2, 8, 2, 6, 64, 1),
    (200000, 15, 24, 1, 21, 512, 8)])
def test_tile_sweep_emulation(tile_check_exe, n, m, tiles, chains, seed, nt, rmax):
    """C++ emulation of the tile-resident sweep kernel step by step on the
    tile layout (own batches, thread runs and tails, slot totals, published
    dw, ghost cells after the neighbour hand-off) against a plain serial
    local-form chromatic sweep: same field to 1e-11 after 2 sweeps; also
    checks the layout (each nonzero once, local rows, exported slots,
    neighbour lists).  Small NT/RMAX force several batches per colour."""
    import subprocess

    out = subprocess.run([str(tile_check_exe), str(n), str(m), str(tiles), str(chains), str(seed), str(nt),
                          str(rmax)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


@pytest.mark.parametrize("args", [("30000", "15", "64", "3", "5", "512", "8", "8", "0"),
                                  ("20000", "10", "40", "1", "2", "256", "16", "1", "0"),
                                  ("20000", "10", "48", "3", "3", "512", "8", "4", "1")])
def test_tile_layout_independent_of_host_threads(tile_check_exe, args):
    """The tile layout is built per tile on host threads and concatenated in
    tile order: every layout array (hashed) is the same with 1 and 8 threads."""
    import os
    import subprocess

    outs = []
    for th in ("1", "8"):
        env = dict(os.environ, NNGP_HOST_THREADS=th)
        out = subprocess.run([str(tile_check_exe), *args], capture_output=True, text=True, env=env)
        assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
        outs.append(out.stdout.split("layout=")[1].split()[0])
    assert outs[0] == outs[1]


@pytest.mark.parametrize("n,m,tiles,chains,seed,nt,rmax,G", [
    (3000, 10, 16, 3, 1, 256, 16, 1), (1500, 10, 16, 3, 2, 64, 4, 1), (60000, 15, 64, 3, 5, 512, 8, 1),
    (5000, 15, 24, 3, 6, 256, 16, 8), (40, 3, 8, 4, 7, 64, 1, 2)])
def test_tile_sweep_emulation_split_schedule(tile_check_exe, n, m, tiles, chains, seed, nt, rmax, G):
    """Interior-first layouts (NNGP_TILE_SPLIT=1, kernels.hip tile_phase_ib):
    the emulation runs the kernel's schedule -- per colour c every tile's
    interior batches, then the hand-off of colour c-1, then the boundary
    batches -- so an interior slot that read a row still missing its
    colour-(c-1) ghost update would break the 1e-11 bar against the serial
    sweep."""
    import subprocess

    out = subprocess.run([str(tile_check_exe), str(n), str(m), str(tiles), str(chains), str(seed), str(nt), str(rmax),
                          str(G), "1"], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


@pytest.mark.parametrize("n,m,tiles,G,chains,seed", [
    (3000, 10, 16, 2, 1, 1), (5000, 15, 24, 8, 3, 2), (2000, 8, 12, 3, 2, 3), (400, 5, 16, 16, 1, 4),
    (60000, 15, 64, 8, 1, 5), (8, 2, 8, 8, 1, 6)])
def test_tile_shard_plan_emulation(tile_check_exe, n, m, tiles, G, chains, seed):
    """Tile shard: the emulation with one granule buffer per
    rank, poisoned before every colour, so a ghost cell of another rank's
    slot only sees the draw through the plan's remote puts; the remote-reader
    masks must equal the brute-force set of reader ranks, and the ranks' slot
    ranges hold exactly their tiles' slots.  Same 1e-11 bar against the
    serial sweep."""
    import subprocess

    out = subprocess.run([str(tile_check_exe), str(n), str(m), str(tiles), str(chains), str(seed), "256", "16",
                          str(G)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
    assert G == 1 or int(out.stdout.split("remote_puts=")[1].split()[0]) > 0 or n < 16


@pytest.mark.parametrize("n,m,tiles,chains,seed,rmax,G,waves", [
    (3000, 10, 16, 3, 1, 8, 1, 7), (60000, 15, 64, 3, 5, 8, 1, 7), (20000, 10, 40, 1, 2, 8, 4, 7),
    (5000, 15, 24, 2, 6, 4, 8, 3), (400, 5, 16, 4, 7, 1, 2, 7)])
def test_tile_sweep_emulation_wave_local(tile_check_exe, n, m, tiles, chains, seed, rmax, G, waves):
    """Wave-local layouts (NNGP_TILE_WL=1, tiles.hip tile_phase_wl): 64-lane
    batches of at most kWaveSlotsMax slots in rounds of `waves` balanced by
    cells.  The emulation applies the batches of a colour one after another
    -- the kernel's waves run them side by side, which gives the same result
    because the batches of one colour touch disjoint rows -- and checks the
    field against the serial sweep (1e-11) and the layout, incl. the tile
    shard's remote puts (G > 1)."""
    import subprocess

    out = subprocess.run([str(tile_check_exe), str(n), str(m), str(tiles), str(chains), str(seed), "64", str(rmax),
                          str(G), "0", "2", str(waves)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


@pytest.mark.parametrize("n,m,tiles,chains,seed,G", [
    (3000, 10, 16, 3, 1, 1), (60000, 15, 64, 3, 5, 1), (20000, 10, 40, 4, 2, 4), (400, 5, 16, 3, 7, 2)])
def test_tile_sweep_emulation_wave_local_interior_first(tile_check_exe, n, m, tiles, chains, seed, G):
    """Interior-first wave-local layouts (NNGP_TILE_SPLIT=1 on wave-local
    batches, tiles.hip tile_phase_wlib): per colour the interior run, then the
    boundary run, each cut into 64-lane batches in rounds of 7 waves.  The
    emulation runs the kernel's schedule -- every tile's interior batches of
    colour c, the ghost adds of colour c-1, the boundary batches of c -- and
    checks the field against the serial sweep (1e-11) and the layout."""
    import subprocess

    out = subprocess.run([str(tile_check_exe), str(n), str(m), str(tiles), str(chains), str(seed), "64", "8",
                          str(G), "1", "2", "7"], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


def test_interior_first_wave_local_barrier_counts_match():
    """Interior-first wave-local tiles (tiles.hip tile_phase_wlib, opt-in): the
    cell waves pass three workgroup barriers per phase (A: the hand-off is in,
    B: the ghost adds are done, C: the boundary batches are done) and the
    exchange wave's lagged phase (tile_phase_xw<..., LAG = 1>) must pass the
    same three, also at ph = 0 where it has nothing to hand off; a mismatch
    pairs barriers wrongly (an LDS race or a spin timeout)."""
    src = (next(ROOT.glob("*_amd")) / "csrc" / "tiles.hip").read_text()
    wlib = src.split("void tile_phase_wlib(", 1)[1].split("\n}\n", 1)[0]
    assert wlib.count("__syncthreads()") == 3, wlib.count("__syncthreads()")
    xw = src.split("void tile_phase_xw(", 1)[1].split("\n}\n", 1)[0]
    first = xw.split("if (LAG && ph == 0) {", 1)[1].split("return;", 1)[0]
    assert first.count("__syncthreads()") == 3
    # the lagged phase (wave-local: no own-batch barriers): after the polls,
    # after the ghost adds, and C (not in the epilogue ph = nph)
    rest = xw.split("return;", 1)[1].split("// hand-off: every (foreign slot, chain)", 1)[1]
    assert "if (LAG && ph < S.nph) __syncthreads();" in rest
    assert rest.count("__syncthreads()") == 3, rest.count("__syncthreads()")


def test_exchange_wave_barrier_count_matches_own_draw():
    """The exchange wave of a tile (tiles.hip tile_phase_xw) holds no cells and
    passes the own batches' workgroup barriers by count: kOwnDrawBarriers must
    equal the __syncthreads() in tile_own_draw (a mismatch pairs the barriers
    wrongly: an LDS race or a spin timeout), and tile_phase_xw must use it."""
    import re

    src = (next(ROOT.glob("*_amd")) / "csrc" / "tiles.hip").read_text()
    k = int(re.search(r"constexpr int kOwnDrawBarriers = (\d+);", src).group(1))
    body = src.split("void tile_own_draw(", 1)[1].split("\ntemplate", 1)[0]
    assert body.count("__syncthreads()") == k, (body.count("__syncthreads()"), k)
    xw = src.split("void tile_phase_xw(", 1)[1].split("\ntemplate", 1)[0]
    assert "q < kOwnDrawBarriers; ++q) __syncthreads();" in xw


def test_configs4_tile_shard_geometry(tile_check_exe):
    """configs[4] (BASELINE.json: n = 1e7, m = 20, colour classes sharded over
    8 GPUs) at its per-rank tile shape, scaled down: a G = 8 tile shard of
    n = 1.25e6 with 32 tiles per rank has the tiles of the real layout (8 x 256
    tiles of n/T = 4,883 locations, m = 20); at n = 1e7 itself the largest
    tile holds 6,907 local rows (scripts/layout_stats.cpp 1e7 20 2048: 2m44s
    on the host, too long for this suite) against 6,568 here.  The emulation
    (one chain, one sweep) checks the remote-reader plan and the sweep at that
    geometry.  The LDS a 512-thread workgroup needs with r in LDS: 3 chains
    (the bench's chain count) exceed a CU's 160 KiB, 2 chains fit -- so
    configs[4] at 3 chains runs the tile shard with r in global memory (RG
    tiles, whose LDS is far below the CU's) and a 2-chain context the LDS
    tiles (DESIGN.md §6 "configs[4] on eight GPUs")."""
    import subprocess

    out = subprocess.run([str(tile_check_exe), "1250000", "20", "256", "1", "11", "448", "8", "8", "0", "1"],
                         capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr
    kv = dict(x.split("=", 1) for x in out.stdout.split()[1:])
    assert kv["G"] == "8" and kv["T"] == "256" and int(kv["remote_puts"]) > 0
    lds = [0] + [int(v) for v in kv["lds"].split(",")]
    lds_rg = [0] + [int(v) for v in kv["lds_rg"].split(",")]
    cu = int(kv["cu_lds"])
    assert cu == 160 * 1024
    rows = int(kv["max_rows"])
    assert 6000 < rows <= 6907, rows
    assert lds[3] > cu, (lds, cu)      # 3 chains: r alone is rows x 24 B
    assert lds[2] <= cu, (lds, cu)     # 2 chains fit
    assert lds_rg[3] <= cu // 4, lds_rg
    # the real layout's largest tile only widens the gap at 3 chains
    assert 6907 * 3 * 8 > cu


@pytest.mark.parametrize("n,m,G,sweeps,seed", [(3000, 10, 2, 2, 1), (5000, 15, 3, 2, 2), (2000, 5, 8, 2, 3),
                                               (50, 3, 4, 1, 4), (1, 0, 2, 1, 5), (20000, 15, 8, 1, 6),
                                               (4000, 12, 1, 2, 7)])
def test_shard_plan_emulation(tmp_path, n, m, G, sweeps, seed):
    """C++ emulation of the colour-sharded sweep on its plan (graph_prep.cpp
    build_shard_plan): G ranks with their own r and w replicas, own chunks,
    exchange regions, ghost cells and replica updates reproduce the
    single-rank sweep bitwise after every colour; the ranks' segments
    partition every colour; normal pairs cover every owned location."""
    import subprocess

    csrc = next(ROOT.glob("*_amd")) / "csrc"
    exe = tmp_path / "shard_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(csrc), str(ROOT / "tests/cpp/shard_check.cpp"),
                    str(csrc / "graph_prep.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(n), str(m), str(G), str(sweeps), str(seed)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


def test_predict_fixed_effects_closed_form(P):
    """mcmc_nngp_predict_fixed_effects (predict.R:67-104) on a hand-made list:
    beta_0 de-centred by X_mean (:94), columns matched by name (:87), no
    intercept by default (:81-85), burn-in on the saved iterations (:73)."""
    import pandas as pd

    beta0 = np.array([[1.0], [2.0], [3.0], [4.0]])
    beta = np.array([[0.5, -1.0], [0.6, -1.1], [0.7, -1.2], [0.8, -1.3]])
    L = {"X": {"names": ["a", "b"], "X_mean": np.array([10.0, 20.0])},
         "records": {"chain_1": {"saved_field": np.array([1.0, 2.0, 3.0, 4.0]),
                                 "iterations": np.array([[0, 0.0], [4, 1.0]]),
                                 "params": {"beta_0": beta0, "beta": beta}}}}
    Xp = pd.DataFrame({"b": [1.0, 2.0], "a": [3.0, 0.5]})
    out = P.mcmc_nngp_predict_fixed_effects(L, Xp, burn_in=0.5)
    s = out["predicted_fixed_effects_samples"][0]
    # stored iterations 3, 4 (> .5 * 4); model matrix columns (b, a) -> beta (b, a)
    exp = np.array([[beta[k, 1] * 1.0 + beta[k, 0] * 3.0, beta[k, 1] * 2.0 + beta[k, 0] * 0.5] for k in (2, 3)])
    np.testing.assert_allclose(s, exp, rtol=1e-15)
    out = P.mcmc_nngp_predict_fixed_effects(L, Xp, burn_in=0.5, add_intercept=True)
    s = out["predicted_fixed_effects_samples"][0]
    b0 = beta0[2:, 0] - beta[2:] @ np.array([10.0, 20.0])
    exp2 = np.column_stack([b0, b0]) + exp
    np.testing.assert_allclose(s, exp2, rtol=1e-14)


def test_predict_oracle_reuses_factor_like_predict_R(O):
    """The oracle's predict.R restatement recomputes the factor only at the
    first appearance of a shape (!duplicated, predict.R:23,32): a later return
    to an earlier shape keeps the most recent factor (a reference quirk)."""
    rng = np.random.default_rng(0)
    n, m = 60, 4
    locs = rng.uniform(size=(n, 2))
    pred = rng.uniform(size=(7, 2))
    a, b = np.log(0.3), np.log(0.1)
    fields = rng.normal(size=(3, n))
    L = {"locs": locs, "space_time_model": {"covfun": {"stationary_covfun": "exponential_isotropic",
                                                       "shape_params": ["log_range"]}},
         "records": {"chain_1": {"saved_field": np.array([1.0, 2.0, 3.0]),
                                 "params": {"shape": np.array([[a], [b], [a]]), "log_scale": np.zeros((3, 1)),
                                            "beta_0": np.zeros((3, 1)), "field": fields}}}}
    z = [rng.normal(size=(3, 7))]
    got = O.predict_field(L, pred, z, burn_in=0.0, m=m)[0]
    allloc = np.vstack([locs, pred])
    NN = O.find_ordered_nn(allloc, m)
    Lb = O.vecchia_linv("exponential_isotropic", [1.0, np.exp(b), 0.0], allloc, NN)
    u = O.linv_mult(Lb, np.concatenate([fields[2], np.zeros(7)]), NN)[:n]
    x = O.tri_solve(Lb, NN, np.concatenate([u, z[0][2]]))
    np.testing.assert_allclose(got[2], x[n:], rtol=1e-13, atol=1e-13)
    # and the dense form: B x = c(B11 w, z)
    B = O.dense_B(Lb, NN)
    np.testing.assert_allclose(B @ x, np.concatenate([B[:n, :n] @ fields[2], z[0][2]]), atol=1e-10)


class _FailingCtx:
    """Stand-in device context whose proposal factor (which = 1) fails with a
    given nngp status: exercises the MH step's error handling on the host."""

    def __init__(self, status):
        self.status = status

    def factor(self, which, covfun, cp):
        from nngp_amd._lib import NNGPError

        if which == 1:
            raise NNGPError(self.status, "injected")

    def set_field(self, f):
        pass

    def set_mu(self, mu, b0):
        pass

    def beta0_stats(self):
        return 1.0, 0.0

    def sum_squared_residuals(self, b0):
        return 1.0

    def get_field(self):
        return np.zeros(4)

    def sweep(self, *a):
        pass


class _FailingStepCtx(_FailingCtx):
    """The same failure through the one-sync MH step entry points
    (nngp_ancillary_step_chains / nngp_sufficient_step_chains): a CHOL
    failure is a per-chain status, any other failure raises."""

    n_chains = 1

    def _step(self):
        from nngp_amd._lib import NNGP_ERR_CHOL, NNGPError

        if self.status != NNGP_ERR_CHOL:
            raise NNGPError(self.status, "injected")
        return np.array([self.status], np.int32)

    def ancillary_step_chains(self, mask, covfun, cps, b0, dls, lnv):
        assert mask == 1 and cps.shape[0] == 1
        return self._step(), np.array([np.nan])

    def sufficient_step_chains(self, mask, covfun, cps, b0, lsp, lsc):
        assert mask == 1 and cps.shape[0] == 1
        return self._step(), np.array([np.nan]), np.array([np.nan])


def _drive_one(g, ctx):
    """Run a chain program against one context (update_gaussian._run_chain's
    loop): -> the request kinds it issued, in order."""
    from nngp_amd.update_gaussian import _serve_one

    kinds = []
    try:
        req = next(g)
        while True:
            kinds.append((req[0], req[2] is not None if req[0] in ("astep", "sstep") else True))
            req = g.send(_serve_one(ctx, req))
    except StopIteration:
        return kinds


def _program(ctx, on_chol_error):
    from nngp_amd.update_gaussian import _chain_program

    va = {"n_obs": 4, "n_locs": 4, "locs_match": np.arange(1, 5)}
    stm = {"covfun": {"stationary_covfun": "exponential_isotropic", "shape_params": ["log_range"]}}
    state = {"params": {"beta_0": 0.0, "beta": None, "log_scale": -5.0, "shape": np.array([0.0]),
                        "log_noise_variance": 0.0, "field": np.zeros(4)},
             "transition_kernels": {"covariance_params_sufficient": {"logvar": -2.0},
                                    "covariance_params_ancillary": {"logvar": -2.0},
                                    "log_noise_variance": {"logvar": -1.0}}}
    return _chain_program(0, state, ctx, {"X": None, "locs": []}, np.array([0.0, 1.0, 2.0, 3.0]), stm, va,
                          1, 0.0, True, 1, 0, 1, on_chol_error)


def test_mh_proposal_factor_failures(P):
    """update_Gaussian.R:123,179: GpGp raises on a non positive definite local
    covariance, which ends the update (default on_chol_error="error"); with
    "reject" only that status rejects the proposal; every other failure
    (here a HIP error) propagates in both modes."""
    from nngp_amd._lib import NNGP_ERR_CHOL, NNGP_ERR_HIP, NNGPError

    for Ctx in (_FailingCtx, _FailingStepCtx):  # separate calls / one-sync step entry points
        with pytest.raises(NNGPError) as e:
            _drive_one(_program(Ctx(NNGP_ERR_CHOL), "error"), Ctx(NNGP_ERR_CHOL))
        assert e.value.status == NNGP_ERR_CHOL
        kinds = _drive_one(_program(Ctx(NNGP_ERR_CHOL), "reject"), Ctx(NNGP_ERR_CHOL))
        # both proposals rejected (their ratio / log-likelihoods unused), the iteration goes on
        assert kinds == [("astep", True), ("sstep", True), ("sweep", True), ("ssr", True)], kinds
        for mode in ("error", "reject"):
            with pytest.raises(NNGPError) as e:
                _drive_one(_program(Ctx(NNGP_ERR_HIP), mode), Ctx(NNGP_ERR_HIP))
            assert e.value.status == NNGP_ERR_HIP


def test_r_shim_wraps_every_abi_entry_point():
    """rpkg/src/nngp_shim.c: one registered .Call routine per function of
    include/nngp.h (nngp_ctx_last_error / status_string included), and the
    shim compiles (a declarations-only R API stand-in under tests/cpp: this
    image has no R; `R CMD INSTALL rpkg` builds it against R's headers)."""
    import subprocess

    root = Path(__file__).resolve().parent.parent
    hdr = (root / "include" / "nngp.h").read_text()
    shim = (root / "rpkg" / "src" / "nngp_shim.c").read_text()
    declared = set(re.findall(r"\b(nngp_[a-z0-9_]+)\s*\(", hdr)) - {"nngp_ctx"}
    for fn in sorted(declared):
        assert re.search(rf"\b{fn}\s*\(", shim.split("#include \"nngp.h\"")[1]), f"{fn} not called by the shim"
    registered = set(re.findall(r"E\((C_nngp_[a-z0-9_]+),", shim))
    defined = set(re.findall(r"^SEXP (C_nngp_[a-z0-9_]+)\(", shim, re.M))
    assert registered == defined and len(defined) >= len(declared) - 2
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-cast-function-type", "-fsyntax-only",
                        f"-I{root / 'tests' / 'cpp' / 'r_api_stub'}", f"-I{root / 'include'}",
                        str(root / "rpkg" / "src" / "nngp_shim.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rfun = (root / "rpkg" / "R" / "nngp.R").read_text() + (root / "rpkg" / "R" / "mcmc_nngp_update_Gaussian.R").read_text()
    for c in defined:
        assert c in rfun, f"{c} has no R wrapper"


def test_log_unit_accuracy(tmp_path):
    """device_common.h log_unit (the log in the AS241 tail of the sweep's
    normals, hardware reciprocal + atanh series) within 2 ulp of libm's log
    over 4e6 of the sweep's uniforms and their scalings down to 2^-112
    (host build of the same header with hipcc; no GPU needed)."""
    import subprocess

    root = Path(__file__).resolve().parent.parent
    exe = tmp_path / "log_unit_check"
    inc = root / "improving-performances-of-mcmc-for-nearest-neighbor-gaussian-process-models-with-full-data-augmentat_amd" / "csrc"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", f"-I{inc}", str(root / "tests" / "cpp" / "log_unit_check.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "max_ulp" in r.stdout


def test_r_records_transpose_matches_row_major(tmp_path):
    """rpkg/src/nngp_rows.h (C_nngp_get_records): k row-major record rows ->
    the first k rows of R's column-major records$field matrix, in cache
    blocks, straight out of the bound vector (no temporary) -- checked
    against numpy for sizes around the 64 x 64 block edges."""
    import subprocess

    root = Path(__file__).resolve().parent.parent
    src = tmp_path / "t.c"
    src.write_text(r"""
#include <stdio.h>
#include <stdlib.h>
#include "nngp_rows.h"
int main(int argc, char** argv) {
  const ptrdiff_t ld = atol(argv[1]), k = atol(argv[2]), n = atol(argv[3]);
  double* s = malloc(sizeof(double) * (k * n + 1));
  double* d = malloc(sizeof(double) * (ld * n + 1));
  for (ptrdiff_t e = 0; e < k * n; ++e) s[e] = (double)e;
  for (ptrdiff_t e = 0; e < ld * n; ++e) d[e] = -1.0;
  nngp_rows_to_colmajor(s, d, ld, k, n);
  fwrite(d, sizeof(double), ld * n, stdout);
  return 0;
}
""")
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-O2", "-std=c99", "-Wall", "-Werror", f"-I{root / 'rpkg' / 'src'}", str(src), "-o", str(exe)],
                   check=True)
    for ld, k, n in [(1, 1, 1), (3, 3, 7), (64, 64, 64), (65, 65, 129), (200, 130, 70), (40, 17, 1000)]:
        out = subprocess.run([str(exe), str(ld), str(k), str(n)], capture_output=True, check=True).stdout
        got = np.frombuffer(out, np.float64).reshape(n, ld).T  # column-major ld x n
        rows = np.arange(k * n, dtype=np.float64).reshape(k, n)
        np.testing.assert_array_equal(got[:k], rows)
        assert np.all(got[k:] == -1.0)


def test_chain_groups_split_where_tiles_exceed_the_lds(P, monkeypatch):
    """context.make_chain_views: a chain group whose context fell back to the
    colour engine for the LDS (engine_fallback 1) or keeps r in global memory
    is reopened as two halves, recursively, when half the chains' rows fit the
    LDS; other fallbacks, NNGP_SPLIT_CHAINS=0 and NNGP_TILE_R=global keep one
    context (host logic, fake contexts: no GPU)."""
    opened, closed = [], []

    class Fake:
        def __init__(self, *a, device=0, n_chains=1):
            self.n_chains = n_chains
            opened.append(n_chains)
            fits = n_chains <= fits_at
            note = "tiles" if fits else ("colours (tile engine not used: tile layout needs 170000 B of LDS per tile"
                                         if lds else "colours (tile engine not used: residency)")
            if not fits and rg:
                note = "tiles: 256 tiles of 512 threads, r in global memory"
            self.info = {"sweep_engine": 1 if fits or rg else 0,
                         "engine_fallback": 0 if fits or rg else (1 if lds else 2),
                         "engine_note": note, "tile_rows_needed": rows, "device_lds": 160 * 1024}

        def view(self, k):
            return (self, k)

        def close(self):
            closed.append(self.n_chains)

    monkeypatch.setattr(P.context, "ChainContext", Fake)
    monkeypatch.delenv("NNGP_SPLIT_CHAINS", raising=False)
    monkeypatch.delenv("NNGP_TILE_R", raising=False)
    fits_at, lds, rg, rows = 2, True, False, 5000
    v = P.context.make_chain_views(None, None, None, None, None, 4, devices=[0])
    assert opened == [4, 2, 2] and closed == [4]
    assert [k for _, k in v] == [0, 1, 0, 1] and v[0][0] is v[1][0] and v[2][0] is not v[0][0]
    opened.clear(); closed.clear()
    fits_at = 1
    v = P.context.make_chain_views(None, None, None, None, None, 3, devices=[0])
    assert opened == [3, 2, 1, 1, 1] and closed == [3, 2] and [k for _, k in v] == [0, 0, 0]
    opened.clear(); closed.clear()
    fits_at, lds = 2, False  # another reason (residency): no split
    v = P.context.make_chain_views(None, None, None, None, None, 4, devices=[0])
    assert opened == [4] and closed == []
    opened.clear(); closed.clear()
    lds = True
    monkeypatch.setenv("NNGP_SPLIT_CHAINS", "0")
    P.context.make_chain_views(None, None, None, None, None, 4, devices=[0])
    assert opened == [4] and closed == []
    monkeypatch.delenv("NNGP_SPLIT_CHAINS")
    opened.clear(); closed.clear()
    rows = 20000  # half the chains' rows still beyond the LDS (n = 1e7 on one GPU): no split
    P.context.make_chain_views(None, None, None, None, None, 4, devices=[0])
    assert opened == [4] and closed == []
    opened.clear(); closed.clear()
    rows, rg = 6907, True  # a tile shard with r in global memory (configs[4] at 3 chains): 2 + 1
    v = P.context.make_chain_views(None, None, None, None, None, 3, devices=[0])
    assert opened == [3, 2, 1] and closed == [3]
    opened.clear(); closed.clear()
    monkeypatch.setenv("NNGP_TILE_R", "global")  # asked for: kept
    P.context.make_chain_views(None, None, None, None, None, 3, devices=[0])
    assert opened == [3] and closed == []
