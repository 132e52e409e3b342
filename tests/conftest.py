import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long statistical test")


@pytest.fixture(scope="session")
def P():
    import _pkgload

    return _pkgload.load()


@pytest.fixture(scope="session")
def O():
    import oracle

    return oracle


@pytest.fixture(scope="session")
def printed():
    return json.loads((GOLDEN / "vignette_printed.json").read_text())


@pytest.fixture(scope="session")
def toy():
    return dict(np.load(GOLDEN / "vignette_toy.npz"))


def make_problem(P, n, m, d=2, seed=0, order=True, dup_frac=0.0):
    """Synthetic ordered locations + NNarray + colouring (+ duplicated obs)."""
    rng = np.random.default_rng(seed)
    locs = rng.uniform(size=(n, d))
    if order:
        locs = locs[P.order_maxmin(locs) - 1]
    NN = P.find_ordered_nn(locs, m)
    col = P.naive_greedy_coloring(NN)
    lm = np.arange(1, n + 1, dtype=np.int32)
    if dup_frac > 0:
        extra = rng.choice(n, int(dup_frac * n), replace=False) + 1
        lm = np.concatenate([lm, extra.astype(np.int32)])
    y = rng.normal(size=len(lm))
    return locs, NN, col, lm, y


@pytest.fixture(scope="session")
def heavy():
    """Heavy_metals/processed_data.RDS (run_script.R:8-12) as parsed by
    tests/golden/make_heavy_metals.py: observed_locs (lon/lat), observed_field,
    X_locs as a data.frame with its 3 factors in their stored level order."""
    import pandas as pd

    d = np.load(Path(__file__).resolve().parent / "golden" / "heavy_metals.npz")
    cols = {}
    num = dict(zip(d["X_num_names"], d["X_num"].T))
    for c in d["column_order"]:
        if c in num:
            cols[c] = num[c]
        else:
            levels = list(d[f"levels_{c}"])
            cols[c] = pd.Categorical.from_codes(d[f"fac_{c}"] - 1, categories=levels)
    return {"observed_locs": d["observed_locs"], "observed_field": d["observed_field"],
            "X_locs": pd.DataFrame(cols)}


# Sweep engines of the device context (capi.hip): "colors" = one launch per
# colour class; "tiles" = the tile-resident persistent sweep with many small
# tiles (NNGP_TILES=24: every small test problem has halos, neighbour
# hand-offs and several tiles per XCD; contexts whose 24-tile layout does not
# fit a CU's LDS fall back to colour launches, as in production);
# "tiles-default" = the production engine choice and tile count (exchange-wave
# tiles: the last wave of each tile polls the hand-offs); "tiles-classic" =
# the same tiles without the exchange wave (NNGP_TILE_XW=0: every wave polls).
# GPU test modules that exercise the sweep run under all four.
ENGINES = {"colors": {"NNGP_ENGINE": "colors"},
           "tiles": {"NNGP_TILES": "24"},  # automatic: colours where 24 tiles exceed the LDS
           "tiles-default": {},
           "tiles-classic": {"NNGP_TILE_XW": "0"}}


@pytest.fixture(params=list(ENGINES))
def engine(request, monkeypatch):
    monkeypatch.delenv("NNGP_TILES", raising=False)
    monkeypatch.delenv("NNGP_ENGINE", raising=False)
    monkeypatch.delenv("NNGP_TILE_XW", raising=False)
    for k, v in ENGINES[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param
