"""Import helper: the package directory name is not a Python identifier
(it carries the reference repo's name), so it is loaded under the alias
``nngp_amd``.  Used by tests/, bench.py and __graft_entry__.py."""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_NAME = ("improving-performances-of-mcmc-for-nearest-neighbor-gaussian-process-models"
            "-with-full-data-augmentat_amd")
PKG_DIR = ROOT / PKG_NAME
ALIAS = "nngp_amd"


def load():
    if ALIAS in sys.modules:
        return sys.modules[ALIAS]
    spec = importlib.util.spec_from_file_location(ALIAS, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[ALIAS] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[ALIAS]
        raise
    return mod
