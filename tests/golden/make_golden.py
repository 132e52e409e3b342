"""Generate the committed golden fixtures (run once in the build container).

Sources:
* the values PRINTED in the reference's rendered vignette
  (/root/reference/Vignette.md) -- parsed as text, stored as data;
* the vignette's toy inputs regenerated bit-for-bit (7 printed digits) with
  the R RNG emulator (oracle/r_rng.py), `Vignette.rmd:26-48`.

Outputs (tests read ONLY these; /root/reference is absent on the GPU box):
  tests/golden/vignette_printed.json  -- printed golden values
  tests/golden/vignette_toy.npz       -- regenerated toy inputs

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
from __future__ import annotations

import json
import re
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT / "oracle"))


def _block_after(lines, marker, start=0):
    """Return the printed '##' lines of the first output block after `marker`."""
    i = start
    while marker not in lines[i]:
        i += 1
    # skip to first '    ##' line
    while not lines[i].startswith("    ##"):
        i += 1
    out = []
    while i < len(lines) and lines[i].startswith("    ##"):
        out.append(lines[i][6:].rstrip("\n"))
        i += 1
    return out, i


def _numbers(line):
    return [float(t) for t in re.findall(r"-?\d+\.?\d*(?:e[-+]?\d+)?", line)]


def parse_vignette(md_path: Path) -> dict:
    lines = md_path.read_text().splitlines()
    g = {}
    blk, _ = _block_after(lines, "head(mcmc_nngp_list$observed_locs)")
    g["observed_locs_head"] = [_numbers(l)[1:] for l in blk[1:]]
    blk, _ = _block_after(lines, "head(mcmc_nngp_list$X$X)")
    g["X_head"] = [_numbers(l)[1:] for l in blk[1:]]
    blk, _ = _block_after(lines, "head(mcmc_nngp_list$locs)")
    g["locs_head"] = [_numbers(l)[1:] for l in blk[1:]]
    blk, _ = _block_after(lines, "head(mcmc_nngp_list$vecchia_approx$NNarray)")
    nn = []
    for l in blk[1:]:
        toks = l.split()[1:]
        nn.append([None if t == "NA" else int(t) for t in toks])
    g["NNarray_head"] = nn
    blk, _ = _block_after(lines, "MRF_adjacency_mat[1:30, 1:30]")
    rows = []
    for l in blk:
        m = re.match(r"\s*\[\s*(\d+),\]\s+(.*)$", l)
        if m:
            rows.append([1 if t == "1" else 0 for t in m.group(2).split()])
    assert len(rows) == 30 and all(len(r) == 30 for r in rows)
    g["moral_block_30"] = rows
    blk, _ = _block_after(lines, "print(mcmc_nngp_list$vecchia_approx$locs_match[1:100])")
    lm = []
    for l in blk:
        lm += [int(t) for t in l.split("]", 1)[1].split()]
    g["locs_match_100"] = lm
    blk, _ = _block_after(lines, "print(mcmc_nngp_list$vecchia_approx$hctam_scol_1[1:100])")
    h = []
    for a, bline in zip(blk[0::2], blk[1::2]):
        h += [int(t) for t in bline.split()]
    g["hctam_scol_1_100"] = h
    blk, _ = _block_after(lines, "print(estimations$covariance_params$GpGp_covparams)")
    g["GpGp_covparams"] = {l.split()[0]: _numbers(l)[-5:] for l in blk[1:]}
    blk, _ = _block_after(lines, "print(estimations$fixed_effects)")
    fe = {}
    for l in blk[1:4]:
        fe[l.split()[0]] = _numbers(l)[-5:]
    g["fixed_effects"] = fe
    blk, _ = _block_after(lines, "head(estimations$field)")
    g["field_head"] = [_numbers(l)[1:] for l in blk[1:]]
    g["summary_columns"] = ["mean", "q0.025", "median", "q0.975", "sd"]
    g["_source"] = "Vignette.md (printed outputs of the reference's vignette)"
    return g


def main():
    ref = Path(sys.argv[1]) if len(sys.argv) > 1 else Path("/root/reference")
    g = parse_vignette(ref / "Vignette.md")
    (HERE / "vignette_printed.json").write_text(json.dumps(g, indent=1))
    from r_rng import vignette_toy
    v = vignette_toy()
    np.savez_compressed(HERE / "vignette_toy.npz", **v)
    print("wrote", HERE / "vignette_printed.json", HERE / "vignette_toy.npz")


if __name__ == "__main__":
    main()
