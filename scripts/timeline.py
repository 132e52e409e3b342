"""Tile engine per-phase timeline (NNGP_PROBE=2 build path): thread 0 of every
tile stamps the 100 MHz clock at the start of each colour phase, after the
draw (granules published), after the hand-off poll and at the phase end.
Usage: timeline.py [n] [m] [chains] [n_sweeps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ["NNGP_PROBE"] = "2"
out = "/tmp/tile_timeline.bin"
os.environ["NNGP_DBG_OUT"] = out
import _pkgload  # noqa: E402
import bench  # noqa: E402

P = _pkgload.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 15
C = int(sys.argv[3]) if len(sys.argv) > 3 else 3
S = int(sys.argv[4]) if len(sys.argv) > 4 else 10
cp = [1.0, 0.05, 0.0]
wl = bench.make_workload(P, n, m, "matern15_isotropic", cp, seed=1000, device=0, chains=C)
ctx = bench.open_context(P, wl, "matern15_isotropic", cp, 0, C, seed=7)
info = ctx.info
K = info["n_colors"]
T = info["n_tiles"]
print({k: info[k] for k in ("sweep_engine", "n_tiles", "tile_rows_max", "n_ghost_cells", "n_colors")})
args = ([wl["beta0"]] * C, [wl["log_scale"]] * C, [wl["log_noise_variance"]] * C, [77 + k for k in range(C)])
for rep in range(4):
    t = time.perf_counter()
    ctx.sweep_chains(S, *args, [rep * S] * C)
    el = time.perf_counter() - t
nph = S * K
raw = np.fromfile(out, dtype=np.uint64)[: T * 512 * 16].reshape(T, 512, 16)[:, :nph]  # tiles.hip kTimelineSlots
spins = raw[..., 5].astype(np.float64)
d = raw[..., [0, 1, 2, 3, 4, 6]].astype(np.float64) / 100.0  # us
miss = d[..., 1] == 0              # (tile, colour) with no own batch: no publish stamp
d[..., 1][miss] = d[..., 0][miss]
d -= d[:, 0, 0].min()
start, pub, hand, end, landed, scat = d[..., 0], d[..., 1], d[..., 2], d[..., 3], d[..., 4], d[..., 5]
scat = np.where(raw[..., 6] == 0, pub, scat)
own = pub - start                  # own batches up to the draw barrier (publish)
rest = hand - pub                  # scatter + stream issue + hand-off poll
tail = end - hand                  # ghost adds + next batch prep
dur = end - start
print(f"C={C} last call {el*1e3:.3f} ms wall, launch span {end[:, -1].max():.1f} us, {end[:, -1].max()/nph:.2f} us/phase")
print("per tile per phase (mean / p90 / max over tiles, averaged over phases):")
for nm, a in (("own->publish", own), ("publish->scattered", scat - pub), ("scattered->prepped", landed - scat),
              ("prepped->handoff", hand - landed),
              ("handoff->end", tail), ("phase", dur)):
    print(f"  {nm:18s} mean {a.mean():6.2f}  p90 {np.percentile(a, 90, axis=0).mean():6.2f}  max {a.max(axis=0).mean():6.2f}")
xwd = raw[..., 7].astype(np.float64)
if (xwd > 0).any():  # exchange-wave tiles: the wave's polls done (stamp 7)
    xw = np.where(xwd > 0, xwd / 100.0 - raw[:, 0, 0].astype(np.float64).min() / 100.0, hand)
    print(f"  xw polls done - publish: mean {(xw - pub).mean():6.2f}  p90 {np.percentile(xw - pub, 90):6.2f}")
# slots 9..15 (wave-local tiles): each cell wave's last publish of the phase;
# with the neighbour lists appended to the dump: the latest publish of the
# tiles this tile reads granules from -> skew (own publish -> it) and transit
# (it -> the exchange wave has every granule)
allraw = np.fromfile(out, dtype=np.uint64)
tail_i = np.frombuffer(allraw[T * 512 * 16:].tobytes(), dtype=np.int32)
if tail_i.size > T * K + 1 and (xwd > 0).any() and (raw[..., 9] > 0).any():
    nb_ptr = tail_i[: T * K + 1]
    nb = tail_i[T * K + 1:]
    base = raw[:, 0, 0].astype(np.float64).min()
    wp = raw[..., 9:16].astype(np.float64)
    lastpub = np.where(wp > 0, wp / 100.0 - base / 100.0, -np.inf).max(axis=2)  # (T, nph)
    lastpub = np.where(np.isfinite(lastpub), lastpub, pub)
    xwt = np.where(xwd > 0, xwd / 100.0 - base / 100.0, hand)
    prod = np.full((T, nph), -np.inf)
    for t_ in range(T):
        for ph in range(nph):
            c = ph % K
            lo, hi = nb_ptr[t_ * K + c], nb_ptr[t_ * K + c + 1]
            if hi > lo:
                prod[t_, ph] = lastpub[nb[lo:hi], ph].max()
    ok = np.isfinite(prod) & (xwd > 0)
    print(f"  own first publish -> own last publish  mean {(lastpub - pub)[ok].mean():6.2f}")
    sk = (prod - lastpub)[ok]
    tr = (xwt - prod)[ok]
    print(f"  own last publish -> producers' last publish (skew) mean {sk.mean():6.2f}  p10 {np.percentile(sk, 10):6.2f} "
          f"p90 {np.percentile(sk, 90):6.2f}")
    print(f"  producers' last publish -> all granules in (transit) mean {tr.mean():6.2f}  p10 {np.percentile(tr, 10):6.2f} "
          f"p90 {np.percentile(tr, 90):6.2f}")
    print(f"  phase start -> producers' last publish mean {(prod - start)[ok].mean():6.2f};"
          f" neighbours per (tile, colour) mean {np.diff(nb_ptr).mean():.1f}")
print(f"  poll spins (max over the tile's threads): mean {spins.mean():.2f}, p90 {np.percentile(spins, 90):.0f}, "
      f"share of phases with spins {(spins > 0).mean():.2f}")
# critical path: per phase, the spread of publish times across tiles
spread = pub.max(axis=0) - pub.min(axis=0)
print(f"  publish spread across tiles per phase: mean {spread.mean():.2f} us")
# by colour (phases of the last sweeps)
byc = dur.reshape(T, S, K).mean(axis=(0, 1))
ownc = own.reshape(T, S, K).mean(axis=(0, 1))
ownmax = own.reshape(T, S, K).max(axis=0).mean(axis=0)
print("per colour: phase mean / own mean / own max over tiles")
print(" ".join(f"{c}:{byc[c]:.1f}/{ownc[c]:.1f}/{ownmax[c]:.1f}" for c in range(K)))
# per colour, every segment of the cell waves' chain (mean over tiles and sweeps)
segs = [("own", own), ("scatter", scat - pub), ("prep", landed - scat), ("wait", hand - landed), ("ghost", tail)]
print("per colour segments (us): " + " / ".join(n for n, _ in segs))
for c in range(K):
    print(f"  c{c:2d} " + " ".join(f"{a.reshape(T, S, K)[:, :, c].mean():5.2f}" for _, a in segs) +
          f"  = {byc[c]:5.2f}")
if os.environ.get("NNGP_TIMELINE_KEEP"):
    import shutil
    shutil.copy(out, os.environ["NNGP_TIMELINE_KEEP"])
ctx.close()
