"""Device idle gaps of a rocprofv3 trace (kernels + memory copies) and the
HIP API calls the host made inside them (diagnostic for the MCMC
iterations: scripts/mcmc_api.sh).  Window: from the 3rd sweep launch to the
last one.  Per gap kind (device op before -> device op after): total idle
time per iteration, the API time inside it by function, and the rest
(host code between API calls: Python, ctypes, the library's own host work).
Usage: api_gaps.py <rocprofv3 output dir> [last K sweep launches: the window
runs from the K-th last to the last one, default 10 = the 9 iterations inside
mcmc_prof.py's timed call]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]


def rows_of(pattern):
    fs = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


dev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows_of("*kernel_trace.csv")]
for r in rows_of("*memory_copy_trace.csv"):
    dev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", r.get("Operation", "?"))))
dev.sort()
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in rows_of("*hip_api_trace.csv"))
sw = [i for i, r in enumerate(dev) if "sweep_tiles_kernel" in r[2] or "sweep_color_kernel" in r[2]]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
a, b = sw[-K], sw[-1]
iters = b and len([i for i in sw if a <= i < b])
win = dev[a:b + 1]
t0, t1 = win[0][0], win[-1][0]
busy_end = win[0][1]
gaps = defaultdict(lambda: {"idle": 0, "n": 0, "api": defaultdict(int), "apin": defaultdict(int)})
prev = win[0]
for r in win[1:]:
    if r[0] > busy_end + 2000:  # idle > 2 us
        g = gaps[(prev[2], r[2])]
        g["idle"] += r[0] - busy_end
        g["n"] += 1
        for s, e, f in api:
            if e < busy_end or s > r[0]:
                continue
            g["api"][f] += min(e, r[0]) - max(s, busy_end)
            g["apin"][f] += 1
    busy_end = max(busy_end, r[1])
    prev = r
span = (t1 - t0) / 1e6 / iters
idle = sum(g["idle"] for g in gaps.values()) / 1e6 / iters
print(f"{iters} iterations, {span:.3f} ms/it, device idle {idle:.3f} ms/it")
for k, g in sorted(gaps.items(), key=lambda x: -x[1]["idle"])[:14]:
    at = sum(g["api"].values())
    print(f"{g['idle'] / 1e6 / iters:7.3f} ms/it {g['n'] / iters:5.1f}/it  {k[0]} -> {k[1]}   "
          f"(API {at / 1e6 / iters:.3f}, other host {(g['idle'] - at) / 1e6 / iters:.3f} ms/it)")
    for f, t in sorted(g["api"].items(), key=lambda x: -x[1])[:5]:
        print(f"        {t / 1e6 / iters:7.3f} ms/it {g['apin'][f] / iters:5.1f}/it  {f}")
tot = defaultdict(lambda: [0, 0])
for s, e, f in api:
    if t0 <= s <= t1:
        tot[f][0] += e - s
        tot[f][1] += 1
print("all HIP API time in the window:")
for f, (t, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:14]:
    print(f"  {t / 1e6 / iters:7.3f} ms/it {c / iters:6.1f}/it {t / c / 1e3:8.1f} us  {f}")
