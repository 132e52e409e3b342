"""Per-kernel device time and host gaps per MCMC iteration, between the
sweep launches of a rocprofv3 kernel trace (diagnostic): iteration = from
one sweep_tiles launch to the next, the first `skip` and last of them
dropped (warm-up and the end-of-call record copies)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(path)))
sw = [i for i, r in enumerate(rows) if "sweep_tiles_kernel" in r[2] or "sweep_color_kernel" in r[2]]
a, b = sw[skip], sw[-1]
win = rows[a:b]
iters = len([i for i in sw if a <= i < b])
span = rows[b][0] - rows[a][0]
tot = defaultdict(lambda: [0, 0])
busy = 0
gaps = defaultdict(lambda: [0, 0])
for r in win:
    tot[r[2]][0] += r[1] - r[0]
    tot[r[2]][1] += 1
    busy += r[1] - r[0]
for p, q in zip(win, win[1:]):
    g = q[0] - p[1]
    if g > 0:
        k = (p[2][:36], q[2][:36])
        gaps[k][0] += g
        gaps[k][1] += 1
print(f"{iters} iterations, {span / 1e6 / iters:.3f} ms/it, busy {busy / 1e6 / iters:.3f} ms/it")
for k, (d, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:16]:
    print(f"{d / 1e6 / iters:8.3f} ms/it {c / iters:6.1f}/it {d / c / 1e3:8.1f} us  {k[:80]}")
print("gaps:")
for k, (d, c) in sorted(gaps.items(), key=lambda x: -x[1][0])[:12]:
    print(f"{d / 1e6 / iters:8.3f} ms/it {c / iters:6.1f}/it {d / c / 1e3:8.1f} us  {k[0]} -> {k[1]}")
