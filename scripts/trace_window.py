"""Per-kernel device time inside the last `ms` milliseconds of a rocprofv3
kernel trace (diagnostic: the timed MCMC iterations of scripts/mcmc_prof.py)."""
import csv
import sys
from collections import defaultdict

path, ms = sys.argv[1], float(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
rows.sort()
t1 = rows[-1][1]
t0 = t1 - ms * 1e6
win = [r for r in rows if r[0] >= t0]
tot = defaultdict(lambda: [0, 0])
busy = 0
for s, e, k in win:
    tot[k][0] += e - s
    tot[k][1] += 1
    busy += e - s
span = (win[-1][1] - win[0][0]) / 1e6
print(f"window {span:.2f} ms, {len(win)} launches, busy {busy / 1e6:.2f} ms ({100 * busy / 1e6 / span:.0f}%)")
for k, (d, c) in sorted(tot.items(), key=lambda x: -x[1][0]):
    print(f"{d / 1e6 / iters:8.3f} ms/it {c / iters:7.1f} calls/it  {d / c / 1e3:8.1f} us  {k[:90]}")
