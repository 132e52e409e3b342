"""Summarise a rocprofv3 rocpd database (kernel name, calls, total/avg us)."""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
print(f"{'kernel':70s} {'calls':>7s} {'total_us':>12s} {'avg_us':>10s} {'%':>6s}")
for name, calls, tot, avg, pct in rows:
    print(f"{name[:70]:70s} {calls:7d} {tot:12.1f} {avg:10.3f} {pct:6.2f}")
if len(sys.argv) > 2:
    pat = sys.argv[2]
    durs = [r[0] for r in c.execute("select duration from kernels where name like ?", (f"%{pat}%",))]
    import statistics
    if durs:
        durs = [d / 1000.0 for d in durs]
        print(f"{pat}: n={len(durs)} median={statistics.median(durs):.3f}us min={min(durs):.3f} max={max(durs):.3f}")
