"""Busy time vs wall time of the last ancillary proposal in a kernel trace:
per-kernel durations and the gaps between consecutive tri kernels."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last batch: from the last row_stats-kernel group onwards
idx = [i for i, r in enumerate(rows) if "row_stats" in r["Kernel_Name"]]
first = idx[-3] if len(idx) >= 3 else 0
seq = rows[first:]
t0 = int(seq[0]["Start_Timestamp"])
busy = 0
gaps = []
prev_end = None
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    if prev_end is not None:
        gaps.append(s - prev_end)
    prev_end = e
    name = r["Kernel_Name"].split("(")[0]
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} us  grid={r.get('Grid_Size', '?'):>8}  {name[:60]}")
wall = prev_end - t0
print(f"kernels {len(seq)}  wall {wall / 1e3:.1f} us  busy {busy / 1e3:.1f} us  "
      f"gaps total {sum(gaps) / 1e3:.1f} us  mean gap {sum(gaps) / max(len(gaps), 1) / 1e3:.2f} us")
