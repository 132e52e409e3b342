"""Per-dispatch averages of PMC counters for one kernel from rocprofv3 csv runs
(diagnostic).  usage: pmc_summary.py <pmc dir> <kernel substring>"""
import csv
import glob
import sys
from collections import defaultdict

root, pat = sys.argv[1], sys.argv[2]
acc = defaultdict(list)
for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    # counters are reported per dimension instance; sum per dispatch = total / dispatches
    print(f"{k:28s} rows {len(v):6d} mean {sum(v) / len(v):14.1f}")
