"""Summarise rocprofv3 --pmc csv passes (diagnostic).

Per-dispatch means of every counter for kernels matching a pattern, plus the
FETCH_SIZE / WRITE_SIZE calibration on known-byte kernels (scripts/micro/
calib.hip: 512 MiB read as 8-, 4- and 2-byte lanes, 512 MiB written as 8-byte
lanes), as MI355X_MICROARCH.md's HBM section prescribes ("calibrate on a known
byte count in your own access pattern").  The corrected HBM traffic per launch
= FETCH_SIZE x (bytes / FETCH_SIZE of the 8-byte read kernel) + WRITE_SIZE x
(bytes / WRITE_SIZE of the 8-byte write kernel).
usage: pmc_summary.py <pmc dir> <kernel substring> [--json out] [--chains C]"""
import argparse
import csv
import glob
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("pattern")
ap.add_argument("--json")
ap.add_argument("--chains", type=int, default=3)
ap.add_argument("--sweeps-per-dispatch", type=float, default=None)
a = ap.parse_args()

KNOWN = 512 << 20


def means(dirs, pat):
    acc = defaultdict(list)
    for d in dirs:
        for f in glob.glob(f"{a.root}/{d}/run_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if pat in r["Kernel_Name"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


sweep, counts = means(["fetch", "write", "tcc", "ea"], a.pattern)
cal = {}
for kern in ("rd8", "rd4", "rd2", "wr8"):
    m, _ = means(["cal_fetch", "cal_write"], kern)
    cal[kern] = {k: v * 1024 / KNOWN for k, v in m.items() if k in ("FETCH_SIZE", "WRITE_SIZE")}
for k in sorted(sweep):
    print(f"{a.pattern} {k:22s} per dispatch {sweep[k]:14.1f}  ({counts[k]} dispatches)")
for k, v in cal.items():
    print(f"calibration {k}: counter bytes / true bytes = {v}")
f_read = 1.0 / cal["rd8"]["FETCH_SIZE"] if cal.get("rd8", {}).get("FETCH_SIZE") else None
f_write = 1.0 / cal["wr8"]["WRITE_SIZE"] if cal.get("wr8", {}).get("WRITE_SIZE") else None
traffic = None
if f_read and f_write and "FETCH_SIZE" in sweep and "WRITE_SIZE" in sweep:
    traffic = sweep["FETCH_SIZE"] * 1024 * f_read + sweep["WRITE_SIZE"] * 1024 * f_write
    print(f"corrected HBM traffic per launch: {traffic / 1e6:.2f} MB "
          f"(read x{f_read:.3f}, write x{f_write:.3f})")
if a.json:
    json.dump({"kernel": a.pattern, "chains": a.chains, "per_dispatch": sweep, "dispatches": counts,
               "calibration_counter_over_true": cal, "read_correction": f_read, "write_correction": f_write,
               "traffic_bytes_per_launch": traffic,
               "sweeps_per_dispatch": a.sweeps_per_dispatch,
               "workload": {"n": 1000000, "m": 15, "covfun": "matern15_isotropic", "chains": a.chains}},
              open(a.json, "w"), indent=1)
