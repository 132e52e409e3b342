"""Summarise the request-size-resolved PMC passes of scripts/pmc_sizes.sh
(diagnostic).  rocprofv3's FETCH_SIZE = 64 B x TCC_EA0_RDREQ on gfx950: wide
streaming reads travel as 128-B requests (FETCH_SIZE reads half their bytes,
MI355X_MICROARCH.md), the sweep's 16-B hand-off polls as 64-B ones -- one
correction factor cannot serve both.  Here the bytes come from the requests
by size: reads 128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B, writes
64 x WRREQ_64B + 32 x the rest; checked on the known-byte calibration
kernels (scripts/micro/calib.hip: 512 MiB read as 8-, 4-, 2-byte lanes,
written as 8-byte lanes).
usage: pmc_sizes_summary.py <dir> <kernel substring> [--json out] [--chains C] [--sweeps-per-dispatch S]"""
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


def rd_bytes(m):
    return 128 * m.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0) + \
        32 * m.get("TCC_EA0_RDREQ_32B_sum", 0)


def wr_bytes(m):
    w64 = m.get("TCC_EA0_WRREQ_64B_sum", 0)
    return 64 * w64 + 32 * (m.get("TCC_EA0_WRREQ_sum", 0) - w64)


sweep, counts = means(["sw_r", "sw_w", "sw_f", "sw_wr"], a.pattern)
cal = {}
for kern in ("rd8", "rd4", "rd2", "wr8"):
    m, _ = means(["cal_r", "cal_w"], kern)
    cal[kern] = {"read_bytes_over_true": rd_bytes(m) / KNOWN, "write_bytes_over_true": wr_bytes(m) / KNOWN,
                 "counters": m}
for k in sorted(sweep):
    print(f"{a.pattern} {k:26s} per dispatch {sweep[k]:16.1f}  ({counts[k]} dispatches)")
for k, v in cal.items():
    print(f"calibration {k}: read bytes / true {v['read_bytes_over_true']:.4f}, write bytes / true "
          f"{v['write_bytes_over_true']:.4f}")
rd, wr = rd_bytes(sweep), wr_bytes(sweep)
req = sweep.get("TCC_EA0_RDREQ_sum", 0)
mix = {s: sweep.get(f"TCC_EA0_RDREQ_{s}_sum", 0) / req if req else None for s in ("128B", "64B", "32B")}
print(f"sweep read bytes {rd / 1e9:.3f} GB, write bytes {wr / 1e9:.3f} GB per dispatch; read request mix {mix}")
if "FETCH_SIZE" in sweep:
    print(f"  (FETCH_SIZE x 1024 = {sweep['FETCH_SIZE'] * 1024 / 1e9:.3f} GB; x2 streaming correction "
          f"{sweep['FETCH_SIZE'] * 2048 / 1e9:.3f} GB)")
if a.json:
    json.dump({"kernel": a.pattern, "chains": a.chains, "per_dispatch": sweep, "dispatches": counts,
               "calibration": cal, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
               "traffic_bytes_per_launch": rd + wr, "read_request_mix": mix,
               "method": "bytes from TCC_EA0_RDREQ_{128B,64B,32B} and TCC_EA0_WRREQ{,_64B} (scripts/pmc_sizes.sh)",
               "sweeps_per_dispatch": a.sweeps_per_dispatch,
               "workload": {"n": 1000000, "m": 15, "covfun": "matern15_isotropic", "chains": a.chains}},
              open(a.json, "w"), indent=1)
