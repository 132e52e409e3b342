"""Summarise NNGP_PROBE=9 per-chunk timestamps (diagnostic)."""
import sys
import numpy as np

K = int(sys.argv[2])
raw = open(sys.argv[1], "rb").read()
ptr = np.frombuffer(raw[:4 * (K + 1)], np.int32)
st = np.frombuffer(raw[4 * (K + 1):], np.uint64).reshape(-1, 8).astype(np.float64)
names = ["RT1 (cells+slots)", "RT2 gathers+normals", "running sums", "owners", "scatter+drain"]
for c in (0, K // 2, K - 2):
    a, b = ptr[c], ptr[c + 1]
    s = st[a:b]
    d = np.diff(s[:, :6], axis=1)
    rt = s[:, 7]
    print(f"colour {c}: chunks {b - a}, wave start spread (realtime, us) {(rt.max() - rt.min()) / 100:.2f}")
    for k, nm in enumerate(names):
        print(f"   {nm:18s} median {np.median(d[:, k]):8.0f} cyc  p90 {np.percentile(d[:, k], 90):8.0f}")
    print(f"   total             median {np.median(s[:, 5] - s[:, 0]):8.0f} cyc")
