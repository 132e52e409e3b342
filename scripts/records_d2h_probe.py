"""D2H of a chain's records (40 x 1e6 doubles, 320 MB) into host memory:
pageable numpy (the current get_records), a pinned torch tensor, and a numpy
array registered in place (hipHostRegister); plus reserve/free costs."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import _pkgload

P = _pkgload.load()
n, rows = 1_000_000, 40
rng = np.random.default_rng(0)
locs = rng.uniform(size=(n, 2))
NN = P.find_ordered_nn(locs, 5)
col = P.naive_greedy_coloring(NN)
ctx = P.ChainContext(locs, NN, col, np.arange(1, n + 1, dtype=np.int32), rng.normal(size=n), device=0)
ctx.set_field(rng.normal(size=n))
hip = ctypes.CDLL("libamdhip64.so")


def tm(f, label):
    torch.cuda.synchronize(0)
    t = time.perf_counter()
    r = f()
    torch.cuda.synchronize(0)
    print(f"{label}: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
    return r


tm(lambda: ctx.records_reserve(rows), "records_reserve(40)")
for i in range(rows):
    ctx.record_field(i)
out = tm(lambda: ctx.get_records(0, rows), "get_records -> fresh np.zeros (pageable)")
buf = np.empty((rows, n))
buf[:] = 1.0
tm(lambda: P.lib.nngp_get_records(ctx._h, 0, rows, buf.reshape(-1)), "get_records -> touched numpy (pageable)")
pin = tm(lambda: torch.empty((rows, n), dtype=torch.float64, pin_memory=True), "torch pinned alloc 320 MB")
pn = pin.numpy()
tm(lambda: P.lib.nngp_get_records(ctx._h, 0, rows, pn.reshape(-1)), "get_records -> pinned")
buf2 = np.empty((rows, n))
r = tm(lambda: hip.hipHostRegister(ctypes.c_void_p(buf2.ctypes.data), ctypes.c_size_t(buf2.nbytes), 0),
       "hipHostRegister 320 MB (untouched numpy)")
print("register rc", r)
tm(lambda: P.lib.nngp_get_records(ctx._h, 0, rows, buf2.reshape(-1)), "get_records -> registered")
tm(lambda: hip.hipHostUnregister(ctypes.c_void_p(buf2.ctypes.data)), "hipHostUnregister")
tm(lambda: ctx.records_reserve(0), "records_reserve(0)")
ctx.close()
