#!/usr/bin/env python3
"""Synchronous MPI_Reduce_local (fp32 SUM, device-resident) after an idle host
gap of G us between calls (the host spins, the GPU idles): call time and the
CP's dispatch latency (MPIR_Hip_direct_last_split) against G.  A schedule that
waits on the network between its combine steps sees the long-gap figures.
    python tools/idle_gap_probe.py [--count 1048576] [--calls 200]"""
import argparse
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
import ctypes
import torch
import mpich_pip_amd as m

ap = argparse.ArgumentParser()
ap.add_argument("--count", type=int, default=1 << 20)
ap.add_argument("--calls", type=int, default=200)
args = ap.parse_args()
lib = m.load()
fast = m.fast_reduce_local()
a = torch.rand(args.count, device="cuda")
b = torch.rand(args.count, device="cuda")
torch.cuda.synchronize()
ca = (b.data_ptr(), a.data_ptr(), args.count, m.MPI_FLOAT, m.MPI_SUM)
for _ in range(50):
    fast(*ca)
split = (ctypes.c_uint64 * 4)()
for gap_us in (0, 10, 20, 50, 100, 200, 500, 1000, 5000):
    walls, starts = [], []
    lib.MPIR_Hip_direct_profile(1)
    for _ in range(args.calls):
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e6 < gap_us:
            pass
        c0 = time.perf_counter()
        fast(*ca)
        walls.append((time.perf_counter() - c0) * 1e6)
        lib.MPIR_Hip_direct_last_split(split)
        starts.append((split[1] - split[0]) * 1e-3)
    lib.MPIR_Hip_direct_profile(0)
    walls.sort()
    starts.sort()
    n = len(walls)
    print(f"gap {gap_us:5d} us: call median {walls[n // 2]:7.2f} us (p10 {walls[n // 10]:7.2f}, p90 {walls[n * 9 // 10]:7.2f}); "
          f"doorbell -> CP start median {starts[n // 2]:6.2f} us", flush=True)
