#!/usr/bin/env python3
"""Does a kernel in flight on another stream keep the command processor out of
its deep idle?  Before each host gap a one-wave spin kernel
(torch.cuda._sleep) long enough to outlast the gap is launched on a side
stream; the synchronous call after the gap is timed (keep-alive thread off)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
os.environ.setdefault("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US", "0")
import torch
import mpich_pip_amd as m

fast = m.fast_reduce_local()
n = 1 << 20
a = torch.rand(n, device="cuda")
b = torch.rand(n, device="cuda")
torch.cuda.synchronize()
ca = (b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
side = torch.cuda.Stream()
for _ in range(50):
    fast(*ca)
# calibrate _sleep cycles per us
t0 = time.perf_counter()
with torch.cuda.stream(side):
    torch.cuda._sleep(10_000_000)
side.synchronize()
cyc_per_us = 10_000_000 / ((time.perf_counter() - t0) * 1e6)
print(f"_sleep: {cyc_per_us:.0f} cycles per us", flush=True)
for sleeper in (False, True):
    for gap_us in (0, 50, 100, 500, 2000):
        w = []
        for _ in range(100):
            if sleeper:
                with torch.cuda.stream(side):
                    torch.cuda._sleep(int(cyc_per_us * (gap_us + 60)))
            t0 = time.perf_counter()
            while (time.perf_counter() - t0) * 1e6 < gap_us:
                pass
            c0 = time.perf_counter()
            fast(*ca)
            w.append((time.perf_counter() - c0) * 1e6)
            side.synchronize()
        w.sort()
        print(f"sleeper {int(sleeper)} gap {gap_us:5d} us: call median {w[50]:6.2f} us (p10 {w[10]:6.2f}, p90 {w[90]:6.2f})",
              flush=True)
