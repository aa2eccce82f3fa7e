#!/usr/bin/env python3
"""With the direct queue's timestamps off from creation
(MPIR_CVAR_REDUCE_LOCAL_DIRECT_TIMESTAMPS=0), how many synchronous calls after
MPIR_Hip_direct_profile(1) until the CP's dispatch times appear?  Prints the
kernel ns the library reads for the first 40 calls after each of 3 switch-ons."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
import torch
import mpich_pip_amd as m

lib = m.load()
fast = m.fast_reduce_local()
n = 1 << 22
a = torch.rand(n, device="cuda")
b = torch.rand(n, device="cuda")
torch.cuda.synchronize()
for _ in range(20):
    fast(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
for rep in range(3):
    lib.MPIR_Hip_direct_profile(1)
    ns = []
    for _ in range(40):
        fast(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
        ns.append(lib.MPIR_Hip_direct_last_kernel_ns())
    lib.MPIR_Hip_direct_profile(0)
    print(f"switch-on {rep}: " + " ".join(str(x // 1000) for x in ns), flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.01:
        fast(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
