#!/usr/bin/env python3
"""The driver's bench shape (W = 5 warm-up calls, K = 20 timed calls) call by call.

Runs bench.py's headline loop on 4 rotating 256 MiB fp32 pairs and prints, for
each repetition, the value bench.py would report, every timed call's wall time
(perf_counter around the binding), the CP kernel time of the same calls
(direct-dispatch timestamps), and the cost of the closing
torch.cuda.synchronize().  Repetition 0 is what a fresh bench process sees.

    HSA_ALLOCATE_QUEUE_DEV_MEM=1 python tools/k20_probe.py [--reps 6] [--pre-ms 0]
"""
import argparse
import os
import sys
import time

os.environ.setdefault("HSA_ALLOCATE_QUEUE_DEV_MEM", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--pre-ms", type=float, default=0.0, help="GPU work (pair fills) before the first warm-up call")
ap.add_argument("--mib", type=int, default=256, help="MiB per operand; below 256 the pairs are cut into windows")
args = ap.parse_args()

import torch
import mpich_pip_amd as m

lib = m.load()
fast = m.fast_reduce_local()
torch.cuda.set_device(0)
count = 64 << 20
g = torch.Generator(device="cuda").manual_seed(1)
pairs = [((torch.rand(count, device="cuda", generator=g) * 2 - 1),
          (torch.rand(count, device="cuda", generator=g) * 2 - 1)) for _ in range(4)]
torch.cuda.synchronize()
if args.pre_ms > 0:
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.pre_ms:
        for a, b in pairs:
            a.mul_(1.0)
    torch.cuda.synchronize()
wcount = args.mib << 18
nwin = count // wcount
call_args = [(b.data_ptr() + j * wcount * 4, a.data_ptr() + j * wcount * 4, wcount, m.MPI_FLOAT, m.MPI_SUM)
             for a, b in pairs for j in range(nwin)]
alg = 3 * wcount * 4

# idle synchronize cost
ts = []
for _ in range(50):
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e6)
ts.sort()
print(f"idle torch.cuda.synchronize: median {ts[25]:.2f} us, max {ts[-1]:.2f} us", flush=True)

for rep in range(args.reps):
    lib.MPIR_Hip_direct_profile(1)
    for i in range(args.warmup):
        fast(*call_args[i % len(call_args)])
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    wall, kern = [], []
    t0 = time.perf_counter()
    for i in range(args.steps):
        c0 = time.perf_counter()
        fast(*call_args[(args.warmup + i) % len(call_args)])
        wall.append((time.perf_counter() - c0) * 1e6)
        kern.append(lib.MPIR_Hip_direct_last_kernel_ns() * 1e-3)
    s0 = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    lib.MPIR_Hip_direct_profile(0)
    dt = t1 - t0
    print(f"rep {rep}: value {alg * args.steps / dt / 2**30:.1f} GiB/s  ms/step {dt / args.steps * 1e3:.4f}  "
          f"closing sync {(t1 - s0) * 1e6:.1f} us  mean call {sum(wall) / len(wall):.2f} us  "
          f"mean kernel {sum(kern) / len(kern):.2f} us", flush=True)
    print("   calls  " + " ".join(f"{x:.1f}" for x in wall), flush=True)
    print("   kernel " + " ".join(f"{x:.1f}" for x in kern), flush=True)
