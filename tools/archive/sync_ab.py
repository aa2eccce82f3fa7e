#!/usr/bin/env python3
"""Synchronous MPI_Reduce_local cost under one runtime configuration (set by
the environment of this process): per-call time of K fp32 SUM calls at 256 MiB
over 4 rotating pairs (bench.py's step), the direct path's kernel time (CP
timestamps) and the gap between them, and the count-1 device call latency.

    [ENV=...] python3 tools/sync_ab.py --tag NAME [--k 200]

tools/sync_ab.sh runs it under several configurations, interleaved.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="default")
    ap.add_argument("--k", type=int, default=200)
    ap.add_argument("--pairs", type=int, default=4)
    args = ap.parse_args()
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    f = m.fast_reduce_local()
    F, S = m.MPI_FLOAT, m.MPI_SUM
    n = 64 * MIB
    g = torch.Generator(device="cuda").manual_seed(7)
    NP = args.pairs
    pairs = [(torch.rand(n, device="cuda", generator=g), torch.rand(n, device="cuda", generator=g)) for _ in range(NP)]
    small = (torch.rand(4, device="cuda"), torch.rand(4, device="cuda"))
    torch.cuda.synchronize()
    ptrs = [(b.data_ptr(), a.data_ptr()) for a, b in pairs]
    for i in range(10):
        assert f(*ptrs[i % NP], n, F, S) == 0
    d0 = lib.MPIR_Hip_direct_dispatches()
    t0 = time.perf_counter()
    for i in range(args.k):
        f(*ptrs[i % NP], n, F, S)
    dt = (time.perf_counter() - t0) / args.k
    direct = lib.MPIR_Hip_direct_dispatches() - d0
    import ctypes
    lib.MPIR_Hip_direct_profile(1)
    ns = []
    split = (ctypes.c_uint64 * 4)()
    sums = [0.0] * 5
    for i in range(args.k):
        t = time.perf_counter()
        f(*ptrs[i % NP], n, F, S)
        wall = (time.perf_counter() - t) * 1e9
        ns.append(lib.MPIR_Hip_direct_last_kernel_ns())
        lib.MPIR_Hip_direct_last_split(split)
        sp4 = list(split)
        for j, v in enumerate(sp4):
            sums[j] += v
        sums[4] += wall
    lib.MPIR_Hip_direct_profile(0)
    sp = [x / args.k * 1e-3 for x in sums]
    kern = sum(ns) / len(ns) * 1e-3 if min(ns) > 0 else float("nan")
    spp = (small[1].data_ptr(), small[0].data_ptr())
    for _ in range(20):
        f(*spp, 4, F, S)
    lat = []
    for _ in range(500):
        t = time.perf_counter()
        f(*spp, 4, F, S)
        lat.append(time.perf_counter() - t)
    lat.sort()
    lib.MPIR_Hip_direct_profile(1)
    ssum = [0.0] * 4
    for _ in range(200):
        f(*spp, 4, F, S)
        lib.MPIR_Hip_direct_last_split(split)
        for j, v in enumerate(list(split)):
            ssum[j] += v
    lib.MPIR_Hip_direct_profile(0)
    ssp = [x / 200 * 1e-3 for x in ssum]
    alg = 3 * n * 4
    print(f"{args.tag:<28} pairs {NP:2d} call {dt * 1e6:7.2f} us ({alg / dt / 2**30:7.1f} GiB/s, {alg / dt / 8e12:.4f})  "
          f"kernel {kern:7.2f} us  gap {dt * 1e6 - kern:5.2f} us  direct {direct}/{args.k}  "
          f"count-1 median {lat[250] * 1e6:5.2f} us p10 {lat[50] * 1e6:5.2f}", flush=True)
    print(f"{'':<28} split (us from entering the dispatch): doorbell {sp[0]:5.2f}  CP start {sp[1]:6.2f}  "
          f"CP end {sp[2]:7.2f}  host sees completion {sp[3]:7.2f}  whole call (python) {sp[4]:7.2f}", flush=True)
    print(f"{'':<28} count-4 split: doorbell {ssp[0]:5.2f}  CP start {ssp[1]:6.2f}  CP end {ssp[2]:6.2f}  "
          f"host sees completion {ssp[3]:6.2f}", flush=True)


if __name__ == "__main__":
    main()
