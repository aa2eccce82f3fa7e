#!/usr/bin/env python3
"""Where a kernarg-cache miss spends its time: synchronous MPI_Reduce_local
(fp32 SUM) with the arguments of an earlier call (cache hit) against fresh
arguments on every call (BAR write + HDP flush + read-back before the
doorbell), at 4 B, 4 MiB and 256 MiB per operand.

Per mode: the median wall time of the call without profiling, and with
MPIR_Hip_direct_profile on (the timestamped twin queue) the median timeline
of MPIR_Hip_direct_last_split: doorbell rung, CP dispatch start, CP end,
completion seen -- all from entering the dispatch routine -- and the kernel's
CP interval.  (Correctness of fresh-argument calls: tests/test_parity_gpu.py
test_direct_dispatch_fresh_args_every_call.)

    python3 tools/fresh_args_split.py [--calls 400]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=400)
    args = ap.parse_args()
    import mpich_pip_amd as m
    lib = m.load()            # before the HSA runtime starts (the library's ring default)
    import torch
    f = m.fast_reduce_local()
    torch.cuda.set_device(0)
    npairs, noff = 4, 256
    split = (ctypes.c_uint64 * 4)()
    for n in (1, 1 << 20, 64 << 20):
        pairs = [(torch.zeros(n + noff * 64, device="cuda"), torch.ones(n + noff * 64, device="cuda"))
                 for _ in range(npairs)]
        torch.cuda.synchronize()
        hit = [(b.data_ptr(), a.data_ptr()) for a, b in pairs]
        fresh = [(b.data_ptr() + o, a.data_ptr() + o) for o in range(0, noff * 256, 256) for a, b in pairs]
        for mode, argsets in (("hit", hit), ("miss", fresh), ("hit", hit), ("miss", fresh)):
            for i in range(50):
                pb, pa = argsets[i % len(argsets)]
                assert f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM) == 0
            kw0 = lib.MPIR_Hip_direct_kernarg_writes()
            wall = []
            for i in range(args.calls):
                pb, pa = argsets[(50 + i) % len(argsets)]
                t0 = time.perf_counter()
                f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM)
                wall.append(time.perf_counter() - t0)
            writes = (lib.MPIR_Hip_direct_kernarg_writes() - kw0) / args.calls
            lib.MPIR_Hip_direct_profile(1)
            rows = []
            for i in range(args.calls):
                pb, pa = argsets[(50 + args.calls + i) % len(argsets)]
                f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM)
                lib.MPIR_Hip_direct_last_split(split)
                rows.append([split[k] * 1e-3 for k in range(4)] + [lib.MPIR_Hip_direct_last_kernel_ns() * 1e-3])
            lib.MPIR_Hip_direct_profile(0)
            med = lambda xs: sorted(xs)[len(xs) // 2]
            cols = [med([r[k] for r in rows]) for k in range(5)]
            print(f"n={n:9d} {mode:4s} wall {med(wall) * 1e6:8.2f} us  kernarg writes/call {writes:.2f} | profiled: "
                  f"doorbell {cols[0]:5.2f}  cp_start {cols[1]:6.2f}  cp_end {cols[2]:8.2f}  seen {cols[3]:8.2f}  "
                  f"kernel {cols[4]:8.2f} us", flush=True)
        torch.cuda.synchronize()
        del pairs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
