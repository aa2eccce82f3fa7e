#!/usr/bin/env python3
"""Config 2 (fp32 SUM, 64 MiB per operand) A/B: kernel time (direct-dispatch
timestamps) and synchronous per-call time for operand layouts and sizes.

    MPIR_CVAR_REDUCE_LOCAL_KEEP_MB=<n> python3 tools/config2_ab.py [--k 200]

Layouts: "win16" = 16 windows of four 256 MiB pairs (bench.py config2),
"sep8" = 8 separate 64 MiB pairs.  Per layout: mean / median kernel us,
sync us per call (compiled binding, perf_counter over K), and fractions of
8.0 TB/s.  Also 32 and 128 MiB with separate pairs for the size trend.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
MIB = 1 << 20
PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=200)
    args = ap.parse_args()
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    f = m.fast_reduce_local()
    F, S = m.MPI_FLOAT, m.MPI_SUM
    g = torch.Generator(device="cuda").manual_seed(1)

    def measure(name, wins, count):
        alg = 3 * count * 4
        k = args.k
        for i in range(10):
            a, b = wins[i % len(wins)]
            assert f(b, a, count, F, S) == 0
        lib.MPIR_Hip_direct_profile(1)
        d0 = lib.MPIR_Hip_direct_dispatches()
        ns = []
        for i in range(k):
            a, b = wins[i % len(wins)]
            assert f(b, a, count, F, S) == 0
            ns.append(lib.MPIR_Hip_direct_last_kernel_ns())
        lib.MPIR_Hip_direct_profile(0)
        nd = lib.MPIR_Hip_direct_dispatches() - d0
        if nd != k or min(ns) == 0:
            print(f"{name}: {nd} of {k} calls direct, {sum(1 for x in ns if x == 0)} zero timestamps, "
                  f"state {lib.MPIR_Hip_direct_state(0)}, busy skips {lib.MPIR_Hip_direct_busy_skips()}", flush=True)
            return
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            a, b = wins[i % len(wins)]
            f(b, a, count, F, S)
        dt = (time.perf_counter() - t0) / k
        ns.sort()
        mean = sum(ns) / k * 1e-3
        print(f"{name:<10} {count * 4 // MIB:>4} MiB  kernel mean {mean:7.2f} med {ns[k // 2] * 1e-3:7.2f} "
              f"p10 {ns[k // 10] * 1e-3:7.2f} p90 {ns[9 * k // 10] * 1e-3:7.2f} us ({alg / (mean * 1e-6) / PEAK:.4f})  "
              f"sync {dt * 1e6:7.2f} us ({alg / dt / PEAK:.4f})  gap {dt * 1e6 - mean:5.2f} us", flush=True)

    print("keep MiB:", os.environ.get("MPIR_CVAR_REDUCE_LOCAL_KEEP_MB", "64 (default)"))
    count = 16 * MIB
    big = [(torch.rand(4 * count, device="cuda", generator=g), torch.rand(4 * count, device="cuda", generator=g))
           for _ in range(4)]
    if os.environ.get("C2_SYNC"):
        torch.cuda.synchronize()
    wins = [(a.data_ptr() + j * count * 4, b.data_ptr() + j * count * 4) for a, b in big for j in range(4)]
    measure("win16", wins, count)
    del big, wins
    torch.cuda.empty_cache()
    for mib in (32, 64, 128):
        c = mib * MIB // 4
        sep = [(torch.rand(c, device="cuda", generator=g), torch.rand(c, device="cuda", generator=g))
               for _ in range(8)]
        measure("sep8", [(a.data_ptr(), b.data_ptr()) for a, b in sep], c)
        del sep
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
