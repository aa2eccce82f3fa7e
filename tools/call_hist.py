#!/usr/bin/env python3
"""Per-call wall time of bench.py's headline loop (synchronous fp32 SUM,
256 MiB, 4 rotating pairs, compiled binding), to tell a uniform slowdown of a
box from a few long host-side stalls: percentiles, the slowest calls and their
positions, and the loop's aggregate rate with and without them.
  python3 tools/call_hist.py [calls = 3000]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    import mpich_pip_amd as m
    lib = m.load()
    import numpy as np
    import torch
    count = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [((torch.rand(count, device="cuda", generator=g) * 2 - 1), (torch.rand(count, device="cuda", generator=g) * 2 - 1))
             for _ in range(4)]
    ptrs = [(a.data_ptr(), b.data_ptr()) for a, b in pairs]
    torch.cuda.synchronize()
    f = m.fast_reduce_local()
    for i in range(50):
        pin, pio = ptrs[i % 4]
        f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
    t = np.empty(calls, np.int64)
    clk = time.perf_counter_ns
    t0 = clk()
    for i in range(calls):
        pin, pio = ptrs[i % 4]
        a = clk()
        f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
        t[i] = clk() - a
    total = clk() - t0
    us = t / 1e3
    alg = 3 * count * 4
    q = np.percentile(us, [1, 10, 50, 90, 99, 99.9])
    print(f"calls {calls}: p1 {q[0]:.2f} p10 {q[1]:.2f} p50 {q[2]:.2f} p90 {q[3]:.2f} p99 {q[4]:.2f} p99.9 {q[5]:.2f} "
          f"max {us.max():.2f} us; mean {us.mean():.2f} us")
    slow = np.argsort(us)[::-1][:10]
    print("slowest:", ", ".join(f"#{k} {us[k]:.1f}" for k in sorted(slow)))
    for lim in (130.0, 150.0, 300.0, 1000.0):
        print(f"  calls > {lim:.0f} us: {(us > lim).sum()}  (their excess over the median: {np.clip(us - q[2], 0, None)[us > lim].sum():.0f} us)")
    print(f"loop rate {alg * calls / (total / 1e9) / 2**30:.1f} GiB/s = {alg * calls / (total / 1e9) / 8e12:.4f} of 8 TB/s; "
          f"without calls > 150 us {alg * (us <= 150).sum() / (us[us <= 150].sum() / 1e6) / 8e12:.4f}")
    # the bench's own shape: 20 / 100 consecutive calls, worst and best windows
    for w in (20, 100):
        s = np.convolve(us, np.ones(w), "valid")
        print(f"  windows of {w}: best {alg * w / (s.min() / 1e6) / 8e12:.4f}  median {alg * w / (np.median(s) / 1e6) / 8e12:.4f}  "
              f"worst {alg * w / (s.max() / 1e6) / 8e12:.4f} of 8 TB/s")


if __name__ == "__main__" and not os.environ.get("SPLIT_TAIL") and not os.environ.get("COLD"):
    main()


def split_tail(calls: int = 3000):
    """The same loop with the library's per-call profiling on (the timestamped
    twin queue: entry -> doorbell -> CP start -> CP end -> host sees, ns), to
    see which interval the slow calls lose their time in."""
    import ctypes
    import mpich_pip_amd as m
    lib = m.load()
    import numpy as np
    import torch
    count = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [((torch.rand(count, device="cuda", generator=g) * 2 - 1), (torch.rand(count, device="cuda", generator=g) * 2 - 1))
             for _ in range(4)]
    ptrs = [(a.data_ptr(), b.data_ptr()) for a, b in pairs]
    torch.cuda.synchronize()
    f = m.fast_reduce_local()
    lib.MPIR_Hip_direct_profile(1)
    split = (ctypes.c_uint64 * 4)()
    rows = np.empty((calls, 5))
    for i in range(50 + calls):
        pin, pio = ptrs[i % 4]
        a = time.perf_counter_ns()
        f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
        w = time.perf_counter_ns() - a
        lib.MPIR_Hip_direct_last_split(split)
        if i >= 50:
            rows[i - 50] = (w / 1e3, split[0] / 1e3, split[1] / 1e3, (split[2] - split[1]) / 1e3, (split[3] - split[2]) / 1e3)
    lib.MPIR_Hip_direct_profile(0)
    names = ("wall", "entry->doorbell", "entry->CP start", "kernel (CP)", "CP end->host sees")
    med = np.median(rows, axis=0)
    slow = rows[rows[:, 0] > np.percentile(rows[:, 0], 90)]
    print(f"profiled calls {calls}: median / mean of the slowest 10 % / max, us")
    for k, nm in enumerate(names):
        print(f"  {nm:18s} {med[k]:8.2f} {slow[:, k].mean():8.2f} {rows[:, k].max():8.2f}")
    # are the slow kernels clustered (a clock / power state) or scattered?
    kern = rows[:, 3]
    thr = med[3] + 4.0
    slow_i = np.nonzero(kern > thr)[0]
    runs, cur = [], 0
    for a, b in zip(slow_i, slow_i[1:]):
        cur += 1
        if b != a + 1:
            runs.append(cur)
            cur = 0
    if len(slow_i):
        runs.append(cur + 1)
    gaps = np.diff(slow_i)
    print(f"kernels > median + 4 us: {len(slow_i)} of {calls}; runs of consecutive slow calls: "
          f"{np.bincount(runs)[1:].tolist() if runs else []} (count of runs of length 1, 2, ...); "
          f"gap between slow calls: median {np.median(gaps) if len(gaps) else 0:.0f}, "
          f"histogram {np.histogram(gaps, bins=[1, 2, 3, 5, 9, 17, 33, 65, 10**6])[0].tolist() if len(gaps) else []}")
    print("first 200 kernel times (us):", " ".join(f"{x:.0f}" for x in kern[:200]))


if __name__ == "__main__" and os.environ.get("SPLIT_TAIL"):
    split_tail(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)


def cold_start(calls: int = 400):
    """From process start: per-call wall time of the first calls (no warm-up
    beyond allocating and filling the pairs, as bench.py does), to see whether
    the driver's shape (5 warm-up calls, 20 timed) catches a ramp."""
    import mpich_pip_amd as m
    lib = m.load()
    import numpy as np
    import torch
    count = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [((torch.rand(count, device="cuda", generator=g) * 2 - 1), (torch.rand(count, device="cuda", generator=g) * 2 - 1))
             for _ in range(4)]
    ptrs = [(a.data_ptr(), b.data_ptr()) for a, b in pairs]
    torch.cuda.synchronize()
    f = m.fast_reduce_local()
    us = np.empty(calls)
    for i in range(calls):
        pin, pio = ptrs[i % 4]
        a = time.perf_counter_ns()
        f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
        us[i] = (time.perf_counter_ns() - a) / 1e3
    alg = 3 * count * 4
    for lo, hi in ((0, 5), (5, 25), (25, 45), (45, 100), (100, 200), (200, calls)):
        print(f"  calls {lo:4d}-{hi:4d}: mean {us[lo:hi].mean():7.2f} us = {alg / (us[lo:hi].mean() * 1e-6) / 8e12:.4f} of 8 TB/s")


if __name__ == "__main__" and os.environ.get("COLD"):
    cold_start()
