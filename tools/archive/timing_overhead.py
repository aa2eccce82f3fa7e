#!/usr/bin/env python3
"""The bench's timed region around the K calls (VERDICT r5 Weak #2 follow-up):
what the bracketing costs besides the calls -- the Python -> C loop entry and
exit, and torch.cuda.synchronize() on an idle device -- and the raw profiled
split of a few calls, bound near the GPU and unbound.

    python3 tools/archive/timing_overhead.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import mpich_pip_amd as m
    lib = m.load()
    import torch
    import bench
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    out = {"bind": bench.bind_near_gpu(m, 0) if len(sys.argv) < 2 else {"mode": "none"}}
    count = 64 << 20
    g = torch.Generator(device="cuda").manual_seed(1)
    pairs = [(torch.rand(count, device="cuda", generator=g), torch.rand(count, device="cuda", generator=g))
             for _ in range(4)]
    torch.cuda.synchronize()
    sets = tuple((a.data_ptr(), b.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM) for a, b in pairs)
    loop = m.fast_reduce_local_loop()
    assert loop(sets, 0, 10) == 0
    # 1. idle torch.cuda.synchronize()
    v = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        v.append(time.perf_counter() - t0)
    v.sort()
    out["torch_sync_idle_us"] = {"median": round(v[100] * 1e6, 2), "p90": round(v[180] * 1e6, 2)}
    # 2. entry + exit of the C loop with k = 0, and the stamps' view of a k = 20 loop
    st = np.zeros(21, np.int64)
    v = []
    for _ in range(200):
        t0 = time.perf_counter()
        loop(sets, 0, 0, st)
        v.append(time.perf_counter() - t0)
    v.sort()
    out["c_loop_k0_us"] = {"median": round(v[100] * 1e6, 2), "p90": round(v[180] * 1e6, 2)}
    rows = []
    for _ in range(20):
        t0 = time.perf_counter()
        loop(sets, 0, 20, st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        inner = (int(st[-1]) - int(st[0])) * 1e-9
        rows.append(((t1 - t0 - inner) * 1e6, (t2 - t0 - inner) * 1e6))
    rows.sort()
    out["k20_outside_stamps_us"] = {"loop_only_median": round(rows[10][0], 2),
                                    "with_sync_median": round(sorted(r[1] for r in rows)[10], 2)}
    # 3. raw profiled splits
    sp = (ctypes.c_uint64 * 4)()
    lib.MPIR_Hip_direct_profile(1)
    raw = []
    try:
        for i in range(8):
            assert loop(sets, i, 1) == 0
            lib.MPIR_Hip_direct_last_split(sp)
            raw.append(list(sp) + [lib.MPIR_Hip_direct_last_kernel_ns()])
    finally:
        lib.MPIR_Hip_direct_profile(0)
    out["raw_splits_ns"] = raw
    out["placement"] = m.placement(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
