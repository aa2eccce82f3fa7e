#!/usr/bin/env python3
"""How the synchronous call treats device buffers from each HIP allocator
(round 6, after tools/archive/pair_alloc_ab.py found hipDeviceMallocContiguous pairs
~2 us slower per call than hipMalloc ones, kernels alike): per method, one
64 MiB fp32 pair; MPIR_Hip_pointer_kind of each operand, the share of 200
calls the direct path took, the call median, and the profiled split (entry ->
doorbell, doorbell -> CP start, kernel, CP end -> seen), medians, us.

    python3 tools/archive/alloc_kind_probe.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)

import mpich_pip_amd as m  # noqa: E402  (the library first: VRAM rings)

MIB = 1 << 20


def main():
    import numpy as np
    lib = m.load()
    import torch
    import bench
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    bench.bind_near_gpu(m, 0)
    hip = bench.library_hip_runtime(lib)
    vp = ctypes.c_void_p
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemset.argtypes = [vp, ctypes.c_int, ctypes.c_size_t]
    hip.hipFree.argtypes = [vp]
    nb = 64 * MIB
    count = nb // 4
    methods = {"hipMalloc": lambda p: hip.hipMalloc(p, nb),
               "contiguous (0x4)": lambda p: hip.hipExtMallocWithFlags(p, nb, 0x4),
               "fine-grained (0x1)": lambda p: hip.hipExtMallocWithFlags(p, nb, 0x1),
               "uncached (0x3)": lambda p: hip.hipExtMallocWithFlags(p, nb, 0x3)}
    loop = m.fast_reduce_local_loop()
    sp = (ctypes.c_uint64 * 4)()
    for name, alloc in methods.items():
        bufs = []
        for _ in range(2):
            p = vp()
            rc = alloc(ctypes.byref(p))
            if rc != 0:
                print(json.dumps({"method": name, "error": f"allocation failed ({rc})"}), flush=True)
                break
            assert hip.hipMemset(p, 0, nb) == 0
            bufs.append(p.value)
        if len(bufs) < 2:
            continue
        torch.cuda.synchronize()
        pin, pio = bufs
        kinds = [lib.MPIR_Hip_pointer_kind(vp(pin), nb), lib.MPIR_Hip_pointer_kind(vp(pio), nb)]
        sets = ((pin, pio, count, m.MPI_FLOAT, m.MPI_SUM),)
        assert loop(sets, 0, 20) == 0
        d0 = lib.MPIR_Hip_direct_dispatches()
        st = np.zeros(201, np.int64)
        assert loop(sets, 0, 200, st) == 0
        share = (lib.MPIR_Hip_direct_dispatches() - d0) / 200
        calls = np.diff(st) / 1e3
        lib.MPIR_Hip_direct_profile(1)
        rows = []
        try:
            for _ in range(100):
                assert loop(sets, 0, 1) == 0
                lib.MPIR_Hip_direct_last_split(sp)
                rows.append([v - (1 << 64) if v >= (1 << 63) else v for v in sp])
        finally:
            lib.MPIR_Hip_direct_profile(0)
        rows = [r for r in rows if 0 < r[0] < r[3] and 0 < r[2] - r[1] < r[3] - r[0]]

        def med(v):
            return round(float(np.median(v)) / 1e3, 3) if v else None
        print(json.dumps({"method": name, "pointer_kind": kinds, "direct_share": share,
                          "call_median_us": round(float(np.median(calls)), 2),
                          "split": {"host_to_doorbell_us": med([r[0] for r in rows]),
                                    "doorbell_to_start_us": med([r[1] - r[0] for r in rows]),
                                    "kernel_us": med([r[2] - r[1] for r in rows]),
                                    "end_to_seen_us": med([r[3] - r[2] for r in rows])}}), flush=True)
        for b in bufs:
            hip.hipFree(vp(b))


if __name__ == "__main__":
    main()
