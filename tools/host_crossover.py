#!/usr/bin/env python3
"""Both operands in host memory, large counts: the host combine (threads of the
copy pool) against the GPU staging pipeline, fp32 SUM, per call (median).  The
path is switched in-process with MPIR_Hip_set_host_max_bytes: 0 sends every
both-host call through the staging pipeline, the default (no limit) keeps it on
the host.

    python3 tools/host_crossover.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    f = m.fast_reduce_local()
    F, S = m.MPI_FLOAT, m.MPI_SUM
    torch.cuda.init()
    default = lib.MPIR_Hip_set_host_max_bytes(0)
    lib.MPIR_Hip_set_host_max_bytes(default)
    print(f"default host limit: {default:#x}", flush=True)
    for mib in (1, 4, 16, 64, 256):
        n = mib << 18
        a = np.random.default_rng(1).uniform(-1, 1, n).astype(np.float32)
        b = np.random.default_rng(2).uniform(-1, 1, n).astype(np.float32)
        pa = torch.from_numpy(a.copy()).pin_memory()
        pb = torch.from_numpy(b.copy()).pin_memory()
        reps = max(3, min(50, 2000 // mib))
        for mode, limit in (("staged", 0), ("host", default)):
            lib.MPIR_Hip_set_host_max_bytes(limit)
            for name, pin, pio in (("pageable", b.ctypes.data, a.ctypes.data), ("pinned", pb.data_ptr(), pa.data_ptr())):
                assert f(pin, pio, n, F, S) == 0
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    assert f(pin, pio, n, F, S) == 0
                    ts.append(time.perf_counter() - t0)
                ts.sort()
                t = ts[len(ts) // 2]
                print(f"{mode:<7} {name:<9} {mib:>4} MiB  {t * 1e6:9.1f} us  {3 * n * 4 / t / 2**30:6.1f} GiB/s",
                      flush=True)
        lib.MPIR_Hip_set_host_max_bytes(default)


if __name__ == "__main__":
    main()
