#!/usr/bin/env python3
"""Latency of a synchronous MPI_Reduce_local (fp32 MPI_SUM) by operand residency
and count, against the reference's CPU loop on the same host buffers.

    python3 tools/host_latency.py [--reps 200]

Residencies: pageable host -> pageable host, pinned -> pinned, host in -> device
inout, pinned in -> device inout, device in -> host inout, device -> device.  CPU loop: the oracle's restatement of opsum.c's loop
(gcc -O2), timed here as the reference point only (tools/, never the product).
Prints one line per (residency, count): median / p10 / p90 microseconds per call.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)


def stats(ts):
    ts = sorted(ts)
    n = len(ts)
    return ts[n // 2] * 1e6, ts[n // 10] * 1e6, ts[(9 * n) // 10] * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    args = ap.parse_args()
    import torch
    import mpich_pip_amd as m
    import oracle
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    f = m.fast_reduce_local()
    orc = oracle.load()
    F, S = m.MPI_FLOAT, m.MPI_SUM
    counts = [1, 16, 256, 1024, 4096, 16384, 65536, 262144, 1 << 20]
    print(f"{'residency':<22}{'count':>9}{'bytes':>10}{'median_us':>11}{'p10':>9}{'p90':>9}")
    for n in counts:
        a = np.random.default_rng(1).uniform(-1, 1, n).astype(np.float32)
        b = np.random.default_rng(2).uniform(-1, 1, n).astype(np.float32)
        pa = torch.from_numpy(a.copy()).pin_memory()
        pb = torch.from_numpy(b.copy()).pin_memory()
        da = torch.from_numpy(a.copy()).cuda()
        db = torch.from_numpy(b.copy()).cuda()
        torch.cuda.synchronize()
        cases = [
            ("pageable->pageable", b.ctypes.data, a.ctypes.data),
            ("pinned->pinned", pb.data_ptr(), pa.data_ptr()),
            ("host->device", b.ctypes.data, da.data_ptr()),
            ("pinned->device", pb.data_ptr(), da.data_ptr()),
            ("device->host", db.data_ptr(), a.ctypes.data),
            ("device->device", db.data_ptr(), da.data_ptr()),
        ]
        reps = args.reps if n <= (1 << 16) else max(20, args.reps // 10)
        for name, pin, pio in cases:
            for _ in range(5):
                assert f(pin, pio, n, F, S) == 0
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                rc = f(pin, pio, n, F, S)
                ts.append(time.perf_counter() - t0)
                assert rc == 0, m.error_string(rc)
            print(f"{name:<22}{n:>9}{4 * n:>10}{stats(ts)[0]:>11.2f}{stats(ts)[1]:>9.2f}{stats(ts)[2]:>9.2f}",
                  flush=True)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            orc.oracle_reduce_local_nocheck(ctypes.c_void_p(b.ctypes.data), ctypes.c_void_p(a.ctypes.data), n, F, S)
            ts.append(time.perf_counter() - t0)
        print(f"{'cpu loop (oracle)':<22}{n:>9}{4 * n:>10}{stats(ts)[0]:>11.2f}{stats(ts)[1]:>9.2f}{stats(ts)[2]:>9.2f}",
              flush=True)


if __name__ == "__main__":
    main()
