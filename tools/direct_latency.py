#!/usr/bin/env python3
"""Synchronous device-resident MPI_Reduce_local latency (median of 2000 calls,
compiled binding) for shapes the direct AQL dispatch took from the HIP launch
path when it gained every kernel of plan_reduce: ragged counts, equal and
unequal misalignment, the logical / bitwise / MAXLOC ops.  Run twice to compare:

    python3 tools/direct_latency.py                                      # direct
    MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip python3 tools/direct_latency.py  # HIP launch
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
os.environ.setdefault("HSA_ALLOCATE_QUEUE_DEV_MEM", "1")


def main():
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    f = m.fast_reduce_local()
    mode = os.environ.get("MPIR_CVAR_REDUCE_LOCAL_DISPATCH", "direct")
    # (name, datatype, op, count, element bytes, inbuf offset, inoutbuf offset)
    cases = [("fp32 SUM", m.MPI_FLOAT, m.MPI_SUM, 4, 4, 0, 0), ("fp32 SUM", m.MPI_FLOAT, m.MPI_SUM, 1, 4, 0, 0),
             ("fp32 SUM", m.MPI_FLOAT, m.MPI_SUM, 4099, 4, 0, 0),
             ("fp32 SUM +4/+4", m.MPI_FLOAT, m.MPI_SUM, 4096, 4, 4, 4),
             ("fp32 SUM +4/0", m.MPI_FLOAT, m.MPI_SUM, 4099, 4, 4, 0),
             ("fp32 SUM +4/0", m.MPI_FLOAT, m.MPI_SUM, 1 << 20, 4, 4, 0),
             ("fp32 SUM", m.MPI_FLOAT, m.MPI_SUM, (1 << 20) + 7, 4, 0, 0),
             ("int BXOR", m.MPI_INT, m.MPI_BXOR, 4096, 4, 0, 0), ("int LAND", m.MPI_INT, m.MPI_LAND, 4096, 4, 0, 0),
             ("2INT MAXLOC", m.MPI_2INT, m.MPI_MAXLOC, 4096, 8, 0, 0)]
    torch.cuda.init()
    for name, dt, op, n, esz, oi, oo in cases:
        a = torch.zeros(n * esz + 64, dtype=torch.uint8, device="cuda")
        b = torch.zeros(n * esz + 64, dtype=torch.uint8, device="cuda")
        pa, pb = a.data_ptr() + oo, b.data_ptr() + oi
        torch.cuda.synchronize()
        for _ in range(200):
            assert f(pb, pa, n, dt, op) == 0
        d0 = lib.MPIR_Hip_direct_dispatches()
        ts = []
        for _ in range(2000):
            t0 = time.perf_counter()
            f(pb, pa, n, dt, op)
            ts.append(time.perf_counter() - t0)
        went = lib.MPIR_Hip_direct_dispatches() - d0
        ts.sort()
        print(f"{mode:6s} {name:14s} n={n:8d}  median {ts[len(ts) // 2] * 1e6:6.2f} us  p90 "
              f"{ts[len(ts) * 9 // 10] * 1e6:6.2f} us  direct {went}/2000", flush=True)


if __name__ == "__main__":
    main()
