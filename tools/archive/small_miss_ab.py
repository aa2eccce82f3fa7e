#!/usr/bin/env python3
"""Latency of small synchronous MPI_Reduce_local calls through the direct AQL
dispatch, kernarg-cache misses (every call's arguments new: the checked kernel,
whose grid a padded build widens to 8 workgroups) against hits (arguments
repeated: the unchecked kernel).  One library build per process; alternate two
builds with tools/small_miss_ab.sh.

    python3 tools/small_miss_ab.py <dir holding libmpich_reduce_local.so> [--calls 3000] [--rounds 3]

Shapes: fp32 SUM count 1 (1 workgroup), 4099 (2: tile + head/tail), 28672
(7 tiles), and 1000 floats with inbuf 4 B off inoutbuf (the element kernel).
Median us per call of each (shape, hit/miss) cell, per round.
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libdir")
    ap.add_argument("--calls", type=int, default=3000)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import mpich_pip_amd as m
    lib = m.load(os.path.join(os.path.abspath(args.libdir), "libmpich_reduce_local.so"))
    import ctypes
    lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
    import torch
    torch.cuda.set_device(0)
    f = lib.MPI_Reduce_local
    shapes = [("count 1", 1, 0), ("count 4099", 4099, 0), ("7 tiles", 7 * 4096, 0), ("elems +4 B", 1000, 4)]
    nfresh = 1024
    bufs = {}
    for name, n, off in shapes:
        a = torch.zeros(n + 16 + nfresh * 64, device="cuda")
        b = torch.zeros(n + 16 + nfresh * 64, device="cuda")
        bufs[name] = (a, b)
    torch.cuda.synchronize()
    tag = os.path.basename(os.path.abspath(args.libdir))
    for r in range(args.rounds):
        for name, n, off in shapes:
            a, b = bufs[name]
            for kind in ("hit", "miss"):
                # misses: 1024 argument sets 256 B apart (same alignment, same plan)
                if kind == "hit":
                    sets = [(b.data_ptr() + off, a.data_ptr())]
                else:
                    sets = [(b.data_ptr() + off + 256 * j, a.data_ptr() + 256 * j) for j in range(nfresh)]
                for i in range(100):
                    pb, pa = sets[i % len(sets)]
                    assert f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM) == 0
                d0 = lib.MPIR_Hip_direct_dispatches()
                ts = []
                for i in range(args.calls):
                    pb, pa = sets[(100 + i) % len(sets)]
                    t0 = time.perf_counter()
                    f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM)
                    ts.append(time.perf_counter() - t0)
                direct = lib.MPIR_Hip_direct_dispatches() - d0
                print(f"{tag:12s} round {r} {name:11s} {kind:4s} median {statistics.median(ts) * 1e6:7.2f} us "
                      f"(direct {direct}/{args.calls})", flush=True)


if __name__ == "__main__":
    main()
