#!/usr/bin/env python3
"""A/B of two builds of the library on the synchronous fp32 SUM call at 256 MiB:
the bench's headline loop (4 rotating pairs: kernarg-cache hits) and its
fresh-argument loop (pairs shifted by multiples of 256 B: every call a miss),
through ctypes (same Python overhead for both builds).  Run it in alternating
processes, one build per process (tools/sync_lib_ab.sh):

    python3 tools/sync_lib_ab.py <dir holding libmpich_reduce_local.so> [--steps 200] [--rounds 3]
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
    ap.add_argument("libdir")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import mpich_pip_amd as m
    lib = m.load(os.path.join(os.path.abspath(args.libdir), "libmpich_reduce_local.so"))
    import torch
    torch.cuda.set_device(0)
    n = 64 << 20
    slack = 256 * 256 // 4
    pairs = [(torch.rand(n + slack, device="cuda"), torch.rand(n + slack, device="cuda")) for _ in range(4)]
    torch.cuda.synchronize()
    f = lib.MPI_Reduce_local
    hit = [(b.data_ptr(), a.data_ptr()) for a, b in pairs]
    fresh = [(b.data_ptr() + o, a.data_ptr() + o) for o in range(0, 256 * 256, 256) for a, b in pairs]
    for r in range(args.rounds):
        for name, sets in (("hit", hit), ("fresh", fresh)):
            for i in range(50):
                pb, pa = sets[i % len(sets)]
                assert f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM) == 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                pb, pa = sets[(50 + i) % len(sets)]
                f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            print(f"{os.path.basename(os.path.abspath(args.libdir)):12s} round {r} {name:5s} {dt * 1e6:8.2f} us/call  "
                  f"{3 * n * 4 / dt / 8e12:.4f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
