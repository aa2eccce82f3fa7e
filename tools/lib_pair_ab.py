#!/usr/bin/env python3
"""In-process, interleaved A/B of two builds of libmpir_hip.so on the
synchronous fp32 SUM call at 256 MiB (MPIR_Hip_reduce, sync, library stream):
both copies are loaded RTLD_LOCAL from their own paths (each keeps its own
HSA queue, kernarg slots and cache), and blocks of calls alternate between
them, so box-to-box and minute-to-minute clock drift hits both alike (the
alternating-process A/B, tools/sync_lib_ab.sh, is swamped by it on some
boxes).  Two loops per build: 4 rotating pairs (kernarg-cache hits) and pairs
shifted by multiples of 256 B (every call a miss).

    python3 tools/lib_pair_ab.py <dir A> <dir B> [--blocks 30] [--per 20]
"""
import argparse
import ctypes
import faulthandler
import os
import sys
import statistics
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--blocks", type=int, default=30)
    ap.add_argument("--per", type=int, default=20)
    ap.add_argument("--mib", type=int, default=256)
    args = ap.parse_args()
    faulthandler.dump_traceback_later(45, repeat=True, file=sys.stderr)
    libs = {}
    for d in (args.a, args.b):
        lib = ctypes.CDLL(os.path.join(os.path.abspath(d), "libmpir_hip.so"), mode=os.RTLD_LOCAL | os.RTLD_NOW)
        lib.MPIR_Hip_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        lib.MPIR_Hip_reduce.restype = ctypes.c_int
        lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
        libs[os.path.basename(os.path.abspath(d)) + ("" if d == args.a else " ")] = lib
        print("loaded", d, flush=True)
    import torch
    torch.cuda.set_device(0)
    n = args.mib << 18
    slack = 256 * 256 // 4
    pairs = [(torch.rand(n + slack, device="cuda"), torch.rand(n + slack, device="cuda")) for _ in range(4)]
    torch.cuda.synchronize()
    hit = [(b.data_ptr(), a.data_ptr()) for a, b in pairs]
    fresh = [(b.data_ptr() + o, a.data_ptr() + o) for o in range(0, 256 * 256, 256) for a, b in pairs]
    SUM, F32 = 3, 10
    for k, lib in libs.items():    # first call per build: its direct-path init
        rc = lib.MPIR_Hip_reduce(hit[0][0], hit[0][1], n, SUM, F32, None, 1)
        print("first call", k.strip(), "rc", rc, flush=True)
    res = {(k, loop): [] for k in libs for loop in ("hit", "fresh")}
    pos = {(k, loop): 0 for k in libs for loop in ("hit", "fresh")}
    d0 = {k: lib.MPIR_Hip_direct_dispatches() for k, lib in libs.items()}
    for blk in range(-2, args.blocks):
        for loop, sets in (("hit", hit), ("fresh", fresh)):
            order = list(libs.items()) if blk % 2 == 0 else list(libs.items())[::-1]
            for k, lib in order:
                f = lib.MPIR_Hip_reduce
                i0 = pos[(k, loop)]
                for i in range(3):     # settle: this build's queue, clocks
                    pb, pa = sets[(i0 + i) % len(sets)]
                    f(pb, pa, n, SUM, F32, None, 1)
                i0 += 3
                t0 = time.perf_counter()
                for i in range(args.per):
                    pb, pa = sets[(i0 + i) % len(sets)]
                    f(pb, pa, n, SUM, F32, None, 1)
                dt = (time.perf_counter() - t0) / args.per
                pos[(k, loop)] = i0 + args.per
                if blk >= 0:
                    res[(k, loop)].append(dt * 1e6)
        print(f"block {blk} done", flush=True)
    alg = 3 * n * 4
    for (k, loop), v in res.items():
        med = statistics.median(v)
        print(f"{k.strip():14s} {loop:5s} median {med:8.2f} us/call  p10 {sorted(v)[len(v) // 10]:8.2f}  "
              f"p90 {sorted(v)[len(v) * 9 // 10]:8.2f}  frac {alg / (med * 1e-6) / 8e12:.4f}", flush=True)
    for k, lib in libs.items():
        print(f"{k.strip():14s} direct dispatches {lib.MPIR_Hip_direct_dispatches() - d0[k]}", flush=True)


if __name__ == "__main__":
    main()
