#!/usr/bin/env python3
"""Why one resident 256 MiB pair runs slower than another (round 6; round 5
left it open): the bench's per-pair call medians differ by 1-4 us within one
process (`call_distribution.median_us_by_pair`), so the headline depends on
where the allocator put the pairs.  Here one process allocates P pairs
(inbuf, inoutbuf of 256 MiB fp32) with one method, fills them from two seeded
random tensors, and runs the headline call over them rotating (no call finds
its operands in the Infinity Cache), C loop with clock stamps; per pair: the
median call, and the median CP kernel time of profiled calls.

    python3 tools/archive/pair_alloc_ab.py METHOD [pairs = 12] [rounds = 40]
    python3 tools/archive/pair_alloc_ab.py --ab [reps = 3]     # alternates the methods in fresh processes
    SHIFT=1 python3 tools/archive/pair_alloc_ab.py contig       # + each pair with inbuf shifted by S bytes

METHOD: torch (the bench's: one caching-allocator tensor per operand, with the
bench's slack), malloc (hipMalloc per operand), contig (hipExtMallocWithFlags
hipDeviceMallocContiguous per operand), slab (one hipMalloc for all operands).
"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)

import mpich_pip_amd as m  # noqa: E402  (the library first: VRAM rings)

MIB = 1 << 20
NB = 256 * MIB
METHODS = ["torch", "malloc", "contig", "slab"]


def child(method, npairs, rounds):
    import numpy as np
    lib = m.load()
    import torch
    import bench
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    bind = bench.bind_near_gpu(m, 0)
    hip = bench.library_hip_runtime(lib)
    vp = ctypes.c_void_p
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [vp]
    count = NB // 4
    slack = 256 * 1024
    keep, ptrs = [], []

    def raw(nbytes, flags=None):
        p = vp()
        rc = hip.hipMalloc(ctypes.byref(p), nbytes) if flags is None else \
            hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags)
        assert rc == 0, f"allocation failed ({rc})"
        keep.append(p.value)
        return p.value
    if method == "torch":
        ts = [torch.empty(count + slack // 4, device="cuda") for _ in range(2 * npairs)]
        keep_t = ts
        addrs = [t.data_ptr() for t in ts]
    elif method == "malloc":
        addrs = [raw(NB + slack) for _ in range(2 * npairs)]
    elif method == "contig":
        addrs = [raw(NB + slack, 0x4) for _ in range(2 * npairs)]
    elif method == "slab":
        base = raw((NB + slack) * 2 * npairs)
        addrs = [base + i * (NB + slack) for i in range(2 * npairs)]
    else:
        raise SystemExit(f"unknown method {method}")
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    src = [torch.rand(count, device="cuda", generator=g) for _ in range(2)]
    torch.cuda.synchronize()
    for i, a in enumerate(addrs):
        assert hip.hipMemcpy(vp(a), vp(src[i % 2].data_ptr()), NB, 3) == 0
    del src
    torch.cuda.synchronize()
    pairs = [(addrs[2 * i + 1], addrs[2 * i]) for i in range(npairs)]     # (inbuf, inoutbuf)
    sets = tuple((pin, pio, count, m.MPI_FLOAT, m.MPI_SUM) for pin, pio in pairs)
    loop = m.fast_reduce_local_loop()
    k = npairs * rounds
    assert loop(sets, 0, 2 * npairs) == 0
    st = np.zeros(k + 1, np.int64)
    assert loop(sets, 0, k, st) == 0
    calls = np.diff(st) / 1e3
    per_pair = [float(np.median(calls[i::npairs])) for i in range(npairs)]
    # the CP's kernel time per pair (profiled twin queue)
    lib.MPIR_Hip_direct_profile(1)
    kern = [[] for _ in range(npairs)]
    try:
        for r in range(6):
            for i in range(npairs):
                assert loop(sets, i, 1) == 0
                kern[i].append(lib.MPIR_Hip_direct_last_kernel_ns() / 1e3)
    finally:
        lib.MPIR_Hip_direct_profile(0)
    kmed = [float(np.median(v)) for v in kern]
    # SHIFT=1: each pair again with inbuf moved by S bytes against inoutbuf
    # (count reduced to fit the slack): a pair slow for the two operands'
    # relative physical placement changes speed with S; one slow for its own
    # pages does not
    shifts = {}
    if os.environ.get("SHIFT") == "1":
        lib.MPIR_Hip_direct_profile(1)
        try:
            for sh in (0, 4096, 65536, 200704):        # (within the operands' 256 KiB slack)
                c2 = count - sh // 4
                row = []
                for i, (pin, pio) in enumerate(pairs):
                    ks = []
                    for r in range(5):
                        s2 = ((pin + sh, pio, c2, m.MPI_FLOAT, m.MPI_SUM),)
                        assert loop(s2, 0, 1) == 0
                        ks.append(lib.MPIR_Hip_direct_last_kernel_ns() / 1e3)
                        # another pair between repeats: no Infinity Cache reuse
                        assert loop(sets, (i + 1 + r) % npairs, 1) == 0
                    row.append(round(float(np.median(ks)), 2))
                shifts[str(sh)] = row
        finally:
            lib.MPIR_Hip_direct_profile(0)
    out = {"method": method, "pairs": npairs, "calls_per_pair": rounds, "bind": bind.get("mode"),
           "pair_call_median_us": [round(x, 2) for x in per_pair],
           "pair_kernel_median_us": [round(x, 2) for x in kmed],
           "all_calls_median_us": round(float(np.median(calls)), 2), "all_calls_mean_us": round(float(np.mean(calls)), 2),
           "spread_pair_medians_us": round(max(per_pair) - min(per_pair), 2),
           "addresses_MiB": [round(a / MIB) for a in addrs[:6]], "inbuf_shift_kernel_us": shifts}
    print(json.dumps(out), flush=True)
    for a in keep:
        hip.hipFree(vp(a))


def ab(reps):
    res = []
    for r in range(reps):
        order = METHODS[r % len(METHODS):] + METHODS[:r % len(METHODS)]
        for meth in order:
            t0 = time.time()
            p = subprocess.run([sys.executable, os.path.abspath(__file__), meth], capture_output=True, text=True,
                               timeout=240)
            lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not lines:
                print(json.dumps({"method": meth, "error": p.returncode, "stderr": p.stderr.strip().splitlines()[-3:]}),
                      flush=True)
                sys.exit(1)
            d = json.loads(lines[-1])
            d["round"], d["wall_s"] = r, round(time.time() - t0, 1)
            print(json.dumps(d), flush=True)
            res.append(d)
    print("\nmethod | all calls median / mean us (median over processes) | spread of pair medians us "
          "(per process) | pair kernel medians min-max us")
    for meth in METHODS:
        rs = [d for d in res if d["method"] == meth]
        med = sorted(d["all_calls_median_us"] for d in rs)
        mean = sorted(d["all_calls_mean_us"] for d in rs)
        spreads = [d["spread_pair_medians_us"] for d in rs]
        kmin = min(min(d["pair_kernel_median_us"]) for d in rs)
        kmax = max(max(d["pair_kernel_median_us"]) for d in rs)
        print(f"{meth:7s}| {med[len(med) // 2]:7.2f} / {mean[len(mean) // 2]:7.2f} | {spreads} | {kmin:.2f}-{kmax:.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--ab":
        ab(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
    else:
        child(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
