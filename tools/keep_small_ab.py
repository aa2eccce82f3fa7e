#!/usr/bin/env python3
"""The result store policy at small sizes (round 6): a result of at most
MPIR_CVAR_REDUCE_LOCAL_KEEP_MB is stored sc1 (into the Infinity Cache) so its
next reader finds it there; tools/aql/product_split measured that policy
costing a 16 KiB call ~0.45 us (the kernel's end, 6.60 against 6.10 us).  Per
size, in one process, the two policies alternate (MPIR_Hip_set_keep_bytes
64 MiB / 0) over rounds, in two patterns of synchronous calls:
  chain   the result is the next call's inoutbuf (a schedule's next step):
          out += in_k, k rotating over 16 inbufs
  spread  16 distinct (in, out) pairs rotated: nothing re-read soon
C loop, clock stamps; medians per (size, pattern, policy) over rounds, us.

    python3 tools/keep_small_ab.py [rounds = 9] [sizes in KiB, comma-separated]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)

import mpich_pip_amd as m  # noqa: E402  (the library first: VRAM rings)

KIB = 1 << 10


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    import numpy as np
    lib = m.load()
    import torch
    import bench
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    lib.MPIR_Hip_set_keep_bytes.argtypes = [ctypes.c_uint64]
    lib.MPIR_Hip_set_keep_bytes.restype = ctypes.c_uint64
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    bench.bind_near_gpu(m, 0)
    loop = m.fast_reduce_local_loop()
    default_keep = lib.MPIR_Hip_set_keep_bytes(64 << 20)
    # the sc1 side of the A/B stores every size sc1 (the lower bound the library
    # now applies, MPIR_CVAR_REDUCE_LOCAL_KEEP_MIN_MB, is what this measures)
    default_keep_min = lib.MPIR_Hip_set_keep_min_bytes(0) if hasattr(lib, "MPIR_Hip_set_keep_min_bytes") else None
    sizes = [int(x) * KIB for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [16 * KIB, 256 * KIB, 1024 * KIB, 4096 * KIB, 16384 * KIB]
    res = {}
    for nb in sizes:
        count = nb // 4
        ins = [torch.rand(count, device="cuda") * 1e-3 for _ in range(16)]
        outs = [torch.rand(count, device="cuda") for _ in range(16)]
        torch.cuda.synchronize()
        chain = tuple((ins[k].data_ptr(), outs[0].data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM) for k in range(16))
        spread = tuple((ins[k].data_ptr(), outs[k].data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM) for k in range(16))
        n = 2000 if nb <= 1024 * KIB else 500 if nb <= 16384 * KIB else 120
        for r in range(rounds):
            for pol in ((64 << 20, 0) if r % 2 == 0 else (0, 64 << 20)):
                lib.MPIR_Hip_set_keep_bytes(pol)
                for name, sets in (("chain", chain), ("spread", spread)):
                    assert loop(sets, 0, 64) == 0
                    st = np.zeros(n + 1, np.int64)
                    assert loop(sets, 0, n, st) == 0
                    res.setdefault((nb, name, pol), []).append(float(np.median(np.diff(st))) / 1e3)
        del ins, outs
        torch.cuda.empty_cache()
    lib.MPIR_Hip_set_keep_bytes(default_keep)
    if default_keep_min is not None:
        lib.MPIR_Hip_set_keep_min_bytes(default_keep_min)
    print("size KiB | pattern | sc1 (keep) median us | nt median us | nt - sc1")
    rows = []
    for nb in sizes:
        for name in ("chain", "spread"):
            k = sorted(res[(nb, name, 64 << 20)])[rounds // 2]
            t = sorted(res[(nb, name, 0)])[rounds // 2]
            rows.append({"KiB": nb // KIB, "pattern": name, "sc1_us": round(k, 3), "nt_us": round(t, 3)})
            print(f"{nb // KIB:8d} | {name:7s} | {k:8.3f} | {t:8.3f} | {t - k:+.3f}")
    print(json.dumps({"rows": rows, "rounds": rounds}))


if __name__ == "__main__":
    main()
