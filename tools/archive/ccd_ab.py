#!/usr/bin/env python3
"""Which core complex the synchronous call's thread runs on (round 6, after
tools/placement_ab.py): the EPYC sockets hold 8 CCDs each (one L3 per CCD), all
wired to the socket's I/O die, whose PCIe root ports sit in its quadrants; the
doorbell write, the completion signal and the error word travel between the
calling core and the GPU's port.  In ONE process (same queue, signal, buffers),
the calling thread is moved from L3 domain to L3 domain within the CPUs the job
may use, rotating the order each round; per domain and round: the median of
3,000 4 KiB calls and of 300 headline calls (256 MiB fp32 SUM, 4 rotating pairs),
C loop, clock stamps per call.  Prints one JSON line per (round, domain), then
per domain the median over rounds, its NUMA node and whether the GPU is there.

    python3 tools/archive/ccd_ab.py [rounds = 20]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))

import mpich_pip_amd as m  # noqa: E402  (the library first: VRAM rings)

MIB = 1 << 20


def cpulist(txt):
    out = set()
    for part in txt.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def l3_domains(allowed):
    doms = {}
    for c in sorted(allowed):
        try:
            txt = open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read()
        except OSError:
            continue
        key = min(cpulist(txt))
        doms.setdefault(key, set()).add(c)
    return doms


def cpu_node(c):
    for e in os.listdir(f"/sys/devices/system/cpu/cpu{c}"):
        if e.startswith("node") and e[4:].isdigit():
            return int(e[4:])
    return -1


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import numpy as np
    lib = m.load()
    import torch
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    gnode = m.placement(0)["gpu_node"]
    allowed = os.sched_getaffinity(0)
    doms = l3_domains(allowed)
    keys = sorted(doms)
    print(json.dumps({"gpu_node": gnode, "domains": {k: [min(doms[k]), max(doms[k]), len(doms[k])] for k in keys},
                      "HSA_ALLOCATE_QUEUE_DEV_MEM": os.environ.get("HSA_ALLOCATE_QUEUE_DEV_MEM")}), flush=True)
    count = 256 * MIB // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [(torch.rand(count, device="cuda", generator=g), torch.rand(count, device="cuda", generator=g))
             for _ in range(4)]
    small = torch.rand(1024, device="cuda"), torch.rand(1024, device="cuda")
    torch.cuda.synchronize()
    big = tuple((a.data_ptr(), b.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM) for a, b in pairs)
    sset = ((small[0].data_ptr(), small[1].data_ptr(), 1024, m.MPI_FLOAT, m.MPI_SUM),)
    loop = m.fast_reduce_local_loop()
    res = {k: {"small": [], "big": []} for k in keys}
    for r in range(rounds):
        order = keys[r % len(keys):] + keys[:r % len(keys)]
        for k in order:
            os.sched_setaffinity(0, doms[k])
            st = np.zeros(3001, np.int64)
            assert loop(sset, 0, 100) == 0
            assert loop(sset, 0, 3000, st) == 0
            s_med = float(np.median(np.diff(st))) / 1e3
            st = np.zeros(301, np.int64)
            assert loop(big, 0, 8) == 0
            assert loop(big, 0, 300, st) == 0
            b = np.diff(st) / 1e3
            b_med, b_mean = float(np.median(b)), float(np.mean(b))
            res[k]["small"].append(s_med)
            res[k]["big"].append((b_med, b_mean))
            print(json.dumps({"round": r, "domain": k, "cpus": [min(doms[k]), max(doms[k])], "node": cpu_node(k),
                              "small_median_us": round(s_med, 3), "big_median_us": round(b_med, 2),
                              "big_mean_us": round(b_mean, 2)}), flush=True)
    print("\nL3 domain (cpus)    node  GPU's | 4 KiB call median (median over rounds, min-max) | "
          "256 MiB call median / mean")
    for k in keys:
        sm = sorted(res[k]["small"])
        bm = sorted(x[0] for x in res[k]["big"])
        bn = sorted(x[1] for x in res[k]["big"])
        node = cpu_node(k)
        print(f"{k:4d} ({min(doms[k]):3d}-{max(doms[k]):3d}, {len(doms[k]):2d})  {node:4d}  {'yes' if node == gnode else 'no ':5s} | "
              f"{sm[len(sm) // 2]:6.3f} ({sm[0]:.3f}-{sm[-1]:.3f}) | {bm[len(bm) // 2]:7.2f} / {bn[len(bn) // 2]:7.2f}")


if __name__ == "__main__":
    main()
