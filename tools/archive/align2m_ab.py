#!/usr/bin/env python3
"""do operands on 2 MiB-aligned allocations change the
headline loop's slow-launch tail or its median?  Two placements, alternated in
fresh processes (python3 tools/align2m_ab.py runs them):
  bench    the bench's own allocation: torch tensors of 256 MiB + 256 KiB
           (the fresh-argument slack), wherever the caching allocator puts them;
  aligned  hipMalloc'd blocks of 258 MiB whose operand start is rounded up to a
           2 MiB boundary (the allocation itself is checked too).
Each child runs the synchronous fp32 SUM loop over 4 rotating pairs (4000
calls after 200 warm-up) and reports the operand addresses mod 2 MiB, the
median call, the mean, and the share of calls slower than median + 4 us.

    python3 tools/align2m_ab.py [rounds]
"""
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
MIB = 1 << 20


def child(mode):
    import mpich_pip_amd as m
    lib = m.load()
    import torch
    torch.cuda.set_device(0)
    n = 64 * MIB
    keep = []
    ptrs = []
    if mode == "bench":
        for _ in range(4):
            a = torch.rand(n + 65536, device="cuda") * 2 - 1
            b = torch.rand(n + 65536, device="cuda") * 2 - 1
            keep += [a, b]
            ptrs.append((b.data_ptr(), a.data_ptr()))
    else:
        hip = ctypes.CDLL("libamdhip64.so")
        for _ in range(4):
            pair = []
            for _ in range(2):
                p = ctypes.c_void_p()
                assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(258 * MIB)) == 0
                base = (p.value + 2 * MIB - 1) & ~(2 * MIB - 1)
                t = torch.rand(n, device="cuda") * 2 - 1
                assert hip.hipMemcpy(ctypes.c_void_p(base), ctypes.c_void_p(t.data_ptr()), ctypes.c_size_t(4 * n), 3) == 0
                pair.append(base)
            ptrs.append((pair[1], pair[0]))
    torch.cuda.synchronize()
    f = m.fast_reduce_local()
    for i in range(200):
        pb, pa = ptrs[i % 4]
        assert f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM) == 0
    ts = []
    for i in range(4000):
        pb, pa = ptrs[i % 4]
        t0 = time.perf_counter()
        f(pb, pa, n, m.MPI_FLOAT, m.MPI_SUM)
        ts.append((time.perf_counter() - t0) * 1e6)
    med = statistics.median(ts)
    print(json.dumps({"mode": mode, "mod_2MiB": sorted({p % (2 * MIB) for pr in ptrs for p in pr}),
                      "median_us": round(med, 2), "mean_us": round(statistics.mean(ts), 2),
                      "slow_share": round(sum(t > med + 4 for t in ts) / len(ts), 4),
                      "frac_mean": round(3 * 4 * n / (statistics.mean(ts) * 1e-6) / 8e12, 4)}), flush=True)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for r in range(rounds):
        for mode in (("bench", "aligned") if r % 2 == 0 else ("aligned", "bench")):
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode], capture_output=True,
                               text=True, timeout=200)
            lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not lines:
                print(f"{mode} failed: {p.stderr[-1500:]}", flush=True)
                sys.exit(1)
            print(f"round {r} {lines[-1]}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main()
