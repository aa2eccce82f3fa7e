#!/usr/bin/env python3
"""Near / far placement of the synchronous call's host thread.

The synchronous MPI_Reduce_local's host-memory traffic is the doorbell write
(MMIO into the GPU's BAR), the completion signal the CP writes and the caller
polls, and one read of the error word (AQL ring and kernargs sit in VRAM).  This
A/B runs the headline loop (4 rotating 256 MiB fp32 pairs, MPI_SUM, C loop) in
alternated fresh processes whose calling thread is bound to the CPUs of the
GPU's NUMA node ("near"), to the other node's ("far"), or left as launched
("none"), within the CPUs the job may use, and reports per process:
  * the call distribution of K back-to-back calls (median / mean / p90 / slow
    share) and of the first 20 after 5 warm-up calls (the driver's window);
  * the split of K profiled calls (MPIR_Hip_direct_last_split, medians): entry
    -> doorbell, doorbell -> CP dispatch start, kernel, CP end -> host seen;
  * where everything sat: the thread's CPU / node, the GPU's node, the nodes of
    the completion signal and the error word (MPIR_Hip_direct_placement).

    python3 tools/placement_ab.py [rounds] [k] [modes]   # parent: alternates the modes
modes: near | far | none, each optionally with suffixes ":lazy" ":delay" ":flush"
(the waiting knobs) and ":sigg" / ":sigo" (the completion signal of unprofiled
calls allocated on the GPU's node / on another node, MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE).
Output: one JSON line per process, then a summary table (medians over rounds).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)

MIB = 1 << 20
NPAIRS = 4
HBM = 8.0e12


def node_cpus(node: int) -> set:
    out = set()
    try:
        txt = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return out
    for part in txt.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


def nodes():
    try:
        return sorted(int(e[4:]) for e in os.listdir("/sys/devices/system/node") if e.startswith("node") and e[4:].isdigit())
    except OSError:
        return [0]


def stats(calls_ns):
    v = sorted(calls_ns)
    n = len(v)
    med = v[n // 2]
    slow = [x for x in v if x > med + 4000]
    return {"median_us": round(med / 1e3, 2), "mean_us": round(sum(v) / n / 1e3, 2),
            "p90_us": round(v[(9 * n) // 10] / 1e3, 2), "max_us": round(v[-1] / 1e3, 2),
            "slow_share": round(len(slow) / n, 4)}


# mode suffixes: the waiting knobs of direct_dispatch.hip (poll_cfg)
WAITS = {"": {}, "lazy": {"MPIR_CVAR_REDUCE_LOCAL_POLL_DELAY_US": "110", "MPIR_CVAR_REDUCE_LOCAL_POLL_FLUSH": "1"},
         "delay": {"MPIR_CVAR_REDUCE_LOCAL_POLL_DELAY_US": "110"}, "flush": {"MPIR_CVAR_REDUCE_LOCAL_POLL_FLUSH": "1"}}


def child(mode: str, k: int) -> None:
    import numpy as np
    import mpich_pip_amd as m
    lib = m.load()
    import torch
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    gnode = m.placement(0)["gpu_node"]
    where = mode.split(":")[0]
    sig = [x for x in mode.split(":")[1:] if x.startswith("sig")]
    if sig and gnode >= 0:
        # completion signal in the fine-grained pool of the GPU's node (sigg) or
        # of another node (sigo): MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE, read at the
        # first direct call, which is below
        others = [n for n in nodes() if n != gnode]
        node = gnode if sig[0] == "sigg" else (others[0] if others else gnode)
        os.environ["MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE"] = str(node)
    allowed = os.sched_getaffinity(0)
    want = None
    if where == "near" and gnode >= 0:
        want = node_cpus(gnode) & allowed
    elif where == "far" and gnode >= 0:
        others = [n for n in nodes() if n != gnode]
        want = set().union(*(node_cpus(n) for n in others)) & allowed if others else set()
    if want is not None:
        if not want:
            print(json.dumps({"mode": mode, "skipped": "no allowed CPU there", "gpu_node": gnode}), flush=True)
            return
        os.sched_setaffinity(0, want)      # this (the calling) thread only
    count = 256 * MIB // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [(torch.rand(count, device="cuda", generator=g), torch.rand(count, device="cuda", generator=g))
             for _ in range(NPAIRS)]
    torch.cuda.synchronize()
    sets = tuple((a.data_ptr(), b.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM) for a, b in pairs)
    loop = m.fast_reduce_local_loop()
    # the driver's window first: 5 warm-up calls, 20 timed
    st = np.zeros(21, np.int64)
    assert loop(sets, 0, 5) == 0
    assert loop(sets, 5, 20, st) == 0
    window = stats(np.diff(st).tolist())
    # then K back to back
    st = np.zeros(k + 1, np.int64)
    assert loop(sets, 25, k, st) == 0
    long = stats(np.diff(st).tolist())
    place = m.placement(0)      # (the signal node is that of the knob's signal when it is set)
    # the split of profiled calls (timestamped twin queue)
    import ctypes
    sp = (ctypes.c_uint64 * 4)()
    # the profiled calls below use the runtime's signals; the knob's signal
    # covers the unprofiled loops (window20, loop, small loop)
    lib.MPIR_Hip_direct_profile(1)
    rows = []
    try:
        for i in range(min(k, 400)):
            assert loop(sets, i, 1) == 0
            lib.MPIR_Hip_direct_last_split(sp)
            rows.append(tuple(v - (1 << 64) if v >= (1 << 63) else v for v in sp))
    finally:
        lib.MPIR_Hip_direct_profile(0)
    rows = [r for r in rows if 0 < r[0] < r[3] and 0 < r[2] - r[1] < r[3] - r[0]]

    def med(v):
        v = sorted(v)
        return round(v[len(v) // 2] / 1e3, 3)
    split = {"host_to_doorbell_us": med([r[0] for r in rows]),
             "doorbell_to_start_us": med([r[1] - r[0] for r in rows]),
             "kernel_us": med([r[2] - r[1] for r in rows]),
             "end_to_seen_us": med([r[3] - r[2] for r in rows])} if rows else None
    # a 4 KiB call (one workgroup): what of the kernel interval is fixed cost
    small = torch.rand(1024, device="cuda"), torch.rand(1024, device="cuda")
    torch.cuda.synchronize()
    sset = ((small[0].data_ptr(), small[1].data_ptr(), 1024, m.MPI_FLOAT, m.MPI_SUM),)
    st = np.zeros(2001, np.int64)
    assert loop(sset, 0, 50) == 0
    assert loop(sset, 0, 2000, st) == 0
    small_loop = stats(np.diff(st).tolist())
    lib.MPIR_Hip_direct_profile(1)
    srows = []
    try:
        for i in range(400):
            assert loop(sset, 0, 1) == 0
            lib.MPIR_Hip_direct_last_split(sp)
            srows.append(tuple(v - (1 << 64) if v >= (1 << 63) else v for v in sp))
    finally:
        lib.MPIR_Hip_direct_profile(0)
    srows = [r for r in srows if 0 < r[0] < r[3] and 0 < r[2] - r[1] < r[3] - r[0]]
    small_split = {"host_to_doorbell_us": med([r[0] for r in srows]),
                   "doorbell_to_start_us": med([r[1] - r[0] for r in srows]),
                   "kernel_us": med([r[2] - r[1] for r in srows]),
                   "end_to_seen_us": med([r[3] - r[2] for r in srows])} if srows else None
    print(json.dumps({"mode": mode, "bound_cpus": len(want) if want is not None else len(allowed),
                      "placement": place, "window20": window, "loop": long,
                      "frac_at_median": round(3 * 256 * MIB / (long["median_us"] * 1e-6) / HBM, 4),
                      "frac_window20_mean": round(3 * 256 * MIB / (window["mean_us"] * 1e-6) / HBM, 4),
                      "split": split, "small_4KiB": {"loop": small_loop, "split": small_split},
                      "env": {k: v for k, v in os.environ.items() if k.startswith(("MPIR_CVAR_REDUCE_LOCAL_POLL",
                                                                                   "MPIR_CVAR_REDUCE_LOCAL_SIGNAL"))},
                      "direct_state": lib.MPIR_Hip_direct_state(0)}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(sys.argv[2], int(sys.argv[3]))
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        # python3 tools/placement_ab.py --summarize LOG: the table again from a log's JSON lines
        res = [json.loads(ln) for ln in open(sys.argv[2]) if ln.startswith("{")]
        modes = list(dict.fromkeys(d["mode"] for d in res))
        return summarize(res, modes)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["near", "far", "none"]
    res = []
    for r in range(rounds):
        order = modes[r % len(modes):] + modes[:r % len(modes)]
        for mode in order:
            t0 = time.time()
            env = dict(os.environ)
            for suffix in mode.split(":")[1:]:
                env.update(WAITS.get(suffix, {}))
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode, str(k)],
                               capture_output=True, text=True, timeout=240, env=env)
            lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not lines:
                print(json.dumps({"mode": mode, "error": p.returncode, "stderr": p.stderr.strip().splitlines()[-3:]}),
                      flush=True)
                sys.exit(1)
            d = json.loads(lines[-1])
            d["round"] = r
            d["wall_s"] = round(time.time() - t0, 1)
            print(json.dumps(d), flush=True)
            res.append(d)
    summarize(res, modes)


def summarize(res, modes):
    print("\nmode        | loop median / mean us | window20 mean us | host->db | db->start | kernel | end->seen "
          "| 4 KiB call median: db->start, kernel, end->seen | cpu node / gpu / signal / errword")
    for mode in modes:
        rs = [d for d in res if d.get("mode") == mode and "loop" in d]
        if not rs:
            print(f"{mode:11s} | skipped")
            continue

        def mm(f, among=None):
            v = sorted(f(d) for d in (among if among is not None else rs))
            return v[len(v) // 2]
        sp = [d for d in rs if d.get("split")]
        pl = rs[0]["placement"]
        ss = [d for d in rs if (d.get("small_4KiB") or {}).get("split")]
        print(f"{mode:11s} | {mm(lambda d: d['loop']['median_us']):7.2f} / {mm(lambda d: d['loop']['mean_us']):7.2f} | "
              f"{mm(lambda d: d['window20']['mean_us']):7.2f} | "
              + (" | ".join(f"{mm(lambda d, key=key: d['split'][key]):6.3f}" for key in
                            ("host_to_doorbell_us", "doorbell_to_start_us", "kernel_us", "end_to_seen_us"))
                 if sp else "-") +
              (f" | {mm(lambda d: d['small_4KiB']['loop']['median_us'], ss):6.2f}: " if ss else " | ")
              + (", ".join(f"{mm(lambda d, key=key: d['small_4KiB']['split'][key], ss):5.2f}" for key in
                           ("doorbell_to_start_us", "kernel_us", "end_to_seen_us")) if ss else "-") +
              f" | {pl['cpu_node']} / {pl['gpu_node']} / {pl['signal_node']} / {pl['error_word_node']}")


if __name__ == "__main__":
    main()
