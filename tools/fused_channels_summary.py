#!/usr/bin/env python3
"""Summarise tools/fused_channels.sh's rocprofv3 passes: per kernel, the median
over its dispatches (the first two rounds dropped) of every counter, the
per-channel and per-XCD request spread (max / mean, coefficient of variation),
EA read / write requests against the algorithmic bytes, DRAM credit stalls and
average in-flight levels per request (Little's law: LEVEL / REQ = mean cycles
a request is outstanding), and the kernel duration as a fraction of 8 TB/s.

    python3 tools/fused_channels_summary.py gpurun_out/fused_channels
"""
import csv
import glob
import os
import statistics
import sys

MIB32 = 32 << 20
ALG = {"fused_nt": 9 * MIB32, "fused_sc1": 9 * MIB32, "ro8": 8 * MIB32, "tile2": 3 * MIB32,
       "pipe2": 9 * MIB32, "pipe4": 9 * MIB32}
ORDER = ["fused_nt", "fused_sc1", "ro8", "tile2", "pipe2", "pipe4"]


def variant(name):
    if "k_combine_multi" in name:
        return "fused"
    if "k_ro8" in name:
        return "ro8"
    if "k_tile2" in name:
        return "tile2"
    if "k_pipe_s<2>" in name:
        return "pipe2"
    if "k_pipe_s<4>" in name:
        return "pipe4"
    return None


def load(d):
    """{variant: {counter: [values by dispatch order]}} and {variant: [durations us]}"""
    vals, durs = {}, {}
    for pdir in sorted(glob.glob(os.path.join(d, "*"))):
        if not os.path.isdir(pdir):
            continue
        for path in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
            per = {}
            for r in csv.DictReader(open(path)):
                v = variant(r["Kernel_Name"])
                if v:
                    per.setdefault((v, r["Counter_Name"]), []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
            for (v, c), rows in per.items():
                rows.sort()
                xs = [x for _, x in rows]
                if v == "fused":      # launches alternate fused_nt, fused_sc1
                    vals.setdefault("fused_nt", {})[c] = xs[0::2][2:]
                    vals.setdefault("fused_sc1", {})[c] = xs[1::2][2:]
                else:
                    vals.setdefault(v, {})[c] = xs[2:]
        for path in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
            per = {}
            for r in csv.DictReader(open(path)):
                v = variant(r["Kernel_Name"])
                if v:
                    per.setdefault(v, []).append((int(r["Dispatch_Id"]),
                                                  (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
            for v, rows in per.items():
                rows.sort()
                xs = [x for _, x in rows]
                if v == "fused":
                    durs.setdefault("fused_nt", []).extend(xs[0::2][2:])
                    durs.setdefault("fused_sc1", []).extend(xs[1::2][2:])
                else:
                    durs.setdefault(v, []).extend(xs[2:])
    return vals, durs


def med(xs):
    return statistics.median(xs) if xs else float("nan")


def spread(xs):
    m = statistics.mean(xs)
    return max(xs) / m, min(xs) / m, statistics.pstdev(xs) / m


def main():
    d = sys.argv[1]
    vals, durs = load(d)
    ks = [k for k in ORDER if k in vals]
    print("fused combine channel counters: TREE8 fp32 8 x 32 MiB (fused_*), its 8 loads alone (ro8), "
          "the two-operand tile over 32 MiB (tile2); medians over dispatches")
    print(f"{'':34s}" + "".join(f"{k:>14s}" for k in ks))

    def row(label, f, fmt="{:14.3f}"):
        out = []
        for k in ks:
            try:
                out.append(fmt.format(f(k)))
            except (KeyError, ZeroDivisionError, statistics.StatisticsError, ValueError):
                out.append(f"{'-':>14s}")
        print(f"{label:34s}" + "".join(out))

    c = lambda k, n: med(vals[k][n])
    row("kernel us (pmc passes)", lambda k: med(durs[k]), "{:14.2f}")
    row("frac of 8 TB/s", lambda k: ALG[k] / (med(durs[k]) * 1e-6) / 8e12)
    # gfx950 EA read requests are 128 B here (no 32 B ones, 64 B not counted separately)
    row("EA read reqs x 128 B / alg read", lambda k: 128 * c(k, "TCC_EA0_RDREQ_sum") /
        (ALG[k] - (0 if k == "ro8" else MIB32)))
    row("EA write reqs (64 B) / alg write", lambda k: 64 * c(k, "TCC_EA0_WRREQ_64B_sum") / MIB32)
    row("read reqs 32 B share", lambda k: c(k, "TCC_EA0_RDREQ_32B_sum") / c(k, "TCC_EA0_RDREQ_sum"))
    row("RD DRAM credit stall / RD req", lambda k: c(k, "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum") / c(k, "TCC_EA0_RDREQ_sum"))
    row("WR DRAM credit stall / WR req", lambda k: c(k, "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum") / c(k, "TCC_EA0_WRREQ_sum"))
    row("WR EA stall / WR req", lambda k: c(k, "TCC_EA0_WRREQ_STALL_sum") / c(k, "TCC_EA0_WRREQ_sum"))
    row("RD level / RD req (cycles)", lambda k: c(k, "TCC_EA0_RDREQ_LEVEL_sum") / c(k, "TCC_EA0_RDREQ_sum"), "{:14.1f}")
    row("WR level / WR req (cycles)", lambda k: c(k, "TCC_EA0_WRREQ_LEVEL_sum") / c(k, "TCC_EA0_WRREQ_sum"), "{:14.1f}")
    row("RD DRAM reqs / RD reqs", lambda k: c(k, "TCC_EA0_RDREQ_DRAM_sum") / c(k, "TCC_EA0_RDREQ_sum"))
    row("WR DRAM reqs / WR reqs", lambda k: c(k, "TCC_EA0_WRREQ_DRAM_sum") / c(k, "TCC_EA0_WRREQ_sum"))
    row("TCP->TCC read latency (cycles)", lambda k: c(k, "TCP_TCC_READ_REQ_LATENCY_sum") / c(k, "TCP_TCC_READ_REQ_sum"), "{:14.1f}")
    row("TCP->TCC write latency (cycles)", lambda k: c(k, "TCP_TCC_WRITE_REQ_LATENCY_sum") / c(k, "TCP_TCC_WRITE_REQ_sum"), "{:14.1f}")
    row("TCP read reqs (k)", lambda k: c(k, "TCP_TCC_READ_REQ_sum") / 1e3, "{:14.1f}")
    row("TCP write reqs (k)", lambda k: c(k, "TCP_TCC_WRITE_REQ_sum") / 1e3, "{:14.1f}")
    row("TCR->TCP stall / GUI_ACTIVE", lambda k: c(k, "TCP_TCR_TCP_STALL_CYCLES_sum") / c(k, "GRBM_GUI_ACTIVE"))
    row("TCP pending stall / GUI_ACTIVE", lambda k: c(k, "TCP_PENDING_STALL_CYCLES_sum") / c(k, "GRBM_GUI_ACTIVE"))
    row("TCP rd tag-conflict / GUI_ACTIVE", lambda k: c(k, "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum") / c(k, "GRBM_GUI_ACTIVE"))
    row("TCP wr tag-conflict / GUI_ACTIVE", lambda k: c(k, "TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum") / c(k, "GRBM_GUI_ACTIVE"))
    row("GRBM_GUI_ACTIVE (k cycles)", lambda k: c(k, "GRBM_GUI_ACTIVE") / 1e3, "{:14.1f}")
    row("waves", lambda k: c(k, "SQ_WAVES"), "{:14.0f}")
    row("wave cycles / wave", lambda k: c(k, "SQ_WAVE_CYCLES") / c(k, "SQ_WAVES"), "{:14.1f}")
    row("resident waves (wave cyc / GUI)", lambda k: c(k, "SQ_WAVE_CYCLES") / c(k, "GRBM_GUI_ACTIVE"), "{:14.1f}")
    row("VMEM level / VMEM inst (cycles)", lambda k: c(k, "SQ_INST_LEVEL_VMEM") /
        (c(k, "SQ_INSTS_VMEM_RD") + c(k, "SQ_INSTS_VMEM_WR")), "{:14.1f}")
    row("VMEM in flight (level / GUI)", lambda k: c(k, "SQ_INST_LEVEL_VMEM") / c(k, "GRBM_GUI_ACTIVE"), "{:14.1f}")
    row("TCC busy / GUI_ACTIVE", lambda k: c(k, "TCC_BUSY_sum") / c(k, "GRBM_GUI_ACTIVE"))
    row("TCC tag stall / TCC req", lambda k: c(k, "TCC_TAG_STALL_sum") / c(k, "TCC_REQ_sum"))
    row("TCC streaming req / TCC req", lambda k: c(k, "TCC_STREAMING_REQ_sum") / c(k, "TCC_REQ_sum"))
    for kind in ("RD", "WR"):
        for unit, names in (("channel", [f"CH_{kind}_{i:02d}" for i in range(16)]),
                            ("XCD", [f"XCD_{kind}_{x}" for x in range(8)])):
            row(f"{kind} per {unit}: max / mean", lambda k: spread([c(k, n) for n in names])[0])
            row(f"{kind} per {unit}: min / mean", lambda k: spread([c(k, n) for n in names])[1])
            row(f"{kind} per {unit}: CV", lambda k: spread([c(k, n) for n in names])[2])
    print()
    print("per-channel requests (median, thousands), all XCDs summed")
    print(f"{'channel':10s}" + "".join(f"{k + ' RD':>14s}{k + ' WR':>14s}" for k in ks))
    for i in range(16):
        cells = []
        for k in ks:
            for kind in ("RD", "WR"):
                n = f"CH_{kind}_{i:02d}"
                cells.append(f"{c(k, n) / 1e3:14.1f}" if n in vals[k] else f"{'-':>14s}")
        print(f"{i:<10d}" + "".join(cells))
    print()
    print("per-XCD requests (median, thousands), all channels summed")
    for x in range(8):
        cells = []
        for k in ks:
            for kind in ("RD", "WR"):
                n = f"XCD_{kind}_{x}"
                cells.append(f"{c(k, n) / 1e3:14.1f}" if n in vals[k] else f"{'-':>14s}")
        print(f"{x:<10d}" + "".join(cells))


if __name__ == "__main__":
    main()
