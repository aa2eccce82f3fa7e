#!/usr/bin/env python3
"""Condense a rocprofv3 run of tools/profile_r0N.sh into committed evidence.

    python tools/summarize_profile.py gpurun_out/prof_r02 r02 [kernel-name-substring]

The kernel defaults to the one the synchronous call dispatches since round 2
(mpir_tile_SUM_MPIR_HIP_F32, direct AQL dispatch); round 1's runs used
k_reduce_tile_lean<mpir_hip::OpSum, float>.  A trace64/ pass (config 2, 64 MiB
per operand), when present, adds a second table.

Writes, under profiles/:
  <tag>_kernel_stats.csv      rocprofv3 --stats kernel summary (names shortened)
  <tag>_pmc.csv               FETCH_SIZE / WRITE_SIZE rows of the reduce kernel
  <tag>_summary.md            per-launch duration, achieved GB/s, HBM traffic
  pmc_traffic.json            per-launch HBM bytes bench.py reports as roofline.traffic

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of
a wide coalesced streaming read (16 B/lane loads), so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import csv
import json
import os
import statistics
import sys

KERNEL = "mpir_tile_SUM_MPIR_HIP_F32"
KERNEL_LABEL = {"mpir_tile_SUM_MPIR_HIP_F32": "mpir_tile_SUM_MPIR_HIP_F32 (reduce_tile<OpSum,float>, direct AQL dispatch)",
                "k_reduce_tile_lean<mpir_hip::OpSum, float>": "mpir_hip::k_reduce_tile_lean<OpSum,float>"}
PEAK = 8.0e12


def short(name: str) -> str:
    return name if len(name) < 120 else name[:117] + "..."


def main():
    src, tag = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else KERNEL
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)

    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in rows:
            r = dict(r)
            r["Name"] = short(r["Name"])
            w.writerow(r)
    kstat = next(r for r in rows if kernel in r["Name"])
    avg_ns = float(kstat["AverageNs"])

    trace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
             if kernel in r["Kernel_Name"]]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]

    pmc = {}
    out_rows = []
    for name in ("fetch", "write"):
        for r in csv.DictReader(open(os.path.join(src, name, "run_counter_collection.csv"))):
            if kernel in r["Kernel_Name"]:
                pmc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                out_rows.append({k: (short(v) if k == "Kernel_Name" else v) for k, v in r.items()})
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(out_rows[0].keys()))
        w.writeheader()
        w.writerows(out_rows)

    grid = int(trace[0]["Grid_Size_X"])
    operand_bytes = grid // 256 * 16384          # one 16 KiB tile per 256-thread workgroup
    alg = 3 * operand_bytes
    fetch_kb = statistics.median(pmc["FETCH_SIZE"])
    write_kb = statistics.median(pmc["WRITE_SIZE"])
    hbm = int(round((2 * fetch_kb + write_kb) * 1024))
    achieved = alg / (avg_ns * 1e-9)
    d = {
        "kernel": KERNEL_LABEL.get(kernel, kernel),
        "operand_bytes": operand_bytes,
        "algorithmic_bytes_per_launch": alg,
        "hbm_bytes_per_launch": hbm,
        "traffic_over_algorithmic": round(hbm / alg, 5),
        "fetch_size_kb_median": fetch_kb,
        "write_size_kb_median": write_kb,
        "correction": "hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halves wide streaming reads)",
        "rocprof_avg_launch_ns": avg_ns,
        "rocprof_achieved_GBps": round(achieved / 1e9, 1),
        "rocprof_frac_of_peak": round(achieved / PEAK, 4),
        "source": f"profiles/{tag}_kernel_stats.csv, profiles/{tag}_pmc.csv",
    }
    t64 = os.path.join(src, "trace64", "run_kernel_stats.csv")
    k64 = None
    if os.path.exists(t64):
        k64 = next(r for r in csv.DictReader(open(t64)) if kernel in r["Name"])
        tr64 = [r for r in csv.DictReader(open(os.path.join(src, "trace64", "run_kernel_trace.csv")))
                if kernel in r["Kernel_Name"]]
        ob64 = int(tr64[0]["Grid_Size_X"]) // 256 * 16384
        avg64 = float(k64["AverageNs"])
        d["config2_64MiB"] = {"operand_bytes": ob64, "rocprof_avg_launch_ns": avg64,
                              "rocprof_median_launch_ns": statistics.median(
                                  int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr64),
                              "rocprof_frac_of_peak": round(3 * ob64 / (avg64 * 1e-9) / PEAK, 4),
                              "launches": int(k64["Calls"])}
        with open(os.path.join(prof, f"{tag}_kernel_stats_64MiB.csv"), "w", newline="") as f:
            rows64 = list(csv.DictReader(open(t64)))
            w = csv.DictWriter(f, fieldnames=list(rows64[0].keys()))
            w.writeheader()
            for r in rows64:
                r = dict(r)
                r["Name"] = short(r["Name"])
                w.writerow(r)
    # keep the other kernels' entries (config5_fp16, tools/summarize_config5.py)
    pj = os.path.join(prof, "pmc_traffic.json")
    if os.path.exists(pj):
        old = json.load(open(pj))
        for k in ("config5_fp16",):
            if k in old:
                d[k] = old[k]
    json.dump(d, open(pj, "w"), indent=1)
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary ({tag})\n\n")
        f.write(f"Command: `bash {os.environ.get('PROFILE_SCRIPT', 'tools/profile_r03.sh')}` on one MI355X "
                "(bench.py --no-cpu-baseline --no-extras: fp32 MPI_SUM, 256 MiB per operand).\n\n")
        f.write("| quantity | value |\n|---|---|\n")
        f.write(f"| kernel | `{d['kernel']}` |\n")
        f.write(f"| launches traced | {kstat['Calls']} |\n")
        f.write(f"| average / min / max duration | {avg_ns/1e3:.2f} / {float(kstat['MinNs'])/1e3:.2f} / "
                f"{float(kstat['MaxNs'])/1e3:.2f} us |\n")
        f.write(f"| median duration (trace) | {statistics.median(durs)/1e3:.2f} us |\n")
        f.write(f"| algorithmic bytes per launch | {alg:,} (3 x {operand_bytes:,}) |\n")
        f.write(f"| achieved (algorithmic / average) | {achieved/1e9:.1f} GB/s = {achieved/PEAK:.3f} of 8.0 TB/s |\n")
        f.write(f"| FETCH_SIZE (median, KiB) | {fetch_kb:.1f} (x2 gfx950 correction) |\n")
        f.write(f"| WRITE_SIZE (median, KiB) | {write_kb:.1f} |\n")
        f.write(f"| HBM traffic per launch | {hbm:,} B = {hbm/alg:.5f} x algorithmic |\n")
        f.write(f"| grid / workgroup / VGPR / SGPR | {grid // 256} WGs x 256, VGPR {trace[0]['VGPR_Count']}, "
                f"SGPR {trace[0]['SGPR_Count']} |\n")
        if k64 is not None:
            c2 = d["config2_64MiB"]
            f.write(f"\n## Config 2 (64 MiB per operand, `--mib 64`)\n\n| quantity | value |\n|---|---|\n")
            f.write(f"| launches traced | {c2['launches']} |\n")
            f.write(f"| average / median / min / max duration | {c2['rocprof_avg_launch_ns']/1e3:.2f} / "
                    f"{c2['rocprof_median_launch_ns']/1e3:.2f} / {float(k64['MinNs'])/1e3:.2f} / "
                    f"{float(k64['MaxNs'])/1e3:.2f} us |\n")
            f.write(f"| achieved (algorithmic / average) | {c2['rocprof_frac_of_peak']:.3f} of 8.0 TB/s |\n")
            f.write("\n`--mib 64` rotates the bench's 4 pairs, and results of at most 64 MiB are stored `sc1`\n"
                    "(they stay in the 256 MB Infinity Cache), so each call re-reads its inout from the\n"
                    "cache four calls later: this is a cache figure, not config 2. Config 2 proper (16\n"
                    "windows over 2 GiB, nothing re-read) is `config2_64MiB` in the bench line.\n")
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
