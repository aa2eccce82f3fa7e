#!/usr/bin/env python3
"""Condense tools/profile_config5.sh's rocprofv3 passes into committed evidence.

    python3 tools/summarize_config5.py gpurun_out/prof_c5 r04

Writes profiles/<tag>/config5_kernel_stats.csv, profiles/<tag>/config5_summary.md
and the "config5_fp16" entry of profiles/pmc_traffic.json, which bench.py's
config5_combine block reports as traffic.  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: (2 x FETCH_SIZE + WRITE_SIZE) KiB (gfx950's FETCH_SIZE
counts half the bytes of wide streaming reads).
"""
import csv
import glob
import json
import os
import statistics
import sys

PEAK = 8.0e12
MIB = 1 << 20
KERNELS = {
    # key: (name substring(s), algorithmic bytes per launch)
    "two_operand": (("mpir_tile_SUM_MPIR_HIP_F16",), 3 * 256 * MIB),
    # k_combine_multi<OpSum, _Float16, P = 8, TREE = false (CHAIN), ...>, mangled
    "chain8": (("k_combine_multi", "OpSumEDF16_Li8ELb0"), 9 * 128 * MIB),
}


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not hits:
        raise SystemExit(f"{pat} missing under {d}")
    return hits[0]


def match(name, subs):
    return all(s in name for s in subs)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outdir = os.path.join(root, "profiles", tag)
    os.makedirs(outdir, exist_ok=True)
    stats = list(csv.DictReader(open(find(os.path.join(src, "trace"), "*kernel_stats.csv"))))
    with open(os.path.join(outdir, "config5_kernel_stats.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(stats[0].keys()))
        w.writeheader()
        for r in stats:
            r = dict(r)
            r["Name"] = r["Name"] if len(r["Name"]) < 160 else r["Name"][:157] + "..."
            w.writerow(r)
    trace = list(csv.DictReader(open(find(os.path.join(src, "trace"), "*kernel_trace.csv"))))
    pmc = {k: {} for k in KERNELS}
    for part in ("fetch", "write"):
        for r in csv.DictReader(open(find(os.path.join(src, part), "*counter_collection.csv"))):
            for k, (subs, _) in KERNELS.items():
                if match(r["Kernel_Name"], subs):
                    pmc[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res, lines = {}, [f"# config 5's combine at one GPU (fp16), rocprofv3 ({tag})", "",
                      f"Source: `tools/profile_config5.sh` (bench.py --only-config5), `{src}`.", "",
                      "| kernel | launches | avg us | median us | frac of 8 TB/s | HBM bytes / launch | / algorithmic |",
                      "|---|---|---|---|---|---|---|"]
    for k, (subs, alg) in KERNELS.items():
        st = next((r for r in stats if match(r["Name"], subs)), None)
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in trace if match(r["Kernel_Name"], subs)]
        if st is None or not durs or "FETCH_SIZE" not in pmc[k] or "WRITE_SIZE" not in pmc[k]:
            lines.append(f"| {k} | (missing) | | | | | |")
            continue
        avg_ns = float(st["AverageNs"])
        hbm = int(round((2 * statistics.median(pmc[k]["FETCH_SIZE"]) + statistics.median(pmc[k]["WRITE_SIZE"])) * 1024))
        res[k] = {"kernel": st["Name"][:160], "launches": len(durs), "rocprof_avg_us": round(avg_ns * 1e-3, 3),
                  "rocprof_median_us": round(statistics.median(durs) * 1e-3, 3),
                  "frac_of_peak": round(alg / (avg_ns * 1e-9) / PEAK, 4),
                  "algorithmic_bytes_per_launch": alg, "hbm_bytes_per_launch": hbm,
                  "traffic_over_algorithmic": round(hbm / alg, 5)}
        r = res[k]
        lines.append(f"| {k}: `{r['kernel'][:90]}` | {r['launches']} | {r['rocprof_avg_us']} | {r['rocprof_median_us']} "
                     f"| {r['frac_of_peak']} | {hbm:,} | {r['traffic_over_algorithmic']} |")
    open(os.path.join(outdir, "config5_summary.md"), "w").write("\n".join(lines) + "\n")
    p = os.path.join(root, "profiles", "pmc_traffic.json")
    d = json.load(open(p)) if os.path.exists(p) else {}
    d["config5_fp16"] = dict(res, source=f"profiles/{tag}/config5_kernel_stats.csv, profiles/{tag}/config5_summary.md")
    json.dump(d, open(p, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
