#!/usr/bin/env python3
"""Split one `tools/slow_kernel_pmc.sh` pass (per-dispatch counters beside the
kernel trace of the headline loop) into fast and slow launches of the
headline kernel, and print each counter's mean per launch for both.

    python3 tools/slow_pmc_summary.py gpurun_out/slow_pmc<TAG> [kernel-substring]

Slow = longer than the median + 4 us (the isolated slow launches of DESIGN.md
§(d)).  Durations come from the kernel trace (joined on Dispatch_Id), or from
the counter file's own timestamps when it has them.
"""
import csv
import glob
import os
import statistics
import sys


def find(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def main():
    d = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "mpir_tile_SUM_MPIR_HIP_F32"
    dur = {}
    kt = find(d, "*kernel_trace.csv")
    if kt:
        for r in csv.DictReader(open(kt)):
            if kern in r["Kernel_Name"]:
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    cnt = {}
    cc = find(d, "*counter_collection.csv")
    for r in csv.DictReader(open(cc)):
        if kern not in r["Kernel_Name"]:
            continue
        did = r["Dispatch_Id"]
        cnt.setdefault(did, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        if did not in dur and r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    ids = [i for i in cnt if i in dur]
    if not ids:
        print("no dispatches joined")
        return 1
    med = statistics.median(dur[i] for i in ids)
    slow = [i for i in ids if dur[i] > med + 4.0]
    fast = [i for i in ids if dur[i] <= med]
    names = sorted({n for i in ids for n in cnt[i]})
    print(f"{kern}: launches {len(ids)}, median {med:.2f} us, slow (> median + 4 us) {len(slow)}")
    print(f"{'counter':40s} {'fast mean':>16s} {'slow mean':>16s} {'slow/fast':>10s}")
    print(f"{'duration_us':40s} {statistics.mean(dur[i] for i in fast):16.2f} "
          f"{(statistics.mean(dur[i] for i in slow) if slow else float('nan')):16.2f}")
    for n in names:
        fv = statistics.mean(cnt[i].get(n, 0.0) for i in fast)
        sv = statistics.mean(cnt[i].get(n, 0.0) for i in slow) if slow else float("nan")
        ratio = sv / fv if fv else float("nan")
        print(f"{n:40s} {fv:16.1f} {sv:16.1f} {ratio:10.4f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
