"""Per operand pair: the headline kernel's duration and its address-translation
counters, from one rocprofv3 run of the bench's timed loop (round 5).

    rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
        --kernel-trace --output-format csv -d OUT -o run -- \
        python3 bench.py --no-extras --no-cpu-baseline --no-variants --steps 400 --warmup 8
    python tools/archive/pair_pmc.py OUT

The bench rotates NPAIRS = 4 resident pairs, call i on pair i % 4, so the
headline kernel's dispatches, in order, cycle over the pairs (the roofline
readout's repeats after the timed loop included).  Per pair: median duration,
and the median translation misses / hits per dispatch.  A pair that runs slow on
every call with more misses points at its pages' translation (page size); with
the same misses, at where its pages sit.
"""
import csv
import glob
import os
import statistics
import sys

KERNEL = "mpir_tile_SUM_MPIR_HIP_F32"


def main():
    out = sys.argv[1]
    trace = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)
    pmc = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
    dur = {}
    for f in trace:
        for r in csv.DictReader(open(f)):
            if KERNEL in r.get("Kernel_Name", ""):
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    ctr = {}
    for f in pmc:
        for r in csv.DictReader(open(f)):
            if KERNEL in r.get("Kernel_Name", ""):
                ctr.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(set(dur) | set(ctr))
    print(f"{len(ids)} dispatches of {KERNEL} ({len(dur)} timed, {len(ctr)} with counters)")
    if not ids:
        return
    by = {p: [] for p in range(4)}
    for k, d in enumerate(ids):
        by[k % 4].append(d)
    for p in range(4):
        ds = [dur[d] for d in by[p] if d in dur]
        miss = [ctr[d].get("TCP_UTCL1_TRANSLATION_MISS_sum") for d in by[p] if d in ctr]
        hit = [ctr[d].get("TCP_UTCL1_TRANSLATION_HIT_sum") for d in by[p] if d in ctr]
        miss = [x for x in miss if x is not None]
        hit = [x for x in hit if x is not None]
        print(f"  pair slot {p}: {len(ds)} dispatches, duration median {statistics.median(ds) if ds else float('nan'):.2f} us "
              f"(p90 {sorted(ds)[int(0.9 * (len(ds) - 1))] if ds else float('nan'):.2f}); UTCL1 misses median "
              f"{statistics.median(miss) if miss else float('nan'):.0f}, hits {statistics.median(hit) if hit else float('nan'):.0f}")


if __name__ == "__main__":
    main()
