#!/usr/bin/env python3
"""Median kernel duration per kernel name from a rocprofv3 kernel-trace CSV.

    python tools/trace_medians.py <run_kernel_trace.csv> <algorithmic bytes per launch> [skip]

Prints name, launches, median / min duration (us) and median fraction of the
8 TB/s HBM peak; `skip` drops that many first launches of every kernel."""
import collections
import csv
import statistics
import sys

path, alg = sys.argv[1], float(sys.argv[2])
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
d = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for name, v in sorted(d.items(), key=lambda kv: statistics.median(kv[1][skip:] or kv[1])):
    v = v[skip:] or v
    med = statistics.median(v)
    print(f"{name[:90]:90s} n={len(v):3d} median {med:8.2f} min {min(v):8.2f} frac(med) {alg / med / 8e6:.3f}")
