#!/bin/bash
# tools/streams_ab under rocprofv3 --kernel-trace for a few staging skews;
# fraction of 8 TB/s per kernel (algorithmic bytes: (P + 1) x block for k_rw,
# P x block for k_ro) -> gpurun_out/streams_ab.log
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/st
mkdir -p $O
L=gpurun_out/streams_ab.log
: > $L
M=${1:-32}
for SK in ${SKEWS:-4352 0 256 65792 1048832}; do
  d=$O/s$SK
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- tools/streams_ab $M 20 $SK > $d.log 2>&1
  csv=$(find $d -name 'run_kernel_trace.csv' | head -n 1)
  echo "== block $M MiB, skew $SK" >> $L
  python3 - "$csv" $M >> $L <<'PY'
import csv, re, statistics, sys
path, mib = sys.argv[1], int(sys.argv[2])
d = {}
for r in csv.DictReader(open(path)):
    d.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = []
for name, v in d.items():
    m = re.search(r"k_(rwk|rwip|rw|ro)<(\d+)(?:, (\d+))?(?:, (\d+))?>", name)
    if not m:
        continue
    kind, p, il = m.group(1), int(m.group(2)), int(m.group(3) or 0)
    if kind == "rwk":
        kind, il = "rw K%d pol%s" % (il, m.group(4)), 0
    v = v[2:] or v
    med = statistics.median(v)
    alg = (p + (1 if kind.startswith("rw") else 0)) * mib * 1048576
    rows.append((kind, p, il, med, alg / med / 8e6))
for kind, p, il, med, f in sorted(rows):
    print(f"  {kind} P{p} {'interleaved' if il else 'strided    '}  median {med:8.2f} us  frac {f:.3f}")
PY
done
