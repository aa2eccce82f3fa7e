#!/bin/bash
# The product's fused 8-operand combine with its results stored nt (KEEP_MB=0)
# or sc1 (KEEP_MB=1024: every tile), no output left in the Infinity Cache
# between uses (NSETS sets); plus tools/streams_ab at P = 1/2/4/8, nt vs sc1.
# -> gpurun_out/multi_keep_ab.log
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mka
mkdir -p $O
L=gpurun_out/multi_keep_ab.log
: > $L
run() {   # name nsets keep_mb mib skew [16]
  local d=$O/$1
  NSETS=$2 KEEP_MB=$3 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- tools/multi_gap_ab $4 20 $5 $6 > $d.log 2>&1
  local csv=$(find $d -name 'run_kernel_trace.csv' | head -n 1)
  echo "== $1 (NSETS=$2 KEEP_MB=$3, 8 x $4 MiB)" >> $L
  python3 tools/trace_medians.py "$csv" $((9 * $4 * 1048576)) 2 | grep combine_multi >> $L
}
run chain8_nt 4 0 128 4352 16
run chain8_sc1 4 1024 128 4352 16
run tree8_nt 10 0 32 4352
run tree8_sc1 10 1024 32 4352
NSETS=4 SKEWS="4352" bash tools/streams_ab.sh 128
cat gpurun_out/streams_ab.log >> $L
