#!/bin/bash
# Does the fused 8-operand kernel's figure depend on the Infinity Cache?
# tools/multi_gap_ab under rocprofv3 --kernel-trace with 2 rotated operand sets
# (outputs stay in the 256 MB MALL between uses when stored sc1) against enough
# sets that no output survives (NSETS x block > 256 MB), stores sc1 (KEEP_MB
# default 64) or all nt (KEEP_MB=0).  -> gpurun_out/multi_cache_ab.log
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mc
mkdir -p $O
L=gpurun_out/multi_cache_ab.log
: > $L
run() {   # name nsets keep_mb mib skew [16]
  local d=$O/$1
  NSETS=$2 KEEP_MB=$3 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- tools/multi_gap_ab $4 20 $5 $6 > $d.log 2>&1
  local csv=$(find $d -name 'run_kernel_trace.csv' | head -n 1)
  echo "== $1 (NSETS=$2 KEEP_MB=$3, 8 x $4 MiB)" >> $L
  python3 tools/trace_medians.py "$csv" $((9 * $4 * 1048576)) 2 >> $L
}
run tree8_sets2_keep64 2 64 32 4352
run tree8_sets2_nt 2 0 32 4352
run tree8_sets10_keep64 10 64 32 4352
run tree8_sets10_nt 10 0 32 4352
run chain8_sets2_keep64 2 64 128 4352 16
run chain8_sets4_keep64 4 64 128 4352 16
run chain8_sets4_nt 4 0 128 4352 16
