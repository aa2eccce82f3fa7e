#!/bin/bash
# tools/config2_ab at 64 MiB: HIP-event medians per store-policy set, then the
# nt set under rocprofv3 --kernel-trace --stats (the CP's own durations)
set -e
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/config2_ab
mkdir -p $OUT
timeout -k 10 120 tools/config2_ab 64 150 nt
timeout -k 10 120 tools/config2_ab 64 150 sc1
timeout -k 10 120 tools/config2_ab 256 60 nt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- tools/config2_ab 64 150 nt > $OUT/rocprof.log 2>&1
python3 tools/trace_medians.py $OUT 2>/dev/null || find $OUT -name "*kernel_stats.csv" -exec cat {} \;
