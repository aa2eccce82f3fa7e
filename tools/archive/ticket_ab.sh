#!/bin/bash
# tools/ticket_ab.hip under rocprofv3 --kernel-trace at 256 and 64 MiB per operand;
# per-variant medians with tools/trace_medians.py -> gpurun_out/ticket_ab.log
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tk
mkdir -p $O
for M in 256 64; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/m$M -o run -- tools/ticket_ab $M 20 > $O/m$M.log 2>&1
  CSV=$(find $O/m$M -name 'run_kernel_trace.csv' | head -n 1)
  { echo "== $M MiB per operand"; grep -E "check|variant" $O/m$M.log; python3 tools/trace_medians.py "$CSV" $((3 * M * 1048576)); } >> gpurun_out/ticket_ab.log
done
