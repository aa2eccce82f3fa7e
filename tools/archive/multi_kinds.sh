#!/bin/bash
# The fused 8-operand kernel on 8 x 128 MiB blocks (config 5's shape) with
# different element work -- fp16 CHAIN (product), fp16 TREE, f32 CHAIN, u32
# BXOR -- under rocprofv3 --kernel-trace: is the 8-stream read pattern or the
# fp16 chain the limit?  -> gpurun_out/multi_kinds.log
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mk
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- tools/multi_gap_ab 128 10 4352 16 > $O/run.log 2>&1
CSV=$(find $O/t -name 'run_kernel_trace.csv' | head -n 1)
{ cat $O/run.log; python3 tools/trace_medians.py "$CSV" $((9 * 128 * 1048576)) 2; } > gpurun_out/multi_kinds.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/t2 -o run -- tools/multi_gap_ab 32 20 4352 > $O/run2.log 2>&1
CSV=$(find $O/t2 -name 'run_kernel_trace.csv' | head -n 1)
{ echo "== TREE8 fp32 8 x 32 MiB"; python3 tools/trace_medians.py "$CSV" $((9 * 32 * 1048576)) 2; } >> gpurun_out/multi_kinds.log
