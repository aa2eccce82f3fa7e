#!/bin/bash
# Per-dispatch GRBM counters of the headline loop (300 synchronous calls) beside
# the kernel trace: do the isolated slow launches run at a lower clock (same
# busy cycles, more time) or stall (more busy cycles)?  One --pmc pass.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/slow_pmc${TAG:-}
export TMPDIR=/tmp
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${PMC:-GRBM_COUNT GRBM_GUI_ACTIVE} --output-format csv -d $OUT -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-extras --no-variants --steps 300 --warmup 20 > $OUT/run.log 2>&1
echo pmc done
