#!/bin/bash
# rocprofv3 passes for config 2 (64 MiB per operand, 16 rotating windows):
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_c2
export TMPDIR=/tmp
mkdir -p $OUT
P="python3 $R/tools/config2_pmc.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $P --k 64 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P --k 16 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P --k 16 > $OUT/write.log 2>&1
echo profile done
