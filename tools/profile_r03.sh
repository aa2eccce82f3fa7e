#!/bin/bash
# rocprofv3 passes for the round-3 bench workload (run on the GPU box from the
# repo root): kernel trace + stats of the synchronous MPI_Reduce_local loop at
# 256 MiB (direct AQL dispatch) and 64 MiB (config 2), then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes at 256 MiB (TCC slots: FETCH_SIZE 3 +
# WRITE_SIZE 2 > 4, MI355X_MICROARCH.md).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_${1:-r03}
export TMPDIR=/tmp
mkdir -p $OUT
B="python3 $R/bench.py --no-cpu-baseline --no-extras --no-variants"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 50 --warmup 5 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace64 -o run -- $B --mib 64 --steps 64 --warmup 8 > $OUT/trace64.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B --steps 10 --warmup 2 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B --steps 10 --warmup 2 > $OUT/write.log 2>&1
echo profile done
