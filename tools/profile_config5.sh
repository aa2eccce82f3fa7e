#!/bin/bash
# rocprofv3 passes for bench.py's config5_combine block (fp16 two-operand
# MPI_Reduce_local at 256 MiB, fused CHAIN8 fp16 over 8 x 128 MiB): kernel
# trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes
# (MI355X_MICROARCH.md: FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2).  Run on the
# GPU box from the repo root; summarise with tools/summarize_config5.py.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/prof_c5${1:-}
export TMPDIR=/tmp
mkdir -p $OUT
cd /tmp
B="$R/bench.py --only-config5"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B --steps 20 --warmup 3 > $OUT/trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B --steps 6 --warmup 1 > $OUT/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B --steps 6 --warmup 1 > $OUT/write.log 2>&1
echo config5 profile done
