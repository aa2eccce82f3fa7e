#!/bin/bash
# Interleaved runs of tools/sync_ab.py under several runtime configurations
# (one process each).  Run from the repo root on the GPU box.
#   bash tools/sync_ab.sh [rounds=3] [set=all|vram] > gpurun_out/sync_ab.log
R=${1:-3}
SET=${2:-all}
for r in $(seq 1 $R); do
    timeout -k 10 120 python3 -u tools/sync_ab.py --tag "ring in host memory" || exit 1
    HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 120 python3 -u tools/sync_ab.py --tag "ring in VRAM" || exit 1
    if [ "$SET" = all ]; then
        MPIR_CVAR_REDUCE_LOCAL_DIRECT_SIGNAL=interrupt timeout -k 10 120 python3 -u tools/sync_ab.py --tag "interrupt signal" || exit 1
        MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip timeout -k 10 120 python3 -u tools/sync_ab.py --tag "HIP path" || exit 1
        MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 120 python3 -u tools/sync_ab.py --tag "HIP path, ring in VRAM" || exit 1
    fi
done
