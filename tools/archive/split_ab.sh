#!/bin/bash
# Timeline split of the synchronous call under packet / queue variants
# (tools/sync_ab.py, one process each; experiments only).
for r in 1 2; do
HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 120 python3 -u tools/sync_ab.py --tag "VRAM ring, acq agent" || exit 1
HSA_ALLOCATE_QUEUE_DEV_MEM=1 MPIR_CVAR_REDUCE_LOCAL_DIRECT_ACQUIRE=none timeout -k 10 120 python3 -u tools/sync_ab.py --tag "VRAM ring, acq none" || exit 1
HSA_ALLOCATE_QUEUE_DEV_MEM=1 MPIR_CVAR_REDUCE_LOCAL_DIRECT_RELEASE=agent timeout -k 10 120 python3 -u tools/sync_ab.py --tag "VRAM ring, rel agent" || exit 1
HSA_ALLOCATE_QUEUE_DEV_MEM=1 MPIR_CVAR_REDUCE_LOCAL_DIRECT_ACQUIRE=none MPIR_CVAR_REDUCE_LOCAL_DIRECT_RELEASE=none timeout -k 10 120 python3 -u tools/sync_ab.py --tag "VRAM ring, no fences" || exit 1
done
