#!/bin/bash
# Mixed-residency latency with and without the copy-pool split of the slot
# copies (tools/host_latency.py; one process each).
for r in 1 2; do
  MPIR_CVAR_REDUCE_LOCAL_MIXED_SPLIT_KB=1048576 HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 200 python3 -u tools/host_latency.py --reps 100 | grep -E "host->device|device->host|pinned->device" | awk '{print "nosplit", $0}' || exit 1
  HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 200 python3 -u tools/host_latency.py --reps 100 | grep -E "host->device|device->host|pinned->device" | awk '{print "split256", $0}' || exit 1
done
