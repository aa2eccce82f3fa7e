#!/bin/bash
# Store-policy A/B against operand rotation depth (tools/sync_ab.py, one
# process each): does a policy win only when the bench's own rotation lets a
# later call re-read an earlier call's result from the MALL?
#   bash tools/pairs_ab.sh [rounds=3] > gpurun_out/pairs_ab.log
for r in $(seq 1 ${1:-3}); do
  for np in 4 8; do
    HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 120 python3 -u tools/sync_ab.py --tag "whole<=64M (default)" --pairs $np || exit 1
    HSA_ALLOCATE_QUEUE_DEV_MEM=1 MPIR_CVAR_REDUCE_LOCAL_KEEP_MODE=tail timeout -k 10 120 python3 -u tools/sync_ab.py --tag "tail 64M" --pairs $np || exit 1
    HSA_ALLOCATE_QUEUE_DEV_MEM=1 MPIR_CVAR_REDUCE_LOCAL_KEEP_MB=0 timeout -k 10 120 python3 -u tools/sync_ab.py --tag "all nt" --pairs $np || exit 1
  done
done
