#!/bin/bash
# Does an idle HSA queue that merely exists slow the calls' queue?  Synchronous
# 256 / 64 MiB rates with 0, 1 and 2 extra idle queues
# (MPIR_CVAR_REDUCE_LOCAL_DIRECT_IDLE_QUEUES), and with the keep-alive knob at
# 0 / 40 (never armed by back-to-back calls), alternated processes, 300 calls.
set -o pipefail
mkdir -p gpurun_out/lq
L=gpurun_out/lq/lazy_queues_ab.log
: > $L
for i in 1 2 3 4; do
  for cfg in "IDLE=0 KA=0" "IDLE=0 KA=40" "IDLE=1 KA=0" "IDLE=2 KA=0"; do
    eval $cfg
    for mib in 256 64; do
      v=$(MPIR_CVAR_REDUCE_LOCAL_DIRECT_IDLE_QUEUES=$IDLE MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$KA timeout -k 10 100 python bench.py --mib $mib --steps 300 --warmup 50 --no-extras --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'])") || exit 1
      echo "idle_queues $IDLE keepalive $KA mib $mib pass $i: $v" >> $L
    done
  done
done
