#!/bin/bash
# The keep-alive must not cost back-to-back callers: synchronous 256 MiB and
# 64 MiB (4 pairs) rates with MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=0 vs the
# default, alternated processes, 300 calls each; then the idle-gap probe.
set -o pipefail
mkdir -p gpurun_out/kh
L=gpurun_out/kh/keepalive_headline_ab.log
: > $L
for i in 1 2 3 4 5; do
  for k in 0 40; do
    for mib in 256 64; do
      v=$(MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$k timeout -k 10 100 python bench.py --mib $mib --steps 300 --warmup 50 --no-extras --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])") || exit 1
      echo "keepalive_us $k mib $mib pass $i: $v" >> $L
    done
  done
done
for k in 0 40; do
  echo "== idle gaps, keepalive_us $k" >> $L
  MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$k timeout -k 10 120 python tools/idle_gap_probe.py --calls 150 2>&1 | grep "^gap" >> $L || exit 1
done
