#!/bin/bash
# The keep-alive's barrier packet on the calls' own queue (no extra queue for
# the hardware scheduler to map) vs off: spikes (tools/ka_probe.py), idle-gap
# effect (tools/idle_gap_probe.py), back-to-back rates (bench.py, alternated).
set -o pipefail
mkdir -p gpurun_out/ks
L=gpurun_out/ks/keepalive_same_ab.log
: > $L
export MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_QUEUE=same
for k in 0 40; do
  echo "== ka_probe keepalive $k (same queue)" >> $L
  MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$k timeout -k 10 60 python tools/ka_probe.py 2>&1 | grep -E "^rep" >> $L || exit 1
  echo "== idle gaps keepalive $k (same queue)" >> $L
  MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$k timeout -k 10 120 python tools/idle_gap_probe.py --calls 150 2>&1 | grep "^gap" >> $L || exit 1
done
for i in 1 2 3 4; do
  for k in 0 40; do
    for mib in 256 64; do
      v=$(MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US=$k timeout -k 10 100 python bench.py --mib $mib --steps 300 --warmup 50 --no-extras --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'])") || exit 1
      echo "keepalive_us $k mib $mib pass $i: $v" >> $L
    done
  done
done
