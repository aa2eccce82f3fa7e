#!/bin/bash
# Packet release fence scope (MPIR_CVAR_REDUCE_LOCAL_DIRECT_RELEASE: system =
# product, agent, none = no fence, incorrect, the cost ceiling), synchronous
# 256 / 64 MiB call rates in alternated processes, 300 calls each.
set -o pipefail
mkdir -p gpurun_out/sc
L=gpurun_out/sc/scope_ab.log
: > $L
for i in 1 2 3; do
  for r in system agent none; do
    for mib in 256 64; do
      v=$(MPIR_CVAR_REDUCE_LOCAL_DIRECT_RELEASE=$r timeout -k 10 100 python bench.py --mib $mib --steps 300 --warmup 50 --no-extras --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])") || exit 1
      echo "release $r mib $mib pass $i: $v" >> $L
    done
  done
done
