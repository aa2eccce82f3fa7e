#!/bin/bash
# The driver's bench shape (--steps 20 --warmup 5, fresh process each) for two
# bench.py versions alternated: $1 and $2 (scripts in the repo root), $3 rounds.
# Headline loop only (--no-extras --no-cpu-baseline --no-variants).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
mkdir -p gpurun_out
L=gpurun_out/driver_shape_ab.log
: > $L
for k in $(seq 1 ${3:-6}); do
  for b in $1 $2; do
    timeout -k 10 120 python3 $b --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-variants > /tmp/ds.out 2>&1 || { tail -5 /tmp/ds.out; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('/tmp/ds.out') if l.startswith('{')][-1]); print('$b', d['per_gpu']['frac_of_hbm_peak'], d['ms_per_step'])" >> $L
  done
done
cat $L
