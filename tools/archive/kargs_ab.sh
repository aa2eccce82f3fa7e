#!/bin/bash
# Alternating processes, library builds in tools/ab_lib_a and tools/ab_lib_b
# (tools/sync_lib_ab.py: 64 Mi floats, hit and fresh-argument loops), 4 rounds.
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3 4; do
  for l in tools/ab_lib_a tools/ab_lib_b; do
    timeout -k 10 120 python3 tools/sync_lib_ab.py $l --steps 300 --rounds 2 2>&1 | grep "round" >> gpurun_out/kargs_ab.log || exit 1
  done
done
cat gpurun_out/kargs_ab.log
