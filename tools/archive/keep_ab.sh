#!/bin/bash
# Store policy at 64 MiB (config 2, 16 rotating windows, nothing re-read):
# sc1 (default: results <= 64 MiB stay in the Infinity Cache for their next
# reader) against all-nt (MPIR_CVAR_REDUCE_LOCAL_KEEP_MB=0), alternated in
# separate processes.  tools/k20_probe.py reports call and CP kernel time.
set -o pipefail
mkdir -p gpurun_out/keep
L=gpurun_out/keep/keep_ab_${MIB:-64}.log
: > $L
for i in 1 2 3 4; do
  for k in 64 0; do
    echo "== KEEP_MB $k (pass $i)" >> $L
    MPIR_CVAR_REDUCE_LOCAL_KEEP_MB=$k timeout -k 10 100 python -u tools/k20_probe.py --mib ${MIB:-64} --reps 3 --steps 48 2>&1 | grep "^rep" >> $L || exit 1
  done
done
