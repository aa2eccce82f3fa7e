#!/bin/bash
# The synchronous call's wait: pause loop (product) vs MONITORX / MWAITX on the
# completion signal's value line (MPIR_CVAR_REDUCE_LOCAL_WAIT_MWAITX=1);
# 256 / 64 MiB, 300 calls, alternated processes.
set -o pipefail
mkdir -p gpurun_out/mw
L=gpurun_out/mw/mwaitx_ab.log
: > $L
for i in 1 2 3 4; do
  for w in 0 1; do
    for mib in 256 64; do
      v=$(MPIR_CVAR_REDUCE_LOCAL_WAIT_MWAITX=$w timeout -k 10 100 python bench.py --mib $mib --steps 300 --warmup 50 --no-extras --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'])") || exit 1
      echo "mwaitx $w mib $mib pass $i: $v" >> $L
    done
  done
done
