#!/bin/bash
# Queue dispatch timestamps on (default, for bench.py's roofline readout) vs
# off (MPIR_CVAR_REDUCE_LOCAL_DIRECT_TIMESTAMPS=0): synchronous 256 MiB and
# 64 MiB call rates, alternated processes.
set -o pipefail
mkdir -p gpurun_out/ts
L=gpurun_out/ts/ts_ab.log
: > $L
for i in 1 2 3 4; do
  for t in 1 0; do   # 1 = the calls' queue timestamped too (round-2 default)
    for mib in 256 64; do
      v=$(MPIR_CVAR_REDUCE_LOCAL_DIRECT_TIMESTAMPS=$t timeout -k 10 100 python bench.py --mib $mib --steps 300 --warmup 50 --no-extras --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])") || exit 1
      echo "timestamps $t mib $mib pass $i: $v" >> $L
    done
  done
done
