#!/bin/bash
# A/B of the host-thread pool size (MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS=4 vs
# the default, sized from the usable CPUs): bench.py's host_resident /
# pcie_inclusive legs and tools/host_latency.py, alternated on one box.
#   bash tools/host_threads_ab.sh   (on the GPU box, from the repo root)
set -o pipefail
mkdir -p gpurun_out/ht
: > gpurun_out/ht/bench.log
: > gpurun_out/ht/latency.log
for t in 4 default 4 default; do
  if [ $t = default ]; then unset MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS; else export MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS=$t; fi
  echo "== threads $t" >> gpurun_out/ht/bench.log
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ht/b.json 2>&1 || exit 1
  python -c "
import json
for ln in open('gpurun_out/ht/b.json'):
    if ln.startswith('{'):
        d=json.loads(ln); print('value', d['value'], 'host_resident', d['host_resident']['value'], d['host_resident']['pageable_value'], 'pcie', d['pcie_inclusive']['value'], d['pcie_inclusive']['pageable_value'])
" >> gpurun_out/ht/bench.log
  echo "== threads $t" >> gpurun_out/ht/latency.log
  timeout -k 10 300 python tools/host_latency.py --reps 100 2>&1 | grep -E "65536|262144|1048576" | grep -v "^device->device" >> gpurun_out/ht/latency.log || exit 1
done
