#!/bin/bash
# Host combine with the floating pool (MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA=0)
# against the node pools (default), alternated processes, on pageable pairs
# first-touched on each NUMA node (tools/pinned_read_probe.py NUMA_SEQ).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do
for v in 0 1; do
MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA=$v NUMA_SEQ=1 timeout -k 10 200 python3 -u tools/pinned_read_probe.py 7 >> gpurun_out/numa_ab.log 2>&1 || exit 1
done
done
cat gpurun_out/numa_ab.log
