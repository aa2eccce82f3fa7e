#!/bin/bash
# Kernarg preload (-mllvm -amdgpu-kernarg-preload-count=4: the four lean-tile
# arguments arrive in SGPRs at wave launch) vs the plain s_load prologue, on the
# bare HSA dispatch path of tools/aql/prepost (plain mode), alternated processes.
set -o pipefail
mkdir -p gpurun_out/pl
L=gpurun_out/pl/preload_ab.log
: > $L
for i in 1 2 3; do
  for v in prepost_kernel prepost_kernel_preload; do
    echo "== $v pass $i" >> $L
    PLAIN_ONLY=1 ROUNDS=3 HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 100 tools/aql/prepost tools/aql/$v.co 300 | grep "plain" >> $L || exit 1
  done
done
