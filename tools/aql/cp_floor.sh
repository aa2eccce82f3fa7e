#!/bin/bash
# The CP's doorbell -> dispatch start floor on this box (tools/aql/cp_latency,
# idle cases only, HSA alone, one workgroup of the product's tile kernel) in the
# ring / kernarg placements (CP_FLOOR_PLACEMENTS=1: all four; else the library's,
# both in VRAM) and with 0-8 more idle queues on the GPU, the caller bound to the
# GPU's NUMA node (CP_FLOOR_EXTRA: the extra-queue counts, default 0), with the HIP
# runtime absent and up; then the library from C (tools/aql/product_split) and
# the product's own 4 KiB call split on the same box (tools/placement_ab.py, near).
# CP_FLOOR_MODE=noprof: the bare client with and without CP timestamps beside the
# library from C instead.
# Build: the g++ line in tools/aql/cp_latency.cpp's header.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$PWD}
node=$(timeout -k 5 120 python3 -c "
import sys; sys.path.insert(0, 'mpich-pip_amd')
import mpich_pip_amd as m; m.load(); import torch; torch.cuda.set_device(0)
print(m.placement(0)['gpu_node'])") || exit $?
cpus=$(cat /sys/devices/system/node/node$node/cpulist)
allowed=$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0)))))")
pick=$(python3 -c "
a=set(map(int,'$allowed'.split(',')))
s=set()
for part in '$cpus'.split(','):
    x,_,y=part.partition('-'); s.update(range(int(x), int(y or x)+1))
print(','.join(map(str, sorted(a & s))) or '$allowed')")
echo "GPU node $node; caller CPUs $pick"
if [ "$CP_FLOOR_MODE" = noprof ]; then
  # the library's queue runs without CP timestamps: the bare client with and
  # without them (host clock only), then the library from C, twice, alternated
  for r in 1 2; do
    for np in 0 1; do
      echo "== HIP up, ring and kernargs in VRAM, NO_PROFILE=$np"
      env HSA_ALLOCATE_QUEUE_DEV_MEM=1 IDLE_ONLY=1 KARG_VRAM=1 HIP_INIT=1 $([ $np = 1 ] && echo NO_PROFILE=1) \
          timeout -k 5 120 taskset -c $pick tools/aql/cp_latency mpich-pip_amd/lib/libmpir_hip_tiles.hsaco || exit $?
    done
    echo "== the product from C, no torch"
    timeout -k 5 120 taskset -c $pick tools/aql/product_split 4096 || exit $?
  done
  exit 0
fi
for ring in 0 1; do
  for karg in 0 1; do
    [ "$CP_FLOOR_PLACEMENTS" = 1 ] || [ $ring$karg = 11 ] || continue
    for extra in ${CP_FLOOR_EXTRA:-0}; do
      for hip in 0 1; do
        [ $ring$karg = 11 ] || [ $hip = 0 ] || continue
        echo "== ring in $([ $ring = 1 ] && echo VRAM || echo host memory), kernargs $([ $karg = 1 ] && echo VRAM || echo host pool), $extra extra queues, HIP $([ $hip = 1 ] && echo up || echo absent)"
        env HSA_ALLOCATE_QUEUE_DEV_MEM=$ring IDLE_ONLY=1 EXTRA_QUEUES=$extra $([ $karg = 1 ] && echo KARG_VRAM=1) \
            $([ $hip = 1 ] && echo HIP_INIT=1) \
            timeout -k 5 120 taskset -c $pick tools/aql/cp_latency mpich-pip_amd/lib/libmpir_hip_tiles.hsaco || exit $?
      done
    done
  done
done
for r in 1 2; do
  echo "== the product from C, no torch ($r)"
  timeout -k 5 120 taskset -c $pick tools/aql/product_split 4096 || exit $?
done
echo "== the product (placement_ab near, 1 round)"
timeout -k 10 300 python3 -u tools/placement_ab.py 1 2000 near
