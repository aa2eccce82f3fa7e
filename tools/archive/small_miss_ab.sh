#!/bin/bash
# The cost of padding small checked dispatches to 8 workgroups
# (direct_dispatch.hip kMinCheckedGroups): the product build (tools/ab_lib_a,
# padded) against one built with -DMPIR_DIRECT_MIN_CHECKED_GROUPS=1
# (tools/ab_lib_b, unpadded), alternating processes, tools/small_miss_ab.py.
#   build (CPU container):  bash tools/small_miss_ab.sh build
#   run (GPU box):          bash tools/small_miss_ab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname $0)/..}
if [ "$1" = build ]; then
  set -e
  rm -rf tools/ab_lib_a tools/ab_lib_b /tmp/ab_build_b
  mkdir -p tools/ab_lib_a tools/ab_lib_b
  cp mpich-pip_amd/lib/libmpich_reduce_local.so mpich-pip_amd/lib/libmpir_hip.so mpich-pip_amd/lib/libmpir_hip_tiles.hsaco tools/ab_lib_a/
  cp -r mpich-pip_amd/build /tmp/ab_build_b
  rm -f /tmp/ab_build_b/direct_dispatch.o
  make -s -C mpich-pip_amd BUILD=/tmp/ab_build_b LIBDIR=/tmp/ab_lib_b_out \
      HIPFLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-parameter -DMPIR_DIRECT_MIN_CHECKED_GROUPS=1" \
      /tmp/ab_lib_b_out/libmpir_hip.so /tmp/ab_lib_b_out/libmpich_reduce_local.so
  cp /tmp/ab_lib_b_out/libmpir_hip.so /tmp/ab_lib_b_out/libmpich_reduce_local.so tools/ab_lib_b/
  cp mpich-pip_amd/lib/libmpir_hip_tiles.hsaco tools/ab_lib_b/
  echo built
  exit 0
fi
mkdir -p gpurun_out
: > gpurun_out/small_miss_ab.log
for k in 1 2 3; do
  for l in tools/ab_lib_a tools/ab_lib_b; do
    timeout -k 10 150 python3 tools/small_miss_ab.py $l --calls 2000 --rounds 1 >> gpurun_out/small_miss_ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/small_miss_ab.log
