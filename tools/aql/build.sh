#!/bin/bash
# Builds tools/aql/aql_kernels.co (device-only code object) and tools/aql/aql_ab.
set -e
cd "$(dirname "$0")/../.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c -O3 -std=c++17 -ffp-contract=off \
   -Impich-pip_amd/csrc/hip -Impich-pip_amd/csrc/host -Iinclude -o tools/aql/aql_kernels.co tools/aql/aql_kernels.hip
$H --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -o tools/aql/aql_ab tools/aql/aql_ab.cpp \
   -Lmpich-pip_amd/lib -lmpich_reduce_local -lhsa-runtime64 -Wl,-rpath,'$ORIGIN/../../mpich-pip_amd/lib'
