#!/bin/bash
# Builds tools/aql/aql2_kernels.co (device-only code object) and tools/aql/aql2.
set -e
cd "$(dirname "$0")/../.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c -O3 -std=c++17 \
   -o tools/aql/aql2_kernels.co tools/aql/aql2_kernels.hip
$H --offload-arch=gfx950 -O2 -std=c++17 -Itools/aql -o tools/aql/aql2 -x hip tools/aql/aql2.cpp -lhsa-runtime64
