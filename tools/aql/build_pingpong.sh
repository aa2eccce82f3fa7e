#!/bin/bash
# Builds tools/aql/pingpong_kernel.co (device-only code object) and tools/aql/pingpong.
set -e
cd "$(dirname "$0")/../.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 --cuda-device-only --no-gpu-bundle-output -c \
   -o tools/aql/pingpong_kernel.co tools/aql/pingpong_kernel.hip
$H -O2 -std=c++17 -o tools/aql/pingpong tools/aql/pingpong.cpp -lhsa-runtime64
