#!/bin/bash
# Builds tools/aql/prepost_kernel.co (device-only code object) and tools/aql/prepost.
set -e
cd "$(dirname "$0")/../.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only --no-gpu-bundle-output -c \
   -I mpich-pip_amd/csrc/hip -o tools/aql/prepost_kernel.co tools/aql/prepost_kernel.hip
$H -O2 -std=c++17 -o tools/aql/prepost tools/aql/prepost.cpp -lhsa-runtime64
