#!/bin/bash
# Builds tools/aql/concurrent_kernels.co (device-only code object) and tools/aql/concurrent_probe.
set -e
cd "$(dirname "$0")/../.."
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 --cuda-device-only --no-gpu-bundle-output -c \
   -o tools/aql/concurrent_kernels.co tools/aql/concurrent_kernels.hip
g++ -O2 -std=c++17 -I/opt/rocm/include -o tools/aql/concurrent_probe tools/aql/concurrent_probe.cpp \
   -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
