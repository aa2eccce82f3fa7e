#!/bin/bash
# builds tools/aql/kslot_ab (host harness; loads the product code objects at run time)
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 -o kslot_ab kslot_ab.cpp -lhsa-runtime64
