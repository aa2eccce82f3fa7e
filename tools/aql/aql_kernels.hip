// aql_kernels.hip -- device-only code object for tools/aql/aql_ab.cpp: the
// product's tile kernel body behind an unmangled name, plus an empty kernel.
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -c \
//         -O3 -std=c++17 -ffp-contract=off -Impich-pip_amd/csrc/hip -Iinclude ... -o aql_kernels.co
#include "reduce_kernels.hpp"

using namespace mpir_hip;

extern "C" __global__ __launch_bounds__(kThreads) void aql_empty() {}

extern "C" __global__ __launch_bounds__(kThreads) void aql_tile_sum_f32(TileArgs<float> a) {
    reduce_tile_body<OpSum, float>(a);
}
