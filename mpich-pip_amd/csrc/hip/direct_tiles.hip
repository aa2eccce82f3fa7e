// direct_tiles.hip -- device-only code object lib/libmpir_hip_tiles.hsaco for
// the direct AQL dispatch of synchronous calls (direct_dispatch.hip).
//
// One extern "C" kernel per (op, element class) of the hot matrix -- SUM / PROD
// over the integer, real and complex classes, MAX / MIN over the integer and
// real classes -- each the body of k_reduce_tile_lean<Op, T>
// (reduce_kernels.hpp) under a plain name the host looks up:
// mpir_tile_<op>_<element enum>.  Four explicit kernel arguments (in, io,
// vbytes, keep) and nothing else: no hidden arguments (no gridDim), so a bare
// AQL packet launches it.
#include "kernel_table.hpp"

using namespace mpir_hip;

#define MPIR_DIRECT_TILE(OPN, OP, E, T)                                                                   \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_tile_##OPN##_##E(const char *in, char *io, \
                                                                                 uint64_t vbytes, uint64_t keep) { \
        const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;                                          \
        if (base >= vbytes) return;                                                                       \
        reduce_tile<OP, T>(in, io, base, vbytes, keep);                                                   \
    }

#define X(E, T) MPIR_DIRECT_TILE(SUM, OpSum, E, T) MPIR_DIRECT_TILE(PROD, OpProd, E, T)
FOR_INTS(X) FOR_REALS(X) FOR_CPLX(X)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(MAX, OpMax, E, T) MPIR_DIRECT_TILE(MIN, OpMin, E, T)
FOR_INTS(X) FOR_REALS(X)
#undef X
