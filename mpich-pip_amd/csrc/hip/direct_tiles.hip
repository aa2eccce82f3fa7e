// direct_tiles.hip -- device-only code object lib/libmpir_hip_tiles.hsaco for
// the direct AQL dispatch of synchronous calls (direct_dispatch.hip).
//
// Two extern "C" kernels per (op, element class) whose launcher is the tile
// family (reg<Op, T> in the reg_*.hip units: every op on the integer, real,
// complex, pair and x87 classes except the 32-byte ones and REPLACE), under
// plain names the host looks up:
//   mpir_tile_<op>_<element enum>   the body of k_reduce_tile_lean<Op, T>:
//                                   four arguments (in, io, vbytes, keep), for
//                                   16 B-aligned operands of 16 B multiples;
//   mpir_tilex_<op>_<element enum>  the body of k_reduce_tile<Op, T>: one
//                                   TileArgs<T> (80 bytes), the head / tail
//                                   elements of a ragged or 16 B-misaligned
//                                   (but equally misaligned) call combined by
//                                   workgroup 0.
// Neither reads a hidden argument (no gridDim), so a bare AQL packet launches it.
#include "kernel_table.hpp"

using namespace mpir_hip;

#define MPIR_DIRECT_TILE(OPN, OP, E, T)                                                                   \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_tile_##OPN##_##E(const char *in, char *io, \
                                                                                 uint64_t vbytes, uint64_t keep) { \
        const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;                                          \
        if (base >= vbytes) return;                                                                       \
        reduce_tile<OP, T>(in, io, base, vbytes, keep);                                                   \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_tilex_##OPN##_##E(TileArgs<T> a) {       \
        reduce_tile_body<OP, T>(a);                                                                       \
    }

// the (op, class) matrix of reg_sum_prod / reg_max_min / reg_logic / reg_pairs_x87
#define X(E, T) MPIR_DIRECT_TILE(SUM, OpSum, E, T) MPIR_DIRECT_TILE(PROD, OpProd, E, T)
FOR_INTS(X) FOR_REALS(X) FOR_CPLX(X) X(MPIR_HIP_F80, x80)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(MAX, OpMax, E, T) MPIR_DIRECT_TILE(MIN, OpMin, E, T)
FOR_INTS(X) FOR_REALS(X) X(MPIR_HIP_F80, x80)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(LAND, OpLand, E, T) MPIR_DIRECT_TILE(LOR, OpLor, E, T) \
                MPIR_DIRECT_TILE(BAND, OpBand, E, T) MPIR_DIRECT_TILE(BOR, OpBor, E, T) \
                MPIR_DIRECT_TILE(BXOR, OpBxor, E, T)
FOR_INTS(X)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(LXOR, OpLxor, E, T)
FOR_INTS(X) FOR_REALS(X) X(MPIR_HIP_F80, x80)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(MAXLOC, OpMaxloc, E, T) MPIR_DIRECT_TILE(MINLOC, OpMinloc, E, T)
FOR_PAIRS(X)
#undef X
