// direct_tiles.hip -- device-only code object lib/libmpir_hip_tiles.hsaco for
// the direct AQL dispatch of synchronous calls (direct_dispatch.hip).
//
// Five extern "C" kernels per (op, element class) whose launcher is
// launch_reduce (reg<Op, T> in the reg_*.hip units: every op on the integer,
// real, complex, pair and x87 classes; not the 32-byte classes or REPLACE) --
// one per kind of plan_reduce's launch plan (reduce_kernels.hpp), under plain
// names the host looks up:
//   mpir_tile_<op>_<elem>    k_reduce_tile_lean's body (LeanArgs, 32 B):
//                            16 B-aligned operands of 16 B multiples;
//   mpir_tilex_<op>_<elem>   k_reduce_tile's body (TileArgs, 80 B): equal
//                            alignment mod 16, head / tail elements by
//                            workgroup 0;
//   mpir_tiles_<op>_<elem>   k_reduce_shift's body (ShiftArgs, 96 B): unequal
//                            alignment mod 16, two tiles or more;
//   mpir_elems_<op>_<elem>   k_reduce_elems<NATURAL = true / false> (ElemsArgs,
//   mpir_elemsu_<op>_<elem>  32 B, the grid stride an argument): the rest.
// None reads a hidden argument (no gridDim), so a bare AQL packet launches it.
#include "kernel_table.hpp"

using namespace mpir_hip;

#define MPIR_DIRECT_TILE(OPN, OP, E, T)                                                                   \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_tile_##OPN##_##E(const char *in, char *io, \
                                                                                 uint64_t vbytes, uint64_t keep) { \
        reduce_tile<OP, T>(in, io, blockIdx.x, vbytes, keep);                                             \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_tilex_##OPN##_##E(TileArgs<T> a) {       \
        reduce_tile_body<OP, T>(a);                                                                       \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_tiles_##OPN##_##E(ShiftArgs<T> a) {      \
        reduce_shift_body<OP, T>(a);                                                                      \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_elems_##OPN##_##E(                       \
        const char *in, char *io, uint64_t n, uint64_t stride) {                                          \
        reduce_elems<OP, T, true>(in, io, n, stride);                                                     \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_elemsu_##OPN##_##E(                      \
        const char *in, char *io, uint64_t n, uint64_t stride) {                                          \
        reduce_elems<OP, T, false>(in, io, n, stride);                                                    \
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
