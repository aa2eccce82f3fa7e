// reg_logic.hip -- logical and bitwise kernels: LAND / LOR (opland.c, oplor.c:
// integers and _Bool as u8), LXOR (oplxor.c: also the reals, :66-67), BAND /
// BOR / BXOR (opband.c, opbor.c, opbxor.c: integers and byte).
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg<OpLand, T>(MPIR_HIP_OP_LAND, E); reg<OpLor, T>(MPIR_HIP_OP_LOR, E); \
                reg<OpLxor, T>(MPIR_HIP_OP_LXOR, E);
        FOR_INTS(X)
#undef X
#define X(E, T) reg<OpLxor, T>(MPIR_HIP_OP_LXOR, E);
        FOR_REALS(X)
#undef X
#define X(E, T) reg<OpBand, T>(MPIR_HIP_OP_BAND, E); reg<OpBor, T>(MPIR_HIP_OP_BOR, E); \
                reg<OpBxor, T>(MPIR_HIP_OP_BXOR, E);
        FOR_INTS(X)
#undef X
    }
} init;
}  // namespace
