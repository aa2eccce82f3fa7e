// reg_multi_logic.hip -- fused schedule combines (k_combine_multi) for the
// logical ops: LAND / LOR / LXOR over the integers (opland.c, oplor.c,
// oplxor.c) and LXOR over the reals (oplxor.c:66-67).
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg_multi<OpLand, T>(MPIR_HIP_OP_LAND, E); reg_multi<OpLor, T>(MPIR_HIP_OP_LOR, E); \
                reg_multi<OpLxor, T>(MPIR_HIP_OP_LXOR, E);
        FOR_INTS(X)
#undef X
#define X(E, T) reg_multi<OpLxor, T>(MPIR_HIP_OP_LXOR, E);
        FOR_REALS(X)
#undef X
    }
} init;
}  // namespace
