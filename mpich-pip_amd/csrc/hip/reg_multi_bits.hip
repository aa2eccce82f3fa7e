// reg_multi_bits.hip -- fused schedule combines (k_combine_multi) for the
// bitwise ops: BAND / BOR / BXOR over the integers and byte (opband.c,
// opbor.c, opbxor.c).
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg_multi<OpBand, T>(MPIR_HIP_OP_BAND, E); reg_multi<OpBor, T>(MPIR_HIP_OP_BOR, E); \
                reg_multi<OpBxor, T>(MPIR_HIP_OP_BXOR, E);
        FOR_INTS(X)
#undef X
    }
} init;
}  // namespace
