// reg_multi_small.hip -- fused schedule combines (k_combine_multi) for the
// pairs outside reg_multi.hip's main set: SUM / PROD / MAX / MIN over the 8-
// and 16-bit integers, complex PROD, MAXLOC / MINLOC on the 8- and 16-byte
// pair types, and the x87 long double ops.  Without these the pairs ran the
// element-granular k_combine_any (0.08-0.54 of the HBM peak at n = 8,
// profiles/archive/r01s3_multi_sweep.log).
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg_multi<OpSum, T>(MPIR_HIP_OP_SUM, E); reg_multi<OpProd, T>(MPIR_HIP_OP_PROD, E); \
                reg_multi<OpMax, T>(MPIR_HIP_OP_MAX, E); reg_multi<OpMin, T>(MPIR_HIP_OP_MIN, E);
        X(MPIR_HIP_I8, int8_t) X(MPIR_HIP_U8, uint8_t) X(MPIR_HIP_I16, int16_t) X(MPIR_HIP_U16, uint16_t)
        X(MPIR_HIP_F80, x80)
#undef X
        reg_multi<OpLxor, x80>(MPIR_HIP_OP_LXOR, MPIR_HIP_F80);
        reg_multi<OpProd, cf32>(MPIR_HIP_OP_PROD, MPIR_HIP_CF32);
        reg_multi<OpProd, cf64>(MPIR_HIP_OP_PROD, MPIR_HIP_CF64);
#define X(E, T) reg_multi<OpMaxloc, T>(MPIR_HIP_OP_MAXLOC, E); reg_multi<OpMinloc, T>(MPIR_HIP_OP_MINLOC, E);
        FOR_PAIRS(X)
#undef X
    }
} init;
}  // namespace
