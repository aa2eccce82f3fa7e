// reg_multi.hip -- fused schedule combines (k_combine_multi) for the ops the
// reduction collectives are built on (configs 4-5): SUM / PROD / MAX / MIN over
// the 32/64-bit integers and the reals, plus complex SUM.  reg_multi_small /
// _logic / _bits.hip register every other pair of 16 bytes or less; the 32-byte
// types (long double _Complex, MPI_LONG_DOUBLE_INT) and TREE folds of n > 8
// take k_combine_any (one pass, any n) through MPIR_Hip_combine.
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg_multi<OpSum, T>(MPIR_HIP_OP_SUM, E); reg_multi<OpProd, T>(MPIR_HIP_OP_PROD, E); \
                reg_multi<OpMax, T>(MPIR_HIP_OP_MAX, E); reg_multi<OpMin, T>(MPIR_HIP_OP_MIN, E);
        X(MPIR_HIP_I32, int32_t) X(MPIR_HIP_U32, uint32_t) X(MPIR_HIP_I64, int64_t) X(MPIR_HIP_U64, uint64_t)
        X(MPIR_HIP_F16, f16) X(MPIR_HIP_F32, float) X(MPIR_HIP_F64, double)
#undef X
        reg_multi<OpSum, cf32>(MPIR_HIP_OP_SUM, MPIR_HIP_CF32);
        reg_multi<OpSum, cf64>(MPIR_HIP_OP_SUM, MPIR_HIP_CF64);
    }
} init;
}  // namespace
