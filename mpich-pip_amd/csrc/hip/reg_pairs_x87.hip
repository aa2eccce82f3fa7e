// reg_pairs_x87.hip -- MAXLOC / MINLOC on the pair types (opmaxloc.c:79,
// opminloc.c:78), the long double rows computed as x87 in software
// (FLOATING_POINT: SUM, PROD, MAX, MIN, LXOR; its _Complex: SUM, PROD;
// MPI_LONG_DOUBLE_INT: MAXLOC, MINLOC), and REPLACE (a byte copy for every
// class, MPIR_Localcopy of a basic type).
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg<OpMaxloc, T>(MPIR_HIP_OP_MAXLOC, E); reg<OpMinloc, T>(MPIR_HIP_OP_MINLOC, E);
        FOR_PAIRS(X)
#undef X
        reg<OpSum, x80>(MPIR_HIP_OP_SUM, MPIR_HIP_F80);
        reg<OpProd, x80>(MPIR_HIP_OP_PROD, MPIR_HIP_F80);
        reg<OpMax, x80>(MPIR_HIP_OP_MAX, MPIR_HIP_F80);
        reg<OpMin, x80>(MPIR_HIP_OP_MIN, MPIR_HIP_F80);
        reg<OpLxor, x80>(MPIR_HIP_OP_LXOR, MPIR_HIP_F80);
        reg_wide<OpSum, cx80>(MPIR_HIP_OP_SUM, MPIR_HIP_CF80);
        reg_wide<OpProd, cx80, 1>(MPIR_HIP_OP_PROD, MPIR_HIP_CF80);
        reg_wide<OpMaxloc, pldint>(MPIR_HIP_OP_MAXLOC, MPIR_HIP_PLDOUBLEINT);
        reg_wide<OpMinloc, pldint>(MPIR_HIP_OP_MINLOC, MPIR_HIP_PLDOUBLEINT);
        for (int e = 1; e < MPIR_HIP_NELEMS; ++e) reg<OpReplace, uint8_t>(MPIR_HIP_OP_REPLACE, e);
    }
} init;
}  // namespace
