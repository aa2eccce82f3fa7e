// reg_sum_prod.hip -- MPI_SUM / MPI_PROD kernels (opsum.c:21-76, opprod.c:21-96):
// C_INTEGER, FORTRAN_INTEGER, FLOATING_POINT (+EXTRA: char, _Float16), COMPLEX.
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg<OpSum, T>(MPIR_HIP_OP_SUM, E); reg<OpProd, T>(MPIR_HIP_OP_PROD, E);
        FOR_INTS(X) FOR_REALS(X) FOR_CPLX(X)
#undef X
    }
} init;
}  // namespace
