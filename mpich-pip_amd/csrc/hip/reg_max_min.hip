// reg_max_min.hip -- MPI_MAX / MPI_MIN kernels (opmax.c:20-55, opmin.c:19-54):
// integers and reals, no complex.
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {
struct Init {
    Init() {
#define X(E, T) reg<OpMax, T>(MPIR_HIP_OP_MAX, E); reg<OpMin, T>(MPIR_HIP_OP_MIN, E);
        FOR_INTS(X) FOR_REALS(X)
#undef X
    }
} init;
}  // namespace
