/* Compile-and-link check of the public C ABI (tests/test_abi_cpu.py):
 * the headers are self-contained C99 and C++, and each entry point has the
 * exact prototype of the reference interface it replaces (mpi.h.in:1359 for
 * MPI_Reduce_local, mpir_op.h:131-144 for the op kernels).  Nothing is called. */
#include "mpi.h"
#include "mpir_hip_reduce.h"

typedef int (*reduce_local_t)(const void *, void *, int, MPI_Datatype, MPI_Op);
typedef void (*op_kernel_t)(void *, void *, int *, MPI_Datatype *);

int main(void)
{
    reduce_local_t rl[] = { MPI_Reduce_local, PMPI_Reduce_local, MPIR_Reduce_local };
    op_kernel_t ops[] = { MPIR_MAXF, MPIR_MINF, MPIR_SUM, MPIR_PROD, MPIR_LAND, MPIR_BAND, MPIR_LOR, MPIR_BOR,
                          MPIR_LXOR, MPIR_BXOR, MPIR_MINLOC, MPIR_MAXLOC, MPIR_REPLACE, MPIR_NO_OP };
    int (*ar)(const void *, void *, int, MPI_Datatype, MPI_Op, MPIX_Hip_comm, int, void *) = MPIX_Allreduce_hip;
    int (*rd)(const void *, void *, int, MPI_Datatype, MPI_Op, int, MPIX_Hip_comm, int, void *) = MPIX_Reduce_hip;
    int (*rs)(const void *, void *, const int[], MPI_Datatype, MPI_Op, MPIX_Hip_comm, int, void *) =
        MPIX_Reduce_scatter_hip;
    int (*sc)(const void *, void *, int, MPI_Datatype, MPI_Op, MPIX_Hip_comm, int, void *) = MPIX_Scan_hip;
    int (*ex)(const void *, void *, int, MPI_Datatype, MPI_Op, MPIX_Hip_comm, int, void *) = MPIX_Exscan_hip;
    int n = 0;
    unsigned i;
    for (i = 0; i < sizeof(rl) / sizeof(rl[0]); i++)
        n += rl[i] != 0;
    for (i = 0; i < sizeof(ops) / sizeof(ops[0]); i++)
        n += ops[i] != 0;
    n += (ar != 0) + (rd != 0) + (rs != 0) + (sc != 0) + (ex != 0) + (MPIR_Op_table[3] == MPIR_SUM);
    return n == 23 ? 0 : 1;
}
