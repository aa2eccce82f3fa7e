/*
 * mock_preload_app.c -- run with LD_PRELOAD=libmpich_reduce_local_preload.so
 * against tests/progs/mock_installed_mpi.c.  Host buffers, no GPU.
 */
#include <stdio.h>

typedef int MPI_Datatype;
typedef int MPI_Op;
typedef void (MPI_User_function) (void *, void *, int *, MPI_Datatype *);
int MPI_Reduce_local(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op);
int MPI_Op_create(MPI_User_function * fn, int commute, MPI_Op * op);
int mock_allreduce(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op);
void mock_counts(int *pmpi, int *mpir, int *ops);

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)
#define MPI_SUM ((MPI_Op) 0x58000003)
#define MPI_BYTE ((MPI_Datatype) 0x4c00010d)
#define MPI_INT ((MPI_Datatype) 0x4c000405)

static void plus(void *in, void *inout, int *len, MPI_Datatype * dt)
{
    (void) dt;
    for (int i = 0; i < *len; i++)
        ((int *) inout)[i] += ((int *) in)[i];
}

int main(void)
{
    int in[2] = { 1, 2 }, io[2] = { 10, 20 }, pmpi, mpir, ops;
    MPI_Op op;
    CHECK(MPI_Op_create(plus, 1, &op) == 0);           /* libmpi's own store */
    mock_counts(&pmpi, &mpir, &ops);
    CHECK(ops == 1);
    /* user op: the shim hands it on to libmpi's PMPI_Reduce_local */
    CHECK(MPI_Reduce_local(in, io, 2, MPI_INT, op) == 0 && io[0] == 11 && io[1] == 22);
    mock_counts(&pmpi, &mpir, &ops);
    CHECK(pmpi == 1 && mpir == 1);
    /* builtin op: the shim's own validation answers (BYTE + SUM -> MPI_ERR_OP
     * class 9), libmpi is not called */
    CHECK((MPI_Reduce_local(in, io, 2, MPI_BYTE, MPI_SUM) & 0x7f) == 9);
    mock_counts(&pmpi, &mpir, &ops);
    CHECK(pmpi == 1 && mpir == 1);
    /* libmpi's schedules are out of the shim's reach (hidden MPIR_Reduce_local) */
    CHECK(mock_allreduce(in, io, 2, MPI_INT, op) == 0);
    mock_counts(&pmpi, &mpir, &ops);
    CHECK(pmpi == 1 && mpir == 2);
    puts("preload ok");
    return 0;
}
