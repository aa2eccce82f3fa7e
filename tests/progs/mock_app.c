/*
 * mock_app.c -- an application linked against tests/progs/mock_libmpi.c's
 * libmockmpi.so (the drop-in compiled into a hidden-visibility "libmpi").
 * Host buffers only: runs without a GPU.
 */
#include <stdio.h>

#include "mpi_reduce_local.h"

int mock_sched_reduce(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op, MPI_Op * user_handle);
int mock_op_refcount(MPI_Op op);
void mock_err_counts(int *created, int *returned);
int mock_table_ok(void);

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

static void twice_plus(void *in, void *inout, int *len, MPI_Datatype * dt)
{
    int *a = (int *) in, *b = (int *) inout;
    (void) dt;
    for (int i = 0; i < *len; i++)
        b[i] = 2 * b[i] + a[i];
}

int main(void)
{
    int in[3] = { 1, 2, 3 }, io[3] = { 5, 6, 7 }, created = 0, returned = 0, cls = -1, rc;
    MPI_Op op, handle;

    CHECK(MPI_Op_create(twice_plus, 0, &op) == MPI_SUCCESS);
    handle = op;
    /* the schedule holds the op, the application frees it, the reduce still runs */
    CHECK(mock_sched_reduce(in, io, 3, MPI_INT, op, &handle) == MPI_SUCCESS);
    CHECK(handle == MPI_OP_NULL);
    CHECK(io[0] == 11 && io[1] == 14 && io[2] == 17);
    CHECK(mock_op_refcount(op) == 0);                  /* released by the schedule */
    /* a freed op is refused by the public entry point ... */
    rc = MPI_Reduce_local(in, io, 3, MPI_INT, op);
    CHECK(MPI_Error_class(rc, &cls) == MPI_SUCCESS && cls == MPI_ERR_OP);
    /* ... and the failure went through libmpi's (strong) error routines */
    mock_err_counts(&created, &returned);
    CHECK((rc & 0x00100000) != 0 && created >= 2 && returned == 1);
    /* builtin ops: the schedules' MPIR_Op_table is the drop-in's */
    CHECK(mock_table_ok());
    CHECK(mock_sched_reduce(in, io, 0, MPI_INT, MPI_SUM, NULL) == MPI_SUCCESS);
    puts("mock libmpi ok");
    return 0;
}
