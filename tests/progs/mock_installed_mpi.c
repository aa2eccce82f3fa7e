/*
 * mock_installed_mpi.c -- an installed MPICH 3.3 libmpi as INTEGRATION.md
 * Option 2 finds it: built with -fvisibility=hidden, exporting only its public
 * API (mpi.h.in:13).  Its own PMPI_Reduce_local (with MPI_Reduce_local a weak
 * alias, reduce_local.c:11-20), its own MPI_Op_create, and a schedule
 * (mock_allreduce) that calls its internal, hidden MPIR_Reduce_local.
 * Counters show which implementation ran each call.
 */
typedef int MPI_Datatype;
typedef int MPI_Op;
typedef void (MPI_User_function) (void *, void *, int *, MPI_Datatype *);

static int pmpi_calls, mpir_calls, ops_created;
static MPI_User_function *user_fns[16];

int MPIR_Reduce_local(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op)
{
    mpir_calls++;
    if ((((unsigned) op) >> 30) == 2) {            /* a direct user op of this libmpi */
        MPI_User_function *f = user_fns[(unsigned) op & 0xf];
        f((void *) in, inout, &count, &dt);
    }
    return 0;
}

__attribute__((visibility("default")))
int PMPI_Reduce_local(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op)
{
    pmpi_calls++;
    return MPIR_Reduce_local(in, inout, count, dt, op);
}

__attribute__((visibility("default")))
int MPI_Reduce_local(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op)
    __attribute__((weak, alias("PMPI_Reduce_local")));

__attribute__((visibility("default")))
int MPI_Op_create(MPI_User_function * fn, int commute, MPI_Op * op)
{
    (void) commute;
    user_fns[ops_created] = fn;
    *op = (MPI_Op) (0x98000000u | (unsigned) ops_created++);
    return 0;
}

__attribute__((visibility("default")))
int mock_allreduce(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op)
{
    return MPIR_Reduce_local(in, inout, count, dt, op);
}

__attribute__((visibility("default")))
void mock_counts(int *pmpi, int *mpir, int *ops)
{
    *pmpi = pmpi_calls;
    *mpir = mpir_calls;
    *ops = ops_created;
}
