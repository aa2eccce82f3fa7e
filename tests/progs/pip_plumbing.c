/*
 * pip_plumbing.c -- test program for the runtime subset (tests/test_pip_runtime*.py).
 * Run under mpich-pip_amd/bin/mpiexec; prints "key value..." lines that the
 * Python side checks against simulations of the reference schedules.
 *
 *   argv[1] = "cpu": user-op reductions only (no GPU needed)
 *   argv[1] = "gpu": also builtin MPI_SUM reductions (HIP MPIR_Reduce_local)
 *   argv[1] = "mismatch": collectives called with counts that differ across
 *             ranks; every rank prints the error classes it got, then shows
 *             the world still works (no rank is left waiting)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpi.h"

/* non-associative, non-commutative fingerprint op: inout = 31*in + inout */
static void fp_op(void *in, void *inout, int *len, MPI_Datatype *dt)
{
    uint32_t *a = in, *b = inout;
    int i;
    (void) dt;
    for (i = 0; i < *len; i++)
        b[i] = 31u * a[i] + b[i];
}

static uint32_t val(int rank, int i)
{
    return (uint32_t) (rank * 1000003u + (uint32_t) i * 7919u + 17u);
}

int main(int argc, char **argv)
{
    int rank, size, i, root, flag, len;
    const int gpu = argc > 1 && !strcmp(argv[1], "gpu");
    char name[MPI_MAX_PROCESSOR_NAME];
    MPI_Op ops[2];

    MPI_Initialized(&flag);
    if (flag)
        return 3;
    if (MPI_Init(&argc, &argv))
        return 4;
    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Get_processor_name(name, &len);
    printf("hello %d %d %d\n", rank, size, len > 0);
    fflush(stdout);

    if (argc > 1 && !strcmp(argv[1], "mismatch")) {
        /* root 0 sends 2 MiB + 3 bytes (three chunks) where the others expect
         * 1 MiB: longer than the receive buffer; then 100 bytes where the
         * others expect 200: shorter; then a user-op MPI_Reduce where rank 1
         * contributes 5 elements and everyone else (the root too) 3 */
        const int big = (2 << 20) + 3, small = 1 << 20;
        unsigned char *buf = calloc(big, 1);
        uint32_t s5[5] = {1, 2, 3, 4, 5}, r5[5] = {0, 0, 0, 0, 0};
        int c[3], x = rank == 0 ? 77 : 0;
        MPI_Op op;
        for (i = 0; i < big; i++)
            buf[i] = rank == 0 ? (unsigned char) (i * 13) : 0;
        MPI_Error_class(MPI_Bcast(buf, rank == 0 ? big : small, MPI_BYTE, 0, MPI_COMM_WORLD), &c[0]);
        for (i = 0; i < small && (buf[i] == (unsigned char) (i * 13)); i++)
            ;
        flag = i == small && (rank == 0 || buf[small] == 0);        /* the excess was dropped */
        MPI_Error_class(MPI_Bcast(buf, rank == 0 ? 100 : 200, MPI_BYTE, 0, MPI_COMM_WORLD), &c[1]);
        MPI_Op_create(fp_op, 1, &op);
        MPI_Error_class(MPI_Reduce(s5, r5, rank == 1 ? 5 : 3, MPI_UNSIGNED, op, 0, MPI_COMM_WORLD), &c[2]);
        MPI_Op_free(&op);
        MPI_Barrier(MPI_COMM_WORLD);
        MPI_Bcast(&x, 1, MPI_INT, 0, MPI_COMM_WORLD);
        printf("mismatch %d %d %d %d %d %d\n", rank, c[0], c[1], c[2], flag, x);
        free(buf);
        MPI_Finalize();
        return 0;
    }

    /* Bcast: 1 int and a 3 MiB + 5 byte buffer (multi-chunk) from every root */
    for (root = 0; root < size; root++) {
        int x = rank == root ? 4242 + root : -1;
        size_t nb = (3u << 20) + 5, bad = 0;
        unsigned char *big = malloc(nb);
        MPI_Bcast(&x, 1, MPI_INT, root, MPI_COMM_WORLD);
        for (i = 0; i < (int) nb; i++)
            big[i] = rank == root ? (unsigned char) (i * 7 + root) : 0;
        MPI_Bcast(big, (int) nb, MPI_BYTE, root, MPI_COMM_WORLD);
        for (i = 0; i < (int) nb; i++)
            bad += big[i] != (unsigned char) (i * 7 + root);
        printf("bcast %d %d %d %zu\n", rank, root, x, bad);
        free(big);
    }
    fflush(stdout);

    for (i = 0; i < 5; i++)
        MPI_Barrier(MPI_COMM_WORLD);

    /* user-op MPI_Reduce (host function), non-commutative and commutative,
     * every root; counts 3 (binomial) */
    MPI_Op_create(fp_op, 0, &ops[0]);
    MPI_Op_create(fp_op, 1, &ops[1]);
    for (int c = 0; c < 2; c++)
        for (root = 0; root < size; root++) {
            uint32_t s[3], r[3] = {0, 0, 0};
            int rc;
            for (i = 0; i < 3; i++)
                s[i] = val(rank, i);
            rc = MPI_Reduce(s, r, 3, MPI_UNSIGNED, ops[c], root, MPI_COMM_WORLD);
            if (rank == root)
                printf("ureduce %d %d %d %u %u %u\n", c, root, rc, r[0], r[1], r[2]);
        }
    fflush(stdout);

    /* error classes */
    {
        int x = 0, y = 0, c[4];
        MPI_Error_class(MPI_Reduce(&x, &y, 1, MPI_INT, MPI_SUM, size, MPI_COMM_WORLD), &c[0]);
        MPI_Error_class(MPI_Bcast(&x, 1, MPI_INT, 0, (MPI_Comm) 0x44000007), &c[1]);
        MPI_Error_class(MPI_Reduce(&x, &y, -1, MPI_INT, MPI_SUM, 0, MPI_COMM_WORLD), &c[2]);
        MPI_Error_class(MPI_Reduce(&x, &y, 1, MPI_BYTE, MPI_SUM, 0, MPI_COMM_WORLD), &c[3]);
        printf("errs %d %d %d %d\n", c[0], c[1], c[2], c[3]);
    }

    if (gpu) {
        /* builtin MPI_SUM on doubles: count 1 (binomial) and 4099 (> 2048 B:
         * reduce-scatter + gather), every root; inputs are deterministic */
        const int counts[2] = {1, 4099};
        for (int k = 0; k < 2; k++)
            for (root = 0; root < size; root++) {
                int n = counts[k], rc;
                double *s = malloc(sizeof(double) * n), *r = calloc(n, sizeof(double));
                uint64_t h = 1469598103934665603ull;
                for (i = 0; i < n; i++)
                    s[i] = (double) ((rank + 1) * 0.1) + (double) i * 1e-3 + 1.0 / (3.0 + rank + i);
                rc = MPI_Reduce(s, r, n, MPI_DOUBLE, MPI_SUM, root, MPI_COMM_WORLD);
                if (rank == root) {
                    const unsigned char *b = (const unsigned char *) r;
                    for (i = 0; i < n * 8; i++)
                        h = (h ^ b[i]) * 1099511628211ull;
                    printf("dreduce %d %d %d %016llx %.17g\n", n, root, rc, (unsigned long long) h, r[0]);
                }
                free(s);
                free(r);
            }
    }
    fflush(stdout);
    MPI_Op_free(&ops[0]);
    MPI_Op_free(&ops[1]);
    MPI_Finalize();
    MPI_Finalized(&flag);
    return flag ? 0 : 5;
}
