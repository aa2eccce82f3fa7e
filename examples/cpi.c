/*
 * cpi.c -- config 1 of BASELINE.json: pi by the midpoint rule on [0,1] of
 * 4/(1+x^2), rows of the rectangle sum dealt round-robin to the ranks, the
 * interval count broadcast from rank 0 and the partial sums combined with
 * MPI_Reduce(MPI_SUM, MPI_DOUBLE) at rank 0 -- the same program and the same
 * floating-point evaluation order as the reference's examples/cpi.c:18-59,
 * so `mpiexec -n 2` prints the reference's digits
 * (pi is approximately 3.1415926544231318).
 *
 *   make -C mpich-pip_amd examples
 *   mpich-pip_amd/bin/mpiexec -n 2 examples/cpi [intervals]
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "mpi.h"

static double integrand(double x)
{
    return 4.0 / (1.0 + x * x);
}

int main(int argc, char *argv[])
{
    const double pi_ref = 3.141592653589793238462643;
    char host[MPI_MAX_PROCESSOR_NAME];
    int rank, nprocs, hostlen, intervals = 0, k;
    double width, partial, local_sum = 0.0, pi = 0.0, t0 = 0.0;

    MPI_Init(&argc, &argv);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Get_processor_name(host, &hostlen);
    printf("Process %d of %d is on %s\n", rank, nprocs, host);
    fflush(stdout);

    if (rank == 0) {
        intervals = argc > 1 ? atoi(argv[1]) : 10000;
        t0 = MPI_Wtime();
    }
    MPI_Bcast(&intervals, 1, MPI_INT, 0, MPI_COMM_WORLD);

    width = 1.0 / (double) intervals;
    for (k = rank + 1; k <= intervals; k += nprocs)
        local_sum += integrand(width * ((double) k - 0.5));
    partial = width * local_sum;

    MPI_Reduce(&partial, &pi, 1, MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD);

    if (rank == 0) {
        printf("pi is approximately %.16f, Error is %.16f\n", pi, fabs(pi - pi_ref));
        printf("wall clock time = %f\n", MPI_Wtime() - t0);
        fflush(stdout);
    }
    MPI_Finalize();
    return 0;
}
