/*
 * host_small_latency.c -- ns per MPI_Reduce_local / MPIR_Reduce_local on host
 * buffers at small counts (fp64 SUM), beside the oracle's restatement of the
 * reference path (oracle/op_oracle.c: MPI_Reduce_local's validation, the
 * datatype switch and the opsum.c:21-76 loop) and the bare loop itself.
 * VERDICT r3 item 1c; DESIGN.md §Dispatch cites the table it prints.
 *
 * Not product code: the oracle is loaded here only as the comparison.
 *
 *   gcc -O2 -std=gnu99 -Iinclude -o tools/host_small_latency tools/host_small_latency.c \
 *       -Lmpich-pip_amd/lib -lmpich_reduce_local -Wl,-rpath,$PWD/mpich-pip_amd/lib -ldl
 *   tools/host_small_latency            # GPU runtime never started
 *   tools/host_small_latency gpu        # HIP started first: every call classifies its pointers
 *
 * Prints one line per count: median over 15 rounds of the mean ns per call
 * (20000 calls a round; the three callers alternate round by round).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mpi_reduce_local.h"

typedef int (*reduce_fn)(const void *, void *, int, int, int);

static double now_ns(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e9 + ts.tv_nsec;
}

static int cmp(const void *a, const void *b)
{
    double x = *(const double *) a, y = *(const double *) b;
    return x < y ? -1 : x > y;
}

/* the loop of opsum.c for MPI_DOUBLE, compiled here (gcc -O2, like MPICH) */
static __attribute__((noinline)) int bare_loop(const void *in, void *io, int n, int dt, int op)
{
    const double *a = in;
    double *b = io;
    (void) dt;
    (void) op;
    for (int i = 0; i < n; i++)
        b[i] = b[i] + a[i];
    return 0;
}

static int lib_mpi(const void *in, void *io, int n, int dt, int op)
{
    return MPI_Reduce_local(in, io, n, (MPI_Datatype) dt, (MPI_Op) op);
}

static int lib_mpir(const void *in, void *io, int n, int dt, int op)
{
    return MPIR_Reduce_local(in, io, n, (MPI_Datatype) dt, (MPI_Op) op);
}

int main(int argc, char **argv)
{
    static const int counts[] = { 1, 8, 64, 1024 };
    const int rounds = 15, calls = 20000;
    const char *oracle_path = "oracle/liboracle.so";
    void *oh = dlopen(oracle_path, RTLD_NOW);
    reduce_fn orc = oh ? (reduce_fn) dlsym(oh, "oracle_reduce_local") : NULL;
    if (!orc) {
        fprintf(stderr, "%s: %s (run from the repo root after make -C oracle)\n", oracle_path, dlerror());
        return 1;
    }
    if (argc > 1 && !strcmp(argv[1], "gpu")) {
        void *hh = dlopen("libamdhip64.so", RTLD_NOW);
        int (*get_count)(int *) = hh ? (int (*)(int *)) dlsym(hh, "hipGetDeviceCount") : NULL;
        int n = 0;
        if (!get_count || get_count(&n) != 0 || n < 1) {
            fprintf(stderr, "gpu mode: no HIP device\n");
            return 1;
        }
        printf("# HIP started (%d device(s)): every call classifies both pointers\n", n);
    } else {
        printf("# GPU runtime not started by this process\n");
    }
    printf("# fp64 MPI_SUM, host buffers, ns per call (median of %d rounds x %d calls)\n", rounds, calls);
    printf("%6s %12s %14s %16s %10s\n", "count", "bare loop", "oracle MPI_", "MPI_Reduce_local", "MPIR_");
    for (size_t c = 0; c < sizeof counts / sizeof counts[0]; c++) {
        const int n = counts[c];
        double *a = aligned_alloc(64, 64 * ((n * 8 + 63) / 64));
        double *b = aligned_alloc(64, 64 * ((n * 8 + 63) / 64));
        reduce_fn fns[4] = { bare_loop, orc, lib_mpi, lib_mpir };
        double res[4][15];
        for (int i = 0; i < n; i++) {
            a[i] = 1e-300 * (i + 1);
            b[i] = 0.5 * i;
        }
        for (int f = 0; f < 4; f++)
            for (int k = 0; k < 2000; k++)
                if (fns[f](a, b, n, (int) MPI_DOUBLE, (int) MPI_SUM)) {
                    fprintf(stderr, "call %d failed\n", f);
                    return 1;
                }
        for (int r = 0; r < rounds; r++)
            for (int f = 0; f < 4; f++) {
                const double t0 = now_ns();
                for (int k = 0; k < calls; k++)
                    fns[f](a, b, n, (int) MPI_DOUBLE, (int) MPI_SUM);
                res[f][r] = (now_ns() - t0) / calls;
            }
        for (int f = 0; f < 4; f++)
            qsort(res[f], rounds, sizeof(double), cmp);
        printf("%6d %12.1f %14.1f %16.1f %10.1f\n", n, res[0][rounds / 2], res[1][rounds / 2], res[2][rounds / 2],
               res[3][rounds / 2]);
        free(a);
        free(b);
    }
    return 0;
}
