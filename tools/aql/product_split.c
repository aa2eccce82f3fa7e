/*
 * product_split.c -- the library's synchronous MPI_Reduce_local on one 16 KiB
 * tile per operand (4096 floats, SUM, device buffers: the kernel and grid
 * tools/aql/cp_latency dispatches by hand) from a plain C caller with no
 * torch: call time of 2000 unprofiled calls, then the split of 400 profiled
 * ones (MPIR_Hip_direct_last_split), medians, us.  Beside cp_latency on the
 * same box it says what of the library's doorbell -> CP start is the library's.
 *
 *   gcc -O2 -std=gnu99 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o tools/aql/product_split \
 *       tools/aql/product_split.c -Lmpich-pip_amd/lib -lmpich_reduce_local -lmpir_hip \
 *       -Wl,-rpath,$PWD/mpich-pip_amd/lib -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
 *   tools/aql/product_split [count = 4096]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "mpi_reduce_local.h"
#include "mpir_hip_reduce.h"

static int cmp(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}
static double med(double *v, int n) {
    qsort(v, n, sizeof *v, cmp);
    return v[n / 2];
}
static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(int argc, char **argv) {
    const int count = argc > 1 ? atoi(argv[1]) : 4096;
    float *a, *b;
    if (hipSetDevice(0) || hipMalloc((void **)&a, count * 4) || hipMalloc((void **)&b, count * 4) ||
        hipMemset(a, 0, count * 4) || hipMemset(b, 0, count * 4) || hipDeviceSynchronize()) {
        printf("HIP setup failed\n");
        return 2;
    }
    MPIR_Hip_direct_prepare(0);
    enum { K = 2000, KP = 400 };
    static double call[K], s0[KP], s1[KP], s2[KP], s3[KP];
    for (int i = 0; i < 50; ++i)
        if (MPI_Reduce_local(a, b, count, MPI_FLOAT, MPI_SUM)) return 3;
    for (int i = 0; i < K; ++i) {
        const double t0 = now_us();
        if (MPI_Reduce_local(a, b, count, MPI_FLOAT, MPI_SUM)) return 3;
        call[i] = now_us() - t0;
    }
    MPIR_Hip_direct_profile(1);
    int n = 0;
    for (int i = 0; i < KP; ++i) {
        uint64_t sp[4];
        if (MPI_Reduce_local(a, b, count, MPI_FLOAT, MPI_SUM)) return 3;
        MPIR_Hip_direct_last_split(sp);
        const int64_t r0 = (int64_t)sp[0], r1 = (int64_t)sp[1], r2 = (int64_t)sp[2], r3 = (int64_t)sp[3];
        if (!(0 < r0 && r0 < r3 && 0 < r2 - r1 && r2 - r1 < r3 - r0)) continue;
        s0[n] = r0 * 1e-3;
        s1[n] = (r1 - r0) * 1e-3;
        s2[n] = (r2 - r1) * 1e-3;
        s3[n] = (r3 - r2) * 1e-3;
        ++n;
    }
    MPIR_Hip_direct_profile(0);
    printf("product, count %d floats, direct state %d: call median %.2f us; profiled (%d of %d kept): "
           "host->doorbell %.2f, doorbell->CP start %.2f, CP start->end %.2f, CP end->seen %.2f\n",
           count, MPIR_Hip_direct_state(0), med(call, K), n, KP, n ? med(s0, n) : -1, n ? med(s1, n) : -1,
           n ? med(s2, n) : -1, n ? med(s3, n) : -1);
    return 0;
}
