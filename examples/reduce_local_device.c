/*
 * reduce_local_device.c -- MPI_Reduce_local on device buffers from a plain C
 * program, as an MPI application (or an MPICH schedule) calls it: one HIP
 * runtime in the process, buffers from hipMalloc, the public C ABI
 * (include/mpi_reduce_local.h), no Python.  Also reduces a pinned host buffer
 * into a device one and two pageable host buffers, the other classes of
 * operand the library dispatches.
 *
 *   make -C mpich-pip_amd examples        # builds examples/reduce_local_device
 *   examples/reduce_local_device [count = 16777216] [calls = 50]
 *
 * Prints, per case, whether the result equals a sequential loop over the same
 * fp32 inputs bit for bit (one IEEE add per element, as the reference's
 * opsum.c:21-76), and for the device case the mean time per synchronous call.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "mpi_reduce_local.h"

#define HIPOK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* want[i] = a[i] + b[i], as volatile floats so no wider evaluation sneaks in */
static void reference_sum(const float *b, const float *a, float *want, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        volatile float s = a[i] + b[i];
        want[i] = s;
    }
}

static int same(const float *x, const float *y, size_t n)
{
    return memcmp(x, y, n * sizeof(float)) == 0;
}

int main(int argc, char **argv)
{
    const size_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : ((size_t) 1 << 24);
    const int calls = argc > 2 ? atoi(argv[2]) : 50;
    const size_t bytes = n * sizeof(float);
    float *a = malloc(bytes), *b = malloc(bytes), *want = malloc(bytes), *got = malloc(bytes);
    float *da, *db, *pin;
    uint32_t x = 12345;
    int ok = 1, rc;

    if (!a || !b || !want || !got || n > 0x7fffffff)
        return 2;
    for (size_t i = 0; i < n; i++) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        a[i] = (float) ((int32_t) x) * 0x1p-31f;
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        b[i] = (float) ((int32_t) x) * 0x1p-31f;
    }
    reference_sum(b, a, want, n);
    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);

    /* device + device: the kernel in place (direct dispatch) */
    HIPOK(hipMalloc((void **) &da, bytes));
    HIPOK(hipMalloc((void **) &db, bytes));
    HIPOK(hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(db, b, bytes, hipMemcpyHostToDevice));
    rc = MPI_Reduce_local(db, da, (int) n, MPI_FLOAT, MPI_SUM);
    HIPOK(hipMemcpy(got, da, bytes, hipMemcpyDeviceToHost));
    printf("device + device: rc %d, %s\n", rc, rc == 0 && same(got, want, n) ? "bit-exact" : "MISMATCH");
    ok &= rc == 0 && same(got, want, n);
    {
        /* the synchronous call in a loop: inout accumulates b (finite inputs) */
        double t0, t1;
        for (int i = 0; i < 5; i++)
            MPI_Reduce_local(db, da, (int) n, MPI_FLOAT, MPI_SUM);
        t0 = now_s();
        for (int i = 0; i < calls; i++)
            rc |= MPI_Reduce_local(db, da, (int) n, MPI_FLOAT, MPI_SUM);
        t1 = now_s();
        printf("device + device: %d calls, %.2f us per call, %.1f GiB/s (3 x %zu B per call)\n", calls,
               (t1 - t0) / calls * 1e6, 3.0 * bytes * calls / (t1 - t0) / (1u << 30), bytes);
    }

    /* pinned host inbuf + device inoutbuf: staged or read in place */
    HIPOK(hipHostMalloc((void **) &pin, bytes, hipHostMallocDefault));
    memcpy(pin, b, bytes);
    HIPOK(hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    rc = MPI_Reduce_local(pin, da, (int) n, MPI_FLOAT, MPI_SUM);
    HIPOK(hipMemcpy(got, da, bytes, hipMemcpyDeviceToHost));
    printf("pinned + device: rc %d, %s\n", rc, rc == 0 && same(got, want, n) ? "bit-exact" : "MISMATCH");
    ok &= rc == 0 && same(got, want, n);

    /* pageable + pageable: the host combine */
    memcpy(got, a, bytes);
    rc = MPI_Reduce_local(b, got, (int) n, MPI_FLOAT, MPI_SUM);
    printf("host + host: rc %d, %s\n", rc, rc == 0 && same(got, want, n) ? "bit-exact" : "MISMATCH");
    ok &= rc == 0 && same(got, want, n);

    HIPOK(hipHostFree(pin));
    HIPOK(hipFree(da));
    HIPOK(hipFree(db));
    free(a), free(b), free(want), free(got);
    printf("%s\n", ok ? "reduce_local_device ok" : "reduce_local_device FAILED");
    return ok ? 0 : 1;
}
