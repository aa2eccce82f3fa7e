// latency.hip -- host-side cost of one synchronous MPI_Reduce_local call.
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/latency tools/latency.hip \
//         -Lmpich-pip_amd/lib -lmpich_reduce_local -Wl,-rpath,$PWD/mpich-pip_amd/lib
// Prints per-call microseconds for: hipPointerGetAttributes, an empty launch +
// hipStreamSynchronize, MPI_Reduce_local at count 1 / 64 MiB / 256 MiB fp32.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include "mpi_reduce_local.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)
__global__ void empty() {}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);
    size_t n = 64ull << 20;  // floats = 256 MiB
    float *a, *b;
    CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 0, n * 4)); CK(hipMemset(b, 0, n * 4));
    CK(hipDeviceSynchronize());
    const int K = 200;
    hipPointerAttribute_t at;
    double t0 = now();
    for (int i = 0; i < K; ++i) CK(hipPointerGetAttributes(&at, a));
    printf("hipPointerGetAttributes        %8.2f us\n", (now() - t0) / K * 1e6);
    hipStream_t s; CK(hipStreamCreate(&s));
    t0 = now();
    for (int i = 0; i < K; ++i) { hipLaunchKernelGGL(empty, 1, 64, 0, s); CK(hipStreamSynchronize(s)); }
    printf("empty launch + StreamSynchronize %6.2f us\n", (now() - t0) / K * 1e6);
    t0 = now();
    for (int i = 0; i < K; ++i) { hipLaunchKernelGGL(empty, 1, 64, 0, s); while (hipStreamQuery(s) == hipErrorNotReady) {} }
    printf("empty launch + StreamQuery spin %7.2f us\n", (now() - t0) / K * 1e6);
    // (b) launch + hipStreamWriteValue32 into pinned host memory + host spin on it
    volatile unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    t0 = now();
    for (unsigned i = 1; i <= (unsigned)K; ++i) {
        hipLaunchKernelGGL(empty, 1, 64, 0, s);
        CK(hipStreamWriteValue32(s, (void *)flag, i, 0));
        while (*flag != i) {}
    }
    printf("empty launch + WriteValue32 spin %6.2f us\n", (now() - t0) / K * 1e6);
    // (c) event record + hipEventSynchronize
    hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    t0 = now();
    for (int i = 0; i < K; ++i) { hipLaunchKernelGGL(empty, 1, 64, 0, s); CK(hipEventRecord(ev, s)); CK(hipEventSynchronize(ev)); }
    printf("empty launch + EventSynchronize %7.2f us\n", (now() - t0) / K * 1e6);
    // (d) host cost of the launch call alone (async, drained at the end)
    t0 = now();
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(empty, 1, 64, 0, s);
    double tl = now() - t0;
    CK(hipStreamSynchronize(s));
    printf("launch call only (async)        %7.2f us\n", tl / K * 1e6);
    // (e) 256 MiB kernel via the stream API + WriteValue32 spin
    *flag = 0;
    for (unsigned i = 1; i <= 5; ++i) { MPIX_Reduce_local_stream(b, a, (int)n, MPI_FLOAT, MPI_SUM, s); CK(hipStreamWriteValue32(s, (void *)flag, i, 0)); while (*flag != i) {} }
    *flag = 0;
    t0 = now();
    for (unsigned i = 1; i <= 50; ++i) { MPIX_Reduce_local_stream(b, a, (int)n, MPI_FLOAT, MPI_SUM, s); CK(hipStreamWriteValue32(s, (void *)flag, i, 0)); while (*flag != i) {} }
    printf("256 MiB stream call + WriteValue32 spin %8.2f us/call\n", (now() - t0) / 50 * 1e6);
    t0 = now();
    for (unsigned i = 1; i <= 50; ++i) { MPIX_Reduce_local_stream(b, a, (int)n, MPI_FLOAT, MPI_SUM, s); CK(hipStreamSynchronize(s)); }
    printf("256 MiB stream call + StreamSynchronize %8.2f us/call\n", (now() - t0) / 50 * 1e6);
    size_t counts[] = {1, 16u << 20, 64u << 20};
    for (size_t c : counts) {
        for (int w = 0; w < 5; ++w) MPI_Reduce_local(b, a, (int)c, MPI_FLOAT, MPI_SUM);
        int k = c > 1000 ? 50 : K;
        t0 = now();
        for (int i = 0; i < k; ++i) {
            int rc = MPI_Reduce_local(b, a, (int)c, MPI_FLOAT, MPI_SUM);
            if (rc) { printf("rc %d\n", rc); return 1; }
        }
        double us = (now() - t0) / k * 1e6;
        printf("MPI_Reduce_local fp32 count %10zu  %9.2f us/call  %8.1f GiB/s\n", c, us, 12.0 * c / (us * 1e-6) / (1 << 30));
    }
    return 0;
}
