// host_overhead.cpp -- host-side cost of a synchronous MPI_Reduce_local, by
// piece, at count 4 on device buffers (direct dispatch).  Medians over N calls.
//   hipcc -O2 -std=c++17 -Iinclude tools/host_overhead.cpp -o tools/host_overhead \
//         -Lmpich-pip_amd/lib -lmpich_reduce_local -lmpir_hip -Wl,-rpath,$PWD/mpich-pip_amd/lib
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <time.h>
#include <algorithm>
#include <vector>

#include "mpi_reduce_local.h"
#include "mpir_hip_reduce.h"

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
template <class F>
static double med(int n, F f) {
    std::vector<double> v(n);
    for (int i = 0; i < n; ++i) {
        const double t0 = now_us();
        f();
        v[i] = now_us() - t0;
    }
    std::sort(v.begin(), v.end());
    return v[n / 2];
}

int main() {
    float *a, *b;
    hipMalloc(&a, 4096);
    hipMalloc(&b, 4096);
    hipMemset(a, 0, 4096);
    hipMemset(b, 0, 4096);
    hipDeviceSynchronize();
    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);
    for (int i = 0; i < 1000; ++i) MPI_Reduce_local(b, a, 4, MPI_FLOAT, MPI_SUM);
    const int N = 20000;
    printf("MPI_Reduce_local count 4 (direct)   %6.3f us\n", med(N, [&] { MPI_Reduce_local(b, a, 4, MPI_FLOAT, MPI_SUM); }));
    printf("MPIR_Hip_reduce count 4             %6.3f us\n",
           med(N, [&] { MPIR_Hip_reduce(b, a, 4, MPIR_HIP_OP_SUM, MPIR_HIP_F32, nullptr, 1); }));
    hipPointerAttribute_t at;
    printf("hipPointerGetAttributes             %6.3f us\n", med(N, [&] { hipPointerGetAttributes(&at, a); }));
    printf("hipStreamQuery(null)                %6.3f us\n", med(N, [&] { (void)hipStreamQuery(nullptr); }));
    int d;
    printf("hipGetDevice                        %6.3f us\n", med(N, [&] { hipGetDevice(&d); }));
    uint64_t sp[4];
    MPIR_Hip_direct_profile(1);
    std::vector<double> s0, s1, s3;
    for (int i = 0; i < 2000; ++i) {
        MPI_Reduce_local(b, a, 4, MPI_FLOAT, MPI_SUM);
        MPIR_Hip_direct_last_split(sp);
        s0.push_back(sp[0] * 1e-3);
        s1.push_back(sp[1] * 1e-3);
        s3.push_back(sp[3] * 1e-3);
    }
    MPIR_Hip_direct_profile(0);
    std::sort(s0.begin(), s0.end());
    std::sort(s1.begin(), s1.end());
    std::sort(s3.begin(), s3.end());
    printf("inside the dispatch: doorbell %.3f  CP start %.3f  host sees %.3f us (medians)\n", s0[1000], s1[1000],
           s3[1000]);
    return 0;
}
