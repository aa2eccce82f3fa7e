// occupancy_ab.hip -- does the tile kernel want fewer bytes in flight?  The
// product's lean tile body (reduce_tile<OpSum,float>, 256 MiB fp32 SUM, 4
// rotating pairs) launched with a dynamic LDS reservation it never touches, so
// that at most 8 / 6 / 5 / 4 / 3 / 2 workgroups share a CU (160 KiB LDS per CU):
// 256 / 192 / 160 / 128 / 96 / 64 KiB of loads in flight per CU.  HIP events
// per launch, variants shuffled every round; medians.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/occupancy_ab tools/occupancy_ab.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

namespace mpir_hip {
uint64_t keep_bytes() { return 0; }
uint64_t keep_for(uint64_t) { return 0; }
}
using namespace mpir_hip;

extern "C" __global__ __launch_bounds__(kThreads) void occ_tile(const char *in, char *io, uint64_t vbytes) {
    extern __shared__ char reserve[];
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    if (vbytes == 1) reserve[threadIdx.x] = 0;   // never true: keeps the reservation referenced
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    const int rounds = argc > 2 ? atoi(argv[2]) : 30;
    const size_t bytes = mib << 20;
    const int NP = 4;
    std::vector<float *> a(NP), b(NP);
    std::vector<float> h(bytes / 4);
    uint32_t x = 0x5EED;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = (float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f; }
    for (int i = 0; i < NP; ++i) {
        CK(hipMalloc(&a[i], bytes));
        CK(hipMalloc(&b[i], bytes));
        CK(hipMemcpy(a[i], h.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(b[i], h.data(), bytes, hipMemcpyHostToDevice));
    }
    // per-CU workgroup limit -> LDS bytes per workgroup (160 KiB per CU)
    const int limits[] = {8, 6, 5, 4, 3, 2};
    const int nv = sizeof(limits) / sizeof(limits[0]);
    std::vector<std::vector<float>> dur(nv);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const unsigned grid = (unsigned)(bytes / kTileBytes);
    std::vector<int> order(nv);
    for (int i = 0; i < nv; ++i) order[i] = i;
    uint32_t rs = 12345;
    int k = 0;
    for (int r = -3; r < rounds; ++r) {
        for (int i = nv - 1; i > 0; --i) {
            rs = rs * 1664525u + 1013904223u;
            std::swap(order[i], order[(rs >> 8) % (i + 1)]);
        }
        for (int vi : order) {
            const size_t lds = limits[vi] >= 8 ? 0 : (160u * 1024u) / limits[vi] - 64;
            const int p = k++ % NP;
            CK(hipEventRecord(e0, st));
            hipLaunchKernelGGL(occ_tile, dim3(grid), dim3(kThreads), lds, st, (const char *)b[p], (char *)a[p], (uint64_t)bytes);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) dur[vi].push_back(ms * 1e3f);
        }
    }
    printf("%zu MiB fp32 SUM tile kernel, %d rounds, HIP-event medians\n", mib, rounds);
    for (int i = 0; i < nv; ++i) {
        std::sort(dur[i].begin(), dur[i].end());
        const float med = dur[i][dur[i].size() / 2];
        printf("  <= %d WG/CU (%3d KiB in flight/CU)  median %7.2f us  p10 %7.2f  frac %.4f\n", limits[i],
               limits[i] * 32, med, dur[i][dur[i].size() / 10], 3.0 * bytes / (med * 1e-6) / 8e12);
    }
    return 0;
}
