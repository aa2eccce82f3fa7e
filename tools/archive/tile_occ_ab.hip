// tile_occ_ab.hip -- round 4: the two-operand tile kernel (the headline's
// k_reduce_tile_lean<OpSum, float>, reduce_kernels.hpp) at 8 workgroups per CU (as
// launched) against 7 / 6 / 5, capped by an unused dynamic LDS reservation.  The
// eight-read fused combine gained from fewer loads in flight per CU
// (tools/multi_occ_ab.hip); round 2 found the opposite for the tile kernel with HIP
// event brackets around single launches (profiles/archive/r02/occupancy_ab.log);
// this re-measures it on the current kernel as back-to-back batches.
// 256 MiB: 4 rotating pairs, nt stores (keep 0, the library's policy above
// 64 MiB); 64 MiB: 16 rotating windows, sc1 stores (the library's policy).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/tile_occ_ab tools/tile_occ_ab.hip
//   tools/tile_occ_ab [rounds = 12]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

namespace mpir_hip {
uint64_t keep_bytes() { return kKeepBytes; }
uint64_t keep_for(uint64_t vbytes) { return vbytes <= keep_bytes() ? vbytes : 0; }
bool multi_uncapped() { return false; }
}
using namespace mpir_hip;

__global__ void k_fill(float *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = (float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f;
    }
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 12;
    const size_t caps[] = {0, 22 << 10, 26 << 10, 32 << 10};
    const char *names[] = {"8 / CU (as launched)", "7 / CU (22 KiB)", "6 / CU (26 KiB)", "5 / CU (32 KiB)"};
    constexpr int NV = 4;
    CK(hipFuncSetAttribute((const void *)k_reduce_tile_lean<OpSum, float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           64 << 10));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (uint64_t mib : {256ull, 64ull}) {
        const uint64_t vbytes = mib << 20;
        const int nbuf = mib == 256 ? 8 : 32;        // 4 pairs / 16 windows
        std::vector<char *> b(nbuf);
        for (auto &p : b) {
            CK(hipMalloc(&p, vbytes));
            k_fill<<<4096, 256>>>((float *)p, vbytes / 4, (uint32_t)(uintptr_t)p);
        }
        CK(hipDeviceSynchronize());
        const uint64_t keep = keep_for(vbytes);
        const unsigned grid = (unsigned)tile_groups(b[1], vbytes);
        int k = 0;
        auto run = [&](int v) {
            const int pr = k++ % (nbuf / 2);
            hipLaunchKernelGGL((k_reduce_tile_lean<OpSum, float>), dim3(grid), dim3(kThreads), caps[v], s,
                               (const char *)b[2 * pr], b[2 * pr + 1], vbytes, keep);
        };
        std::vector<double> us[NV];
        std::mt19937 rng(5);
        const int batch = mib == 256 ? 24 : 64;
        for (int r = 0; r < rounds + 1; ++r) {
            int order[NV] = {0, 1, 2, 3};
            std::shuffle(order, order + NV, rng);
            for (int v : order) {
                run(v);
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < batch; ++i) run(v);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) us[v].push_back(ms * 1e3 / batch);
            }
        }
        printf("tile kernel fp32 SUM %llu MiB per operand (%s stores), %d rounds x %d back-to-back launches\n",
               (unsigned long long)mib, keep ? "sc1" : "nt", rounds, batch);
        for (int v = 0; v < NV; ++v) {
            std::sort(us[v].begin(), us[v].end());
            const double med = us[v][us[v].size() / 2];
            printf("  %-22s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f\n", names[v], med, us[v][0],
                   3.0 * vbytes / (med * 1e-6) / 8e12);
        }
        for (auto p : b) CK(hipFree(p));
    }
    return 0;
}
