// multi_p24_occ_ab.hip -- the fused combine's P = 4 and P = 2 shapes (256-thread
// workgroups, 4 vectors per lane per operand: k_combine_multi<.., P, U = 4, TH = 256>,
// as reduce_kernels.hpp launch_combine_p launches them) at the occupancy they get
// against caps from an unused dynamic LDS reservation (5 / 4 / 3 / 2 workgroups per
// CU).  The P = 8 shape gained from fewer loads in flight (tools/multi_occ_ab.hip);
// this checks the 4- and 2-rank schedules' folds: config 4 at 4 / 2 ranks (TREE4
// fp32 over 4 x 64 MiB, TREE2 over 2 x 128 MiB) and config 5 (CHAIN4 fp16 over
// 4 x 256 MiB, CHAIN2 over 2 x 512 MiB), blocks at the staging stride (+4352 B),
// the library's store policy.  HIP events around batches of back-to-back launches
// over rotating sets; outputs compared across variants.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/multi_p24_occ_ab tools/multi_p24_occ_ab.hip
//   tools/multi_p24_occ_ab [rounds = 8]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed, int f16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = f16 ? (uint16_t)(x & 0xBFFF) : (uint16_t)((i & 1) ? ((x & 0x803F) | 0x3E00) : x);
    }
}

constexpr size_t kCaps[] = {0, 32 << 10, 40 << 10, 53 << 10, 80 << 10};
const char *kNames[] = {"as launched", "5 / CU (32 KiB)", "4 / CU (40 KiB)", "3 / CU (53 KiB)", "2 / CU (80 KiB)"};
constexpr int kNV = 5;

template <class T, int P, bool TREE>
void launch(const MultiArgs &a, size_t lds, hipStream_t s) {
    constexpr uint32_t tile = 256 * 4 * 16;
    const unsigned grid = (unsigned)((a.vbytes + tile - 1) / tile);
    hipLaunchKernelGGL((k_combine_multi<OpSum, T, P, TREE, 4, 256>), dim3(grid), dim3(256), lds, s, a);
}
template <class T, int P, bool TREE>
void allow() {
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, T, P, TREE, 4, 256>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
}

struct Case {
    const char *name;
    int p;
    uint64_t block;
    bool f16;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 8;
    allow<float, 4, true>();
    allow<float, 2, true>();
    allow<_Float16, 4, false>();
    allow<_Float16, 2, false>();
    const Case cases[] = {{"config4 TREE4 fp32 4 x 64 MiB", 4, 64ull << 20, false},
                          {"config4 TREE2 fp32 2 x 128 MiB", 2, 128ull << 20, false},
                          {"config5 CHAIN4 fp16 4 x 256 MiB", 4, 256ull << 20, true},
                          {"config5 CHAIN2 fp16 2 x 512 MiB", 2, 512ull << 20, true}};
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Case &c : cases) {
        const uint64_t stride = c.block + 4352;
        const uint64_t setbytes = c.p * stride + c.block;
        const int nsets = (int)std::max<uint64_t>(3, (3ull << 30) / setbytes + 1);
        std::vector<char *> sets(nsets);
        for (auto &p : sets) {
            CK(hipMalloc(&p, setbytes));
            k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p, c.f16);
        }
        CK(hipDeviceSynchronize());
        auto args = [&](int k) {
            MultiArgs a{};
            for (int j = 0; j < c.p; ++j) a.in[j] = sets[k % nsets] + j * stride;
            a.out = sets[k % nsets] + c.p * stride;
            a.vbytes = c.block;
            a.keep = keep_for(c.block);
            return a;
        };
        auto run = [&](int k, int v) {
            const MultiArgs a = args(k);
            if (c.f16) {
                if (c.p == 4) launch<_Float16, 4, false>(a, kCaps[v], s);
                else launch<_Float16, 2, false>(a, kCaps[v], s);
            } else {
                if (c.p == 4) launch<float, 4, true>(a, kCaps[v], s);
                else launch<float, 2, true>(a, kCaps[v], s);
            }
        };
        std::vector<char> h0(c.block), h1(c.block);
        run(0, 0);
        CK(hipMemcpyAsync(h0.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        bool same = true;
        for (int v = 1; v < kNV; ++v) {
            run(0, v);
            CK(hipMemcpyAsync(h1.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            same = same && memcmp(h0.data(), h1.data(), c.block) == 0;
        }
        std::vector<double> us[kNV];
        std::mt19937 rng(13);
        const int batch = c.block >= (256ull << 20) ? 8 : 16;
        int k = 1;
        for (int r = 0; r < rounds + 1; ++r) {
            int order[kNV];
            for (int v = 0; v < kNV; ++v) order[v] = v;
            std::shuffle(order, order + kNV, rng);
            for (int v : order) {
                run(k++, v);
                CK(hipEventRecord(e0, s));
                for (int b = 0; b < batch; ++b) run(k++, v);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) us[v].push_back(ms * 1e3 / batch);
            }
        }
        const double bytes = (c.p + 1.0) * c.block;
        printf("%s (keep %s, %d sets, %d rounds x %d launches), outputs identical across variants: %s\n", c.name,
               keep_for(c.block) ? "sc1" : "nt", nsets, rounds, batch, same ? "yes" : "NO");
        for (int v = 0; v < kNV; ++v) {
            std::sort(us[v].begin(), us[v].end());
            const double med = us[v][us[v].size() / 2];
            printf("  %-18s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f\n", kNames[v], med, us[v][0],
                   bytes / (med * 1e-6) / 8e12);
        }
        for (auto p : sets) CK(hipFree(p));
    }
    return 0;
}
