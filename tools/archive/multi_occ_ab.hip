// multi_occ_ab.hip -- the product's fused 8-operand kernel (k_combine_multi<.., P = 8,
// U = 1, TH = 1024>, reduce_kernels.hpp) launched as the library launches it and
// with a dynamic LDS reservation that leaves room for one 1024-thread workgroup
// per CU instead of two (half the loads in flight), and 512-thread shapes at one
// or two workgroups per CU.  tools/fused_write_ab.hip
// (XOR folds, SWEEP=1) found the eight-reads-one-write mix 1-2.5 points faster
// that way.  Cases: config 4's TREE8 fp32 SUM over 8 x 32 MiB blocks and config
// 5's CHAIN8 fp16 SUM over 8 x 128 MiB, operands at the collective's skewed
// staging stride (+4352 B), the library's store policy (keep_for: sc1 for
// outputs <= 64 MiB, else nt).  HIP events around batches of back-to-back
// launches over rotating operand sets (> Infinity Cache), variants alternated
// in shuffled order; outputs compared bit for bit between the two launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/multi_occ_ab tools/multi_occ_ab.hip
//   tools/multi_occ_ab [rounds = 10]
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
uint64_t keep_bytes() { return getenv("KEEP_MB") ? strtoull(getenv("KEEP_MB"), 0, 10) << 20 : kKeepBytes; }
uint64_t keep_for(uint64_t vbytes) { return vbytes <= keep_bytes() ? vbytes : 0; }
bool multi_uncapped() { return false; }
}
using namespace mpir_hip;

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed, int f16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        // fp16: magnitude < 2 (bit 14 clear); fp32 halves: exponent bits kept moderate
        p[i] = f16 ? (uint16_t)(x & 0xBFFF) : (uint16_t)((i & 1) ? ((x & 0x803F) | 0x3E00) : x);
    }
}

// a variant: workgroup size, vectors per lane per operand, dynamic LDS (caps the
// workgroups per CU; 0 = as the library launches it)
struct Var {
    const char *name;
    int th, u;
    size_t lds;
};
const Var kVars[] = {{"1024 x 1, 2 / CU (library)", 1024, 1, 0},
                     {"1024 x 1, 1 / CU", 1024, 1, 96 << 10},
                     {"512 x 2, 1 / CU", 512, 2, 96 << 10},
                     {"512 x 1, 1 / CU", 512, 1, 96 << 10},
                     {"512 x 1, 2 / CU", 512, 1, 64 << 10},
                     {"512 x 2, 2 / CU", 512, 2, 64 << 10}};
constexpr int kNV = sizeof(kVars) / sizeof(kVars[0]);

template <class T, bool TREE, int U, int TH>
void launch_one(const MultiArgs &a, size_t lds, hipStream_t s) {
    const unsigned grid = (unsigned)((a.vbytes + TH * U * 16 - 1) / (TH * U * 16));
    hipLaunchKernelGGL((k_combine_multi<OpSum, T, 8, TREE, U, TH>), dim3(grid), dim3(TH), lds, s, a);
}
template <class T, bool TREE, int U, int TH>
void allow_lds() {
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, T, 8, TREE, U, TH>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
}
template <class T, bool TREE>
void launch(const MultiArgs &a, const Var &v, hipStream_t s) {
    if (v.th == 1024) launch_one<T, TREE, 1, 1024>(a, v.lds, s);
    else if (v.u == 2) launch_one<T, TREE, 2, 512>(a, v.lds, s);
    else launch_one<T, TREE, 1, 512>(a, v.lds, s);
}
template <class T, bool TREE>
void allow_all() {
    allow_lds<T, TREE, 1, 1024>();
    allow_lds<T, TREE, 2, 512>();
    allow_lds<T, TREE, 1, 512>();
}

struct Case {
    const char *name;
    uint64_t block;
    bool f16;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    allow_all<float, true>();
    allow_all<_Float16, false>();
    const Case cases[] = {{"config4 TREE8 fp32 8 x 32 MiB", 32ull << 20, false},
                          {"config5 CHAIN8 fp16 8 x 128 MiB", 128ull << 20, true}};
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Case &c : cases) {
        const uint64_t stride = c.block + 4352;
        const uint64_t setbytes = 8 * stride + c.block;
        const int nsets = (int)std::max<uint64_t>(3, (3ull << 30) / setbytes + 1);
        std::vector<char *> sets(nsets);
        for (auto &p : sets) {
            CK(hipMalloc(&p, setbytes));
            k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p, c.f16);
        }
        CK(hipDeviceSynchronize());
        auto args = [&](int k) {
            MultiArgs a{};
            for (int j = 0; j < 8; ++j) a.in[j] = sets[k % nsets] + j * stride;
            a.out = sets[k % nsets] + 8 * stride;
            a.vbytes = c.block;
            a.keep = keep_for(c.block);
            return a;
        };
        auto run = [&](int k, int v) {
            if (c.f16) launch<_Float16, false>(args(k), kVars[v], s);
            else launch<float, true>(args(k), kVars[v], s);
        };
        // bit-exact: every variant's output equals the library launch's
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
        std::mt19937 rng(11);
        const int batch = 20;
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
        const double bytes = 9.0 * c.block;
        printf("%s (keep %s, %d sets, %d rounds x %d launches), outputs identical across variants: %s\n", c.name,
               keep_for(c.block) ? "sc1" : "nt", nsets, rounds, batch, same ? "yes" : "NO");
        for (int v = 0; v < kNV; ++v) {
            std::sort(us[v].begin(), us[v].end());
            const double med = us[v][us[v].size() / 2];
            printf("  %-28s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f\n", kVars[v].name, med, us[v][0],
                   bytes / (med * 1e-6) / 8e12);
        }
        for (auto p : sets) CK(hipFree(p));
    }
    return 0;
}
