// multi_gapcap_ab.hip -- round 4: the fused combine's load issue gap, re-tuned under
// the LDS caps the library now launches it with (reduce_kernels.hpp multi_lds_cap:
// P = 8 one 1024-thread workgroup per CU, P = 4 three 256-thread workgroups).  The
// kernel below is k_combine_multi's vector path with the gap (a one-instruction
// s_nop after every GAP loads; the library uses GAP = 4 for P = 4 and 8) as a
// template parameter; GAP = 0 issues the loads back to back.  Cases as in
// tools/multi_cap_ab.py: TREE8 fp32 8 x 32 MiB, CHAIN8 fp16 8 x 128 MiB, TREE4 fp32
// 4 x 64 MiB, CHAIN4 fp16 4 x 256 MiB, staging stride +4352 B, the library's store
// policy.  HIP events around batches of back-to-back launches over rotating sets,
// variants shuffled each round; outputs compared across variants.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/multi_gapcap_ab tools/multi_gapcap_ab.hip
//   tools/multi_gapcap_ab [rounds = 8]
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

template <class T, int P, bool TREE, int U, int TH, int GAP>
__global__ __launch_bounds__(TH) void k_gap(MultiArgs a) {
    constexpr uint32_t tile = TH * U * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= a.vbytes) return;
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (U * 1024) + (t & 63) * 16;
    u32x4 x[P][U];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < P; ++j) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
            x[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r, wb + u * 1024, 0, kCachePolicyNT);
            if (GAP > 0 && (u * P + j + 1) % GAP == 0 && u * P + j + 1 < U * P) issue_gap();
        }
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        Pack16<T> pk[P];
#pragma unroll
        for (int j = 0; j < P; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, x[j][u]);
        Pack16<T> res;
#pragma unroll
        for (int k = 0; k < (int)(16 / sizeof(T)); ++k) {
            T v[P];
#pragma unroll
            for (int j = 0; j < P; ++j) v[j] = pk[j].e[k];
            res.e[k] = fold_fast<OpSum, T, P, TREE>(v);
        }
        store16(__builtin_bit_cast(u32x4, res), ro, wb + u * 1024, keep_tile(base, a.vbytes, a.keep));
    }
}

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed, int f16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = f16 ? (uint16_t)(x & 0xBFFF) : (uint16_t)((i & 1) ? ((x & 0x803F) | 0x3E00) : x);
    }
}

typedef void (*kfn)(MultiArgs);
struct Var {
    const char *name;
    kfn k;
};
template <class T, int P, bool TREE, int U, int TH, int GAP>
Var var(const char *name) {
    const kfn k = k_gap<T, P, TREE, U, TH, GAP>;
    CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    return {name, k};
}

struct Case {
    const char *name;
    int p;
    uint64_t block;
    bool f16;
    unsigned th, u;
    size_t lds;
    std::vector<Var> vars;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 8;
    std::vector<Case> cases;
    cases.push_back({"TREE8 fp32 8 x 32 MiB", 8, 32ull << 20, false, 1024, 1, 96 << 10,
                     {var<float, 8, true, 1, 1024, 4>("gap 4 (library)"), var<float, 8, true, 1, 1024, 0>("no gap"),
                      var<float, 8, true, 1, 1024, 1>("gap 1"), var<float, 8, true, 1, 1024, 2>("gap 2")}});
    cases.push_back({"CHAIN8 fp16 8 x 128 MiB", 8, 128ull << 20, true, 1024, 1, 96 << 10,
                     {var<_Float16, 8, false, 1, 1024, 4>("gap 4 (library)"), var<_Float16, 8, false, 1, 1024, 0>("no gap"),
                      var<_Float16, 8, false, 1, 1024, 1>("gap 1"), var<_Float16, 8, false, 1, 1024, 2>("gap 2")}});
    cases.push_back({"TREE4 fp32 4 x 64 MiB", 4, 64ull << 20, false, 256, 4, 53 << 10,
                     {var<float, 4, true, 4, 256, 4>("gap 4 (library)"), var<float, 4, true, 4, 256, 0>("no gap"),
                      var<float, 4, true, 4, 256, 2>("gap 2"), var<float, 4, true, 4, 256, 8>("gap 8")}});
    cases.push_back({"CHAIN4 fp16 4 x 256 MiB", 4, 256ull << 20, true, 256, 4, 53 << 10,
                     {var<_Float16, 4, false, 4, 256, 4>("gap 4 (library)"), var<_Float16, 4, false, 4, 256, 0>("no gap"),
                      var<_Float16, 4, false, 4, 256, 2>("gap 2"), var<_Float16, 4, false, 4, 256, 8>("gap 8")}});
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
        const unsigned grid = (unsigned)(c.block / (c.th * c.u * 16));
        const int nv = (int)c.vars.size();
        auto run = [&](int k, int v) {
            hipLaunchKernelGGL(c.vars[v].k, dim3(grid), dim3(c.th), c.lds, s, args(k));
        };
        std::vector<char> h0(c.block), h1(c.block);
        run(0, 0);
        CK(hipMemcpyAsync(h0.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        bool same = true;
        for (int v = 1; v < nv; ++v) {
            run(0, v);
            CK(hipMemcpyAsync(h1.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            same = same && memcmp(h0.data(), h1.data(), c.block) == 0;
        }
        std::vector<std::vector<double>> us(nv);
        std::mt19937 rng(17);
        const int batch = c.block >= (256ull << 20) ? 8 : 16;
        int k = 1;
        std::vector<int> order(nv);
        for (int r = 0; r < rounds + 1; ++r) {
            for (int v = 0; v < nv; ++v) order[v] = v;
            std::shuffle(order.begin(), order.end(), rng);
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
        printf("%s (cap %zu KiB, keep %s, %d rounds x %d launches), outputs identical across variants: %s\n", c.name,
               c.lds >> 10, keep_for(c.block) ? "sc1" : "nt", rounds, batch, same ? "yes" : "NO");
        for (int v = 0; v < nv; ++v) {
            std::sort(us[v].begin(), us[v].end());
            const double med = us[v][us[v].size() / 2];
            printf("  %-16s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f\n", c.vars[v].name, med, us[v][0],
                   bytes / (med * 1e-6) / 8e12);
        }
        for (auto p : sets) CK(hipFree(p));
    }
    return 0;
}
