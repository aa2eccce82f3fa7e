// fold_policy.hip -- the fused CHAIN8 fp16 fold (config 5's combine) under each
// cache policy of its eight loads and its store.  The library loads and stores
// `nt`; round 2 swept the store policy only.  Same body as the product's
// (combine_multi_tile: 1024 threads, one 16 B vector per lane per operand, issue
// gap every 4 loads, 96 KiB LDS reservation = one workgroup per CU).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/archive/fold_policy tools/archive/fold_policy.hip
//   tools/archive/fold_policy [rounds = 11]
//
// 8 x 128 MiB at the collective's staging stride (block + 4352 B), three operand
// sets rotated (3.4 GiB: nothing survives in the 256 MB Infinity Cache), HIP
// events over batches of 20 back-to-back launches, variants shuffled per round,
// the first round dropped; every variant's output compared bit for bit with the
// library policy's on the same set.  Policy bits: 1 sc0, 2 nt, 16 sc1.
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

template <int LP, int SP>
__global__ __launch_bounds__(1024) void k_fold_pol(MultiArgs a) {
    constexpr uint32_t tile = 1024 * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= a.vbytes) return;
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * 1024 + (t & 63) * 16;
    u32x4 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, wb, 0, LP);
        if ((j + 1) % 4 == 0 && j + 1 < 8) issue_gap();
    }
    Pack16<f16> pk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) pk[j] = __builtin_bit_cast(Pack16<f16>, x[j]);
    Pack16<f16> res;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        f16 e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = pk[j].e[k];
        res.e[k] = fold_fast<OpSum, f16, 8, false>(e);
    }
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, res), ro, wb, 0, SP);
}

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = (uint16_t)(x & 0xBFFF);
    }
}

struct Var {
    const char *name;
    void (*fn)(MultiArgs);
};
#define V(LP, SP, N) Var{N, [](MultiArgs a) { \
    hipLaunchKernelGGL((k_fold_pol<LP, SP>), dim3((unsigned)(a.vbytes / 16384)), dim3(1024), 96 << 10, 0, a); }}
#define ATTR(LP, SP) CK(hipFuncSetAttribute((const void *)k_fold_pol<LP, SP>, \
    hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10))

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 11;
    ATTR(2, 2); ATTR(0, 2); ATTR(1, 2); ATTR(16, 2); ATTR(18, 2); ATTR(2, 0); ATTR(0, 0); ATTR(2, 16);
    const Var vars[] = {V(2, 2, "load nt,      store nt (library)"), V(0, 2, "load default, store nt"),
                        V(1, 2, "load sc0,     store nt"),           V(16, 2, "load sc1,     store nt"),
                        V(18, 2, "load nt|sc1,  store nt"),          V(2, 0, "load nt,      store default"),
                        V(0, 0, "load default, store default"),      V(2, 16, "load nt,      store sc1")};
    constexpr int NV = sizeof(vars) / sizeof(vars[0]);
    const uint64_t block = 128ull << 20, stride = block + 4352, setbytes = 8 * stride + block;
    const int nsets = 3;
    std::vector<char *> sets(nsets);
    for (auto &p : sets) {
        CK(hipMalloc(&p, setbytes));
        k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p);
    }
    CK(hipDeviceSynchronize());
    auto args = [&](int k) {
        MultiArgs a{};
        char *b = sets[k % nsets];
        for (int j = 0; j < 8; ++j) a.in[j] = b + j * stride;
        a.out = b + 8 * stride;
        a.vbytes = block;
        return a;
    };
    // outputs: every variant against the library policy on set 0
    std::vector<char> want(block), got(block);
    int bad = 0;
    for (int v = 0; v < NV; ++v) {
        vars[v].fn(args(0));
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(v ? got.data() : want.data(), args(0).out, block, hipMemcpyDeviceToHost));
        if (v && memcmp(got.data(), want.data(), block) != 0) {
            printf("OUTPUT MISMATCH: %s\n", vars[v].name);
            ++bad;
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> us[NV];
    std::mt19937 rng(7);
    int k = 0;
    const int batch = 20;
    for (int r = 0; r < rounds; ++r) {
        int order[NV];
        for (int v = 0; v < NV; ++v) order[v] = v;
        std::shuffle(order, order + NV, rng);
        for (int v : order) {
            vars[v].fn(args(k++));
            CK(hipEventRecord(e0, 0));
            for (int b = 0; b < batch; ++b) vars[v].fn(args(k++));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) us[v].push_back(ms * 1e3 / batch);
        }
    }
    printf("CHAIN8 fp16 8 x 128 MiB, 1 workgroup / CU, %d rounds x %d back-to-back launches (first round dropped); "
           "outputs %s\n", rounds, batch, bad ? "DIFFER" : "identical");
    for (int v = 0; v < NV; ++v) {
        std::sort(us[v].begin(), us[v].end());
        const double med = us[v][us[v].size() / 2];
        printf("  %-32s median %8.2f us (min %8.2f, max %8.2f)  frac of 8 TB/s %.4f\n", vars[v].name, med, us[v].front(),
               us[v].back(), 9.0 * block / (med * 1e-6) / 8e12);
    }
    for (auto p : sets) CK(hipFree(p));
    return bad ? 1 : 0;
}
