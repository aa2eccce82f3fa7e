// multi_ab.hip -- A/B of workgroup shapes for the fused multi-operand combine
// (k_combine_multi, reduce_kernels.hpp) at the collectives' block sizes:
//   config 4: TREE8 fp32, 8 x 32 MiB -> 32 MiB   (256 MiB allreduce / 8 ranks)
//   config 5: CHAIN8 fp16, 8 x 128 MiB -> 128 MiB (1 GiB reduce-scatter / 8 ranks)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/multi_ab tools/multi_ab.hip
// Variants: threads per WG (256/512/1024), vectors per lane per operand (U),
// cache policy (nt / default), and the product launcher.  Interleaved rounds,
// median of per-launch HIP-event times.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

using namespace mpir_hip;

template <class Op, class T, int P, bool TREE, int U, int TH, int POL>
__global__ __launch_bounds__(TH) void k_multi_x(MultiArgs a) {
    constexpr uint32_t tile = TH * U * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= a.vbytes) return;
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    u32x4 x[P][U];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u)
            x[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r, (u * TH + (int)threadIdx.x) * 16, 0, POL);
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
            res.e[k] = fold_fast<Op, T, P, TREE>(v);
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, res), ro, (u * TH + (int)threadIdx.x) * 16, 0, POL);
    }
}

template <class Op, class T, int P, bool TREE, int U, int TH, int POL>
hipError_t launch_x(const void *const *ins, void *out, uint64_t count, hipStream_t s) {
    MultiArgs a{};
    for (int j = 0; j < P; ++j) a.in[j] = static_cast<const char *>(ins[j]);
    a.out = static_cast<char *>(out);
    a.vbytes = count * sizeof(T);   // buffers are 256 B-aligned and sizes multiples of 16
    constexpr uint32_t tile = TH * U * 16;
    hipLaunchKernelGGL((k_multi_x<Op, T, P, TREE, U, TH, POL>), dim3((unsigned)((a.vbytes + tile - 1) / tile)), dim3(TH), 0, s, a);
    return hipGetLastError();
}

struct MVar {
    std::string name;
    size_t esz;
    hipError_t (*fn)(const void *const *, void *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

static void run_set(const char *title, std::vector<MVar> &vs, size_t bytes, int rounds) {
    const int P = 8, NS = 2;
    std::vector<char *> ins(P * NS), outs(NS);
    for (auto &p : ins) { CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 0x3c, bytes)); }
    for (auto &p : outs) CK(hipMalloc(&p, bytes));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int slot = 0;
    for (int r = -2; r < rounds; ++r)
        for (auto &v : vs) {
            const int s = slot++ % NS;
            const void *ptr[P];
            for (int j = 0; j < P; ++j) ptr[j] = ins[s * P + j];
            CK(hipEventRecord(e0, st));
            CK(v.fn(ptr, outs[s], bytes / v.esz, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) v.ms.push_back(ms);
        }
    printf("%s: 8 x %zu MiB -> 1, %d interleaved rounds\n", title, bytes >> 20, rounds);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2];
        const double gbs = 9.0 * bytes / (med * 1e-3) / 1e9;
        printf("  %-34s median %8.2f us  %7.0f GB/s  frac %.3f\n", v.name.c_str(), med * 1e3, gbs, gbs / 8000.0);
    }
    for (auto p : ins) CK(hipFree(p));
    for (auto p : outs) CK(hipFree(p));
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    std::vector<MVar> t8 = {
        {"product", 4, &launch_combine_p<OpSum, float, 8, true>, {}},
        {"U1 T256 nt", 4, &launch_x<OpSum, float, 8, true, 1, 256, 2>, {}},
        {"U2 T256 nt", 4, &launch_x<OpSum, float, 8, true, 2, 256, 2>, {}},
        {"U1 T512 nt", 4, &launch_x<OpSum, float, 8, true, 1, 512, 2>, {}},
        {"U1 T1024 nt", 4, &launch_x<OpSum, float, 8, true, 1, 1024, 2>, {}},
        {"U2 T512 nt", 4, &launch_x<OpSum, float, 8, true, 2, 512, 2>, {}},
        {"U1 T256 default", 4, &launch_x<OpSum, float, 8, true, 1, 256, 0>, {}},
        {"U2 T256 default", 4, &launch_x<OpSum, float, 8, true, 2, 256, 0>, {}},
        {"U1 T256 nt-load sc-store", 4, &launch_x<OpSum, float, 8, true, 1, 256, 3>, {}},
    };
    run_set("config 4 TREE8 SUM fp32", t8, 32u << 20, rounds);
    for (auto &v : t8) v.ms.clear();
    run_set("TREE8 SUM fp32 (256 MiB operands)", t8, 256u << 20, rounds);
    std::vector<MVar> c8 = {
        {"product", 2, &launch_combine_p<OpSum, f16, 8, false>, {}},
        {"U1 T256 nt", 2, &launch_x<OpSum, f16, 8, false, 1, 256, 2>, {}},
        {"U2 T256 nt", 2, &launch_x<OpSum, f16, 8, false, 2, 256, 2>, {}},
        {"U1 T512 nt", 2, &launch_x<OpSum, f16, 8, false, 1, 512, 2>, {}},
        {"U1 T1024 nt", 2, &launch_x<OpSum, f16, 8, false, 1, 1024, 2>, {}},
        {"U1 T256 default", 2, &launch_x<OpSum, f16, 8, false, 1, 256, 0>, {}},
    };
    run_set("config 5 CHAIN8 SUM fp16", c8, 128u << 20, rounds);
    return 0;
}
