// multi_gap_ab.hip -- A/B of the fused 8-operand combine (config 4's TREE8 fp32
// SUM and config 5's CHAIN8 fp16 SUM, 32 MiB blocks) over workgroup size,
// vectors per lane and the load issue gap.  Run under
//   rocprofv3 --kernel-trace -- tools/multi_gap_ab [MiB=32] [rounds=30]
// and read the kernel durations from the trace (event brackets include the
// host submit gap).  Variant order is shuffled every round; two operand sets
// alternate (> Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/multi_gap_ab tools/multi_gap_ab.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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

// GAP: a gap after every GAP loads (0 = none)
template <class T, bool TREE, int P, int U, int TH, int GAP>
__global__ __launch_bounds__(TH) void k_mx(MultiArgs a) {
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
            if constexpr (GAP > 0) {
                if ((u * P + j + 1) % GAP == 0 && u * P + j + 1 < U * P) issue_gap();
            }
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

// issue order test: odd workgroups load the eight operands in reverse order
template <class T, bool TREE, int TH>
__global__ __launch_bounds__(TH) void k_rev(MultiArgs a) {
    constexpr int P = 8;
    constexpr uint32_t tile = TH * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= a.vbytes) return;
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    const int t = (int)threadIdx.x;
    const int off = (t >> 6) * 1024 + (t & 63) * 16;
    u32x4 x[P];
    if (blockIdx.x & 1) {
#pragma unroll
        for (int j = P - 1; j >= 0; --j) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
            x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kCachePolicyNT);
        }
    } else {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
            x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kCachePolicyNT);
        }
    }
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
    Pack16<T> pk[P];
#pragma unroll
    for (int j = 0; j < P; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, x[j]);
    Pack16<T> res;
#pragma unroll
    for (int k = 0; k < (int)(16 / sizeof(T)); ++k) {
        T v[P];
#pragma unroll
        for (int j = 0; j < P; ++j) v[j] = pk[j].e[k];
        res.e[k] = fold_fast<OpSum, T, P, TREE>(v);
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, res), ro, off, 0, kCachePolicyNT);
}
template <class T, bool TREE, int TH>
hipError_t launch_rev(const void *const *ins, void *out, uint64_t count, hipStream_t s) {
    MultiArgs a{};
    for (int j = 0; j < 8; ++j) a.in[j] = static_cast<const char *>(ins[j]);
    a.out = static_cast<char *>(out);
    a.vbytes = count * sizeof(T);
    hipLaunchKernelGGL((k_rev<T, TREE, TH>), dim3((unsigned)((a.vbytes + TH * 16 - 1) / (TH * 16))), dim3(TH), 0, s, a);
    return hipGetLastError();
}


// software-pipelined: each workgroup folds NT consecutive tiles (U = 1), the
// eight loads of tile t+1 issued before tile t's combine and store, so stores
// leave the workgroup between loads instead of in one burst at its end
template <class T, bool TREE, int TH, int NT>
__global__ __launch_bounds__(TH) void k_pipe(MultiArgs a) {
    constexpr int P = 8;
    constexpr uint32_t tile = TH * 16;
    const int t = (int)threadIdx.x;
    const int off = (t >> 6) * 1024 + (t & 63) * 16;
    const uint64_t base0 = (uint64_t)blockIdx.x * tile * NT;
    u32x4 x[2][P];
    auto load = [&](int buf, uint64_t base) {
        const uint64_t left = base < a.vbytes ? a.vbytes - base : 0;
        const int nrec = (int)(left < tile ? left : tile);
#pragma unroll
        for (int j = 0; j < P; ++j) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
            x[buf][j] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kCachePolicyNT);
            if ((j + 1) % 4 == 0 && j + 1 < P) issue_gap();
        }
    };
    if (base0 >= a.vbytes) return;
    load(0, base0);
#pragma unroll
    for (int k = 0; k < NT; ++k) {
        const uint64_t base = base0 + (uint64_t)k * tile;
        if (k + 1 < NT) load((k + 1) & 1, base + tile);
        if (base >= a.vbytes) break;
        const uint64_t left = a.vbytes - base;
        const int nrec = (int)(left < tile ? left : tile);
        Pack16<T> pk[P];
#pragma unroll
        for (int j = 0; j < P; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, x[k & 1][j]);
        Pack16<T> res;
#pragma unroll
        for (int e = 0; e < (int)(16 / sizeof(T)); ++e) {
            T v[P];
#pragma unroll
            for (int j = 0; j < P; ++j) v[j] = pk[j].e[e];
            res.e[e] = fold_fast<OpSum, T, P, TREE>(v);
        }
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, res), ro, off, 0, kCachePolicyNT);
    }
}
template <class T, bool TREE, int TH, int NT>
hipError_t launch_pipe(const void *const *ins, void *out, uint64_t count, hipStream_t s) {
    MultiArgs a{};
    for (int j = 0; j < 8; ++j) a.in[j] = static_cast<const char *>(ins[j]);
    a.out = static_cast<char *>(out);
    a.vbytes = count * sizeof(T);
    constexpr uint64_t span = (uint64_t)TH * 16 * NT;
    hipLaunchKernelGGL((k_pipe<T, TREE, TH, NT>), dim3((unsigned)((a.vbytes + span - 1) / span)), dim3(TH), 0, s, a);
    return hipGetLastError();
}

typedef hipError_t (*mfn)(const void *const *, void *, uint64_t, hipStream_t);

template <class T, bool TREE, int U, int TH, int GAP, int P = 8>
hipError_t launch_mx(const void *const *ins, void *out, uint64_t count, hipStream_t s) {
    MultiArgs a{};
    for (int j = 0; j < P; ++j) a.in[j] = static_cast<const char *>(ins[j]);
    a.out = static_cast<char *>(out);
    a.vbytes = count * sizeof(T);
    a.keep = keep_bytes();
    constexpr uint32_t tile = TH * U * 16;
    hipLaunchKernelGGL((k_mx<T, TREE, P, U, TH, GAP>), dim3((unsigned)((a.vbytes + tile - 1) / tile)), dim3(TH), 0, s, a);
    return hipGetLastError();
}

struct Var { std::string name; size_t esz; mfn fn; };

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 32;
    int rounds = argc > 2 ? atoi(argv[2]) : 30;
    size_t bytes = mib << 20;
    // NSETS (env, default 2): operand sets rotated; with NSETS x block > 256 MB
    // no output stays in the Infinity Cache from one use to the next
    const int P = 8, NS = getenv("NSETS") ? std::max(2, atoi(getenv("NSETS"))) : 2;
    std::vector<char *> ins(P * NS), outs(NS);
    std::vector<uint32_t> h(bytes / 4);
    uint32_t x = 0x5EED;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = 0x3c003c00u | (x & 0x03ff03ffu); }  // finite fp16 / fp32
    // operand j of set s at base + (s*P + j) * (bytes + skew): skew 0 puts the
    // eight operands at power-of-two strides (like a staging area of equal blocks)
    const size_t skew = argc > 3 ? strtoull(argv[3], 0, 10) : 0;
    char *big;
    CK(hipMalloc(&big, (bytes + skew) * P * NS + 4096));
    for (int k = 0; k < P * NS; ++k) {
        ins[k] = big + (size_t)k * (bytes + skew);
        CK(hipMemcpy(ins[k], h.data(), bytes, hipMemcpyHostToDevice));
    }
    for (auto &p : outs) CK(hipMalloc(&p, bytes));
    // P = 2 / 4 shapes (the first P operands of a set); algorithmic bytes (P+1) x block
    // P = 8 (config 4 block at N = 8): longer contiguous runs per operand and wave
    const bool half = argc > 4 && atoi(argv[4]) == 16;
    std::vector<Var> vs;
    if (!half) vs = {
        {"TREE8 f32 product (U1 T1024)", 4, &launch_combine_p<OpSum, float, 8, true>},
        {"TREE8 f32 U1 T256 gap4", 4, &launch_mx<float, true, 1, 256, 4>},
        {"TREE8 f32 U1 T512 gap4", 4, &launch_mx<float, true, 1, 512, 4>},
        {"TREE8 f32 U1 T1024 gap0", 4, &launch_mx<float, true, 1, 1024, 0>},
        {"TREE8 f32 U1 T1024 gap2", 4, &launch_mx<float, true, 1, 1024, 2>},
        {"TREE8 f32 U1 T1024 gap8", 4, &launch_mx<float, true, 1, 1024, 8>},
        {"TREE8 f32 U2 T512 gap4", 4, &launch_mx<float, true, 2, 512, 4>},
        {"TREE8 f32 U2 T256 gap4", 4, &launch_mx<float, true, 2, 256, 4>},
        {"TREE8 f32 U4 T256 gap4", 4, &launch_mx<float, true, 4, 256, 4>},
        {"TREE8 f32 U4 T256 gap8", 4, &launch_mx<float, true, 4, 256, 8>},
        {"TREE8 f32 U4 T128 gap4", 4, &launch_mx<float, true, 4, 128, 4>},
        {"TREE8 f32 U2 T1024 gap4", 4, &launch_mx<float, true, 2, 1024, 4>},
        {"TREE8 f32 pipe2 T256", 4, &launch_pipe<float, true, 256, 2>},
        {"TREE8 f32 pipe4 T256", 4, &launch_pipe<float, true, 256, 4>},
        {"TREE8 f32 pipe2 T512", 4, &launch_pipe<float, true, 512, 2>},
        {"TREE8 f32 pipe4 T512", 4, &launch_pipe<float, true, 512, 4>},
        {"TREE8 f32 pipe8 T256", 4, &launch_pipe<float, true, 256, 8>},
    };
    else vs = {
        {"CHAIN8 f16 product (U1 T1024)", 2, &launch_combine_p<OpSum, _Float16, 8, false>},
        // the same bytes through the product's fused kernel with other element work:
        // u32 BXOR (no floating point) and f32 SUM -- is the 8-stream pattern or the
        // fp16 chain the limit?
        {"CHAIN8 u32 BXOR product kernel", 4, &launch_combine_p<OpBxor, uint32_t, 8, false>},
        {"CHAIN8 f32 SUM product kernel", 4, &launch_combine_p<OpSum, float, 8, false>},
        {"TREE8 f16 SUM product kernel", 2, &launch_combine_p<OpSum, _Float16, 8, true>},
        {"CHAIN8 f16 U1 T256 gap4", 2, &launch_mx<_Float16, false, 1, 256, 4>},
        {"CHAIN8 f16 U1 T512 gap4", 2, &launch_mx<_Float16, false, 1, 512, 4>},
        {"CHAIN8 f16 U1 T1024 gap0", 2, &launch_mx<_Float16, false, 1, 1024, 0>},
        {"CHAIN8 f16 U1 T1024 gap8", 2, &launch_mx<_Float16, false, 1, 1024, 8>},
        {"CHAIN8 f16 U2 T512 gap4", 2, &launch_mx<_Float16, false, 2, 512, 4>},
        {"CHAIN8 f16 pipe2 T256", 2, &launch_pipe<_Float16, false, 256, 2>},
        {"CHAIN8 f16 pipe4 T256", 2, &launch_pipe<_Float16, false, 256, 4>},
        {"CHAIN8 f16 pipe4 T512", 2, &launch_pipe<_Float16, false, 512, 4>},
    };
    std::vector<std::vector<float>> dur(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::vector<int> order(vs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    uint32_t rs = 777;
    int slot = 0;
    for (int r = -2; r < rounds; ++r) {
        for (size_t i = order.size() - 1; i > 0; --i) {
            rs = rs * 1664525u + 1013904223u;
            std::swap(order[i], order[(rs >> 8) % (i + 1)]);
        }
        for (int vi : order) {
            const int s = slot++ % NS;
            const void *ptr[P];
            for (int j = 0; j < P; ++j) ptr[j] = ins[s * P + j];
            CK(hipEventRecord(e0, st));
            CK(vs[vi].fn(ptr, outs[s], bytes / vs[vi].esz, st));
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) dur[vi].push_back(ms * 1e3f);
        }
    }
    printf("8 x %zu MiB -> 1 (operand stride %zu B), %d rounds; HIP-event medians (the rocprofv3 trace has the kernel times)\n",
           mib, bytes + skew, rounds);
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(dur[i].begin(), dur[i].end());
        const float med = dur[i][dur[i].size() / 2];
        printf("  %-34s median %7.2f us  p10 %7.2f  frac %.4f\n", vs[i].name.c_str(), med, dur[i][dur[i].size() / 10],
               9.0 * bytes / (med * 1e-6) / 8e12);
    }
    // BATCH=1: each variant over `rounds` back-to-back launches between two
    // events (sets rotating): the steady state, with any write-back an sc1
    // store policy defers paid inside the batch
    if (getenv("BATCH")) {
        for (int pass = 0; pass < 2; ++pass)
            for (size_t vi = 0; vi < vs.size(); ++vi) {
                auto launch = [&](int k) {
                    const int s = k % NS;
                    const void *ptr[P];
                    for (int j = 0; j < P; ++j) ptr[j] = ins[s * P + j];
                    CK(vs[vi].fn(ptr, outs[s], bytes / vs[vi].esz, st));
                };
                for (int w = 0; w < 3; ++w) launch(w);
                CK(hipEventRecord(e0, st));
                for (int r = 0; r < rounds; ++r) launch(r);
                CK(hipEventRecord(e1, st));
                CK(hipStreamSynchronize(st));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / rounds;
                if (pass) printf("  batch %-34s %7.2f us per launch  frac %.4f\n", vs[vi].name.c_str(), us,
                                 9.0 * bytes / (us * 1e-6) / 8e12);
            }
    }
    return 0;
}
