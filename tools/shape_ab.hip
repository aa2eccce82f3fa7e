// shape_ab.hip -- interleaved A/B of issue-order variants of the aligned tile
// kernel (fp32 SUM, 256 MiB per operand) against the product launcher.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/shape_ab tools/shape_ab.hip
//   ./tools/shape_ab [MiB_per_operand=256] [rounds=20]
// Variants (all: 16 B per lane per access, buffer_load/store nt, one tile per WG):
//   bar     __syncthreads() between the loads and the stores (a WG's stores leave
//           as one burst after all its loads returned)
//   ioin    all inout loads issued before all in loads (product interleaves them)
//   prio    s_setprio 3 while issuing loads, 0 for the stores
//   wave    each wave owns a contiguous 4 KiB of the tile (product: the four
//           vectors of a lane are 4 KiB apart, waves interleaved at 1 KiB)
//   t512    512-thread WG, 4 vectors per lane (32 KiB tile per operand)
// Four operand pairs rotate (> Infinity Cache); the variant order is shuffled
// every round.  Median / min per variant.
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

enum { V_BAR = 1, V_IOIN = 2, V_PRIO = 4, V_WAVE = 8 };

template <int TH, int FLAGS>
__global__ __launch_bounds__(TH) void k_var(const char *in, char *io, uint64_t vbytes) {
    constexpr uint32_t tile = TH * 4 * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    auto off = [&](int u) {
        if constexpr (FLAGS & V_WAVE) return ((t >> 6) * 4 + u) * 1024 + (t & 63) * 16;
        else return (u * TH + t) * 16;
    };
    u32x4 a[4], b[4];
    if constexpr (FLAGS & V_PRIO) __builtin_amdgcn_s_setprio(3);
    if constexpr (FLAGS & V_IOIN) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off(u), 0, kCachePolicyNT);
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off(u), 0, kCachePolicyNT);
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off(u), 0, kCachePolicyNT);
            b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off(u), 0, kCachePolicyNT);
        }
    }
    if constexpr (FLAGS & V_PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (FLAGS & V_BAR) {
        // force the loads to complete before the barrier
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = combine16<OpSum, float>(a[u], b[u]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(a[u], rio, off(u), 0, kCachePolicyNT);
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(a[u], b[u]), rio, off(u), 0, kCachePolicyNT);
    }
}

template <int TH, int FLAGS>
hipError_t launch_var(const void *in, void *io, uint64_t count, hipStream_t s) {
    const uint64_t vbytes = count * 4;   // 256 B-aligned buffers, multiple of 16 B
    constexpr uint32_t tile = TH * 4 * 16;
    hipLaunchKernelGGL((k_var<TH, FLAGS>), dim3((unsigned)((vbytes + tile - 1) / tile)), dim3(TH), 0, s,
                       (const char *)in, (char *)io, vbytes);
    return hipGetLastError();
}

// the product's body behind another symbol (identical code, other kernel object)
__global__ __launch_bounds__(256) void k_tile_clone(TileArgs<float> a) { reduce_tile_body<OpSum, float>(a); }
hipError_t launch_clone(const void *in, void *io, uint64_t count, hipStream_t s) {
    TileArgs<float> a{(const char *)in, (char *)io, count * 4, (const float *)in, (float *)io, 0,
                      (const float *)in, (float *)io, 0};
    hipLaunchKernelGGL(k_tile_clone, dim3((unsigned)((count * 4 + kTileBytes - 1) / kTileBytes)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// slim kernargs (32 B): head/tail addresses derived from the vector region
struct SlimArgs { const char *in; char *io; uint64_t vbytes; uint32_t nhead, ntail; };
template <bool PRO>
__global__ __launch_bounds__(256) void k_slim(SlimArgs a) {
    OpSum op;
    const unsigned t = threadIdx.x;
    if (PRO && blockIdx.x == 0) {
        const float *hin = reinterpret_cast<const float *>(a.in) - a.nhead;
        float *hio = reinterpret_cast<float *>(a.io) - a.nhead;
        if (t < a.nhead) hio[t] = op(hio[t], hin[t]);
        else if (t >= 64 && t - 64 < a.ntail) {
            const float *tin = reinterpret_cast<const float *>(a.in + a.vbytes);
            float *tio = reinterpret_cast<float *>(a.io + a.vbytes);
            tio[t - 64] = op(tio[t - 64], tin[t - 64]);
        }
    }
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base < a.vbytes) {
        const uint64_t left = a.vbytes - base;
        const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
        __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in + base), 0, nrec, 0x00020000);
        __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(a.io + base), 0, nrec, 0x00020000);
        const int wbase = ((int)t >> 6) * 4096 + ((int)t & 63) * 16;
        u32x4 x[4], y[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wbase + u * 1024, 0, kCachePolicyNT);
            y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wbase + u * 1024, 0, kCachePolicyNT);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(x[u], y[u]), rio, wbase + u * 1024, 0, kCachePolicyNT);
    }
    if (!PRO && blockIdx.x == 0) {
        const float *hin = reinterpret_cast<const float *>(a.in) - a.nhead;
        float *hio = reinterpret_cast<float *>(a.io) - a.nhead;
        if (t < a.nhead) hio[t] = op(hio[t], hin[t]);
        else if (t >= 64 && t - 64 < a.ntail) {
            const float *tin = reinterpret_cast<const float *>(a.in + a.vbytes);
            float *tio = reinterpret_cast<float *>(a.io + a.vbytes);
            tio[t - 64] = op(tio[t - 64], tin[t - 64]);
        }
    }
}
template <bool PRO>
hipError_t launch_slim(const void *in, void *io, uint64_t count, hipStream_t s) {
    SlimArgs a{(const char *)in, (char *)io, count * 4, 0, 0};
    hipLaunchKernelGGL(k_slim<PRO>, dim3((unsigned)((count * 4 + kTileBytes - 1) / kTileBytes)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// H1: the wave kernel plus a block-0 epilogue (head/tail-like scalar fix-up)
// H3: the wave kernel without the early exit (descriptor range 0 past the end)
template <int H>
__global__ __launch_bounds__(256) void k_h(const char *in, char *io, uint64_t vbytes, uint32_t nfix) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    const int t = (int)threadIdx.x;
    auto body = [&](int nrec) {
        __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
        __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
        const int wbase = (t >> 6) * 4096 + (t & 63) * 16;
        u32x4 x[4], y[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wbase + u * 1024, 0, kCachePolicyNT);
            y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wbase + u * 1024, 0, kCachePolicyNT);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(x[u], y[u]), rio, wbase + u * 1024, 0, kCachePolicyNT);
    };
    if constexpr (H == 3) {
        const uint64_t left = vbytes > base ? vbytes - base : 0;
        body((int)(left < kTileBytes ? left : kTileBytes));
    } else {
        if (base < vbytes) {
            const uint64_t left = vbytes - base;
            body((int)(left < kTileBytes ? left : kTileBytes));
        }
        if (blockIdx.x == 0 && (unsigned)t < nfix) {
            float *p = reinterpret_cast<float *>(io) + t;
            *p = *p + reinterpret_cast<const float *>(in)[t];
        }
    }
}
template <int H>
hipError_t launch_h(const void *in, void *io, uint64_t count, hipStream_t s) {
    hipLaunchKernelGGL(k_h<H>, dim3((unsigned)((count * 4 + kTileBytes - 1) / kTileBytes)), dim3(256), 0, s,
                       (const char *)in, (char *)io, count * 4, 0u);
    return hipGetLastError();
}

// the wave kernel's code behind a 72-byte by-value struct (kernarg-size test)
struct Args72 { const char *in; char *io; uint64_t vbytes; uint64_t pad[6]; };
__global__ __launch_bounds__(256) void k_wave72(Args72 a) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= a.vbytes) return;
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(a.io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wbase = (t >> 6) * 4096 + (t & 63) * 16;
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wbase + u * 1024, 0, kCachePolicyNT);
        y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wbase + u * 1024, 0, kCachePolicyNT);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(x[u], y[u]), rio, wbase + u * 1024, 0, kCachePolicyNT);
}
hipError_t launch_wave72(const void *in, void *io, uint64_t count, hipStream_t s) {
    Args72 a{(const char *)in, (char *)io, count * 4, {}};
    hipLaunchKernelGGL(k_wave72, dim3((unsigned)((count * 4 + kTileBytes - 1) / kTileBytes)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// immediate-offset test: the same wave-layout tile with every access's offset
// either folded into the instruction's 12-bit immediate (IMM) or held in its
// own VGPR with immediate 0 (VREG, offsets made opaque to the compiler)
template <bool VREG, int GAP = 0>
__global__ __launch_bounds__(256) void k_off(const char *in, char *io, uint64_t vbytes) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    int off[4];
    const int wb = (t >> 6) * 4096 + (t & 63) * 16;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        off[u] = wb + u * 1024;
        if constexpr (VREG) asm volatile("" : "+v"(off[u]));
    }
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off[u], 0, kCachePolicyNT);
        if constexpr (GAP == 3) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 0"); __builtin_amdgcn_sched_barrier(0); }
        y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off[u], 0, kCachePolicyNT);
        if constexpr (GAP == 3 || GAP == 6) {
            if (u < 3) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 0"); __builtin_amdgcn_sched_barrier(0); }
        }
        if constexpr (GAP == 4) {
            if (u < 3) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 3"); __builtin_amdgcn_sched_barrier(0); }
        }
        if constexpr (GAP == 5) {
            if (u < 3) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 7"); __builtin_amdgcn_sched_barrier(0); }
        }
        // GAP 1: one s_nop after the 2nd pair; GAP 2: after every pair
        if constexpr (GAP == 1) {
            if (u == 1) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 0"); __builtin_amdgcn_sched_barrier(0); }
        }
        if constexpr (GAP == 2) {
            if (u < 3) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 0"); __builtin_amdgcn_sched_barrier(0); }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(x[u], y[u]), rio, off[u], 0, kCachePolicyNT);
        if constexpr (GAP == 6) {
            if (u < 3) { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 0"); __builtin_amdgcn_sched_barrier(0); }
        }
    }
}
template <bool VREG, int GAP = 0>
hipError_t launch_off(const void *in, void *io, uint64_t count, hipStream_t s) {
    hipLaunchKernelGGL((k_off<VREG, GAP>), dim3((unsigned)((count * 4 + kTileBytes - 1) / kTileBytes)), dim3(256), 0, s,
                       (const char *)in, (char *)io, count * 4);
    return hipGetLastError();
}

// vectors per lane / workgroup size with the issue gap (NOP: s_nop count, -1 = no gap)
template <int U, int TH, int NOP>
__global__ __launch_bounds__(TH) void k_uv(const char *in, char *io, uint64_t vbytes) {
    constexpr uint32_t tile = TH * U * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (U * 1024) + (t & 63) * 16;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
        y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
        if constexpr (NOP >= 0) {
            if (u + 1 < U) {
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (NOP == 0) asm volatile("s_nop 0");
                if constexpr (NOP == 1) asm volatile("s_nop 1");
                if constexpr (NOP == 3) asm volatile("s_nop 3");
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(x[u], y[u]), rio, wb + u * 1024, 0, kCachePolicyNT);
}
template <int U, int TH, int NOP>
hipError_t launch_uv(const void *in, void *io, uint64_t count, hipStream_t s) {
    constexpr uint32_t tile = TH * U * 16;
    hipLaunchKernelGGL((k_uv<U, TH, NOP>), dim3((unsigned)((count * 4 + tile - 1) / tile)), dim3(TH), 0, s,
                       (const char *)in, (char *)io, count * 4);
    return hipGetLastError();
}

// refinements of the issue gap: MODE 0 product shape (io, in, nop 0);
// 1 in-first pairs; 2 odd waves s_sleep 1 at start; 3 s_nop 1; 4 s_nop 2
template <int MODE>
__global__ __launch_bounds__(256) void k_g(const char *in, char *io, uint64_t vbytes) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    if constexpr (MODE == 2) {
        if ((t >> 6) & 1) __builtin_amdgcn_s_sleep(1);
    }
    const int wb = (t >> 6) * 4096 + (t & 63) * 16;
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if constexpr (MODE == 1) {
            y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
        } else {
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
            y[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
        }
        if (u < 3) {
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (MODE == 3) asm volatile("s_nop 1");
            else if constexpr (MODE == 4) asm volatile("s_nop 2");
            else asm volatile("s_nop 0");
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(x[u], y[u]), rio, wb + u * 1024, 0, kCachePolicyNT);
}
template <int MODE>
hipError_t launch_g(const void *in, void *io, uint64_t count, hipStream_t s) {
    hipLaunchKernelGGL((k_g<MODE>), dim3((unsigned)((count * 4 + kTileBytes - 1) / kTileBytes)), dim3(256), 0, s,
                       (const char *)in, (char *)io, count * 4);
    return hipGetLastError();
}

struct Var { std::string name; hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t); std::vector<float> ms; };

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    int rounds = argc > 2 ? atoi(argv[2]) : 20;
    size_t bytes = mib << 20;
    const int NS = 4;
    char *in[NS], *io[NS];
    std::vector<float> h(bytes / 4);
    uint32_t x = 0x5EED;
    for (size_t i = 0; i < h.size(); ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; h[i] = (float)(x >> 8) * (1.0f / 16777216.0f) * 2 - 1; }
    for (int s = 0; s < NS; ++s) {
        CK(hipMalloc(&in[s], bytes));
        CK(hipMalloc(&io[s], bytes));
        CK(hipMemcpy(in[s], h.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(io[s], h.data(), bytes, hipMemcpyHostToDevice));
    }
    std::vector<Var> vs = {
        {"product", &launch_reduce<OpSum, float>, {}},
        {"g0 same as product", &launch_g<0>, {}},
        {"g1 in-first", &launch_g<1>, {}},
        {"g2 odd-wave sleep", &launch_g<2>, {}},
        {"g3 nop1", &launch_g<3>, {}},
        {"g4 nop2", &launch_g<4>, {}},
        {"U4 T256 nogap", &launch_uv<4, 256, -1>, {}},
    };
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int slot = 0;
    std::vector<int> order(vs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    uint32_t rs = 12345;
    for (int r = -2; r < rounds; ++r) {
        // a fresh random order every round: no variant keeps a fixed position
        for (size_t i = order.size() - 1; i > 0; --i) {
            rs = rs * 1664525u + 1013904223u;
            std::swap(order[i], order[(rs >> 8) % (i + 1)]);
        }
        for (int vi : order) {
            Var &v = vs[vi];
            int s = slot++ % NS;
            CK(hipEventRecord(e0, st));
            CK(v.fn(in[s], io[s], bytes / 4, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) v.ms.push_back(ms);
        }
    }
    printf("fp32 SUM %zu MiB per operand, %d interleaved rounds, %d rotating pairs\n", mib, rounds, NS);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
        printf("  %-18s median %8.2f us  min %8.2f us  frac(median) %.3f\n", v.name.c_str(), med * 1e3, mn * 1e3,
               3.0 * bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}
