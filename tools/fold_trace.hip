// fold_trace.hip -- where the fused 8-operand fold loses its ~8 points against
// the two-operand tile.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/fold_trace tools/fold_trace.hip
//   tools/fold_trace [launches per variant = 20]
//
// Part 1, workgroup trace.  The product's fold body (combine_multi_tile,
// reduce_kernels.hpp) for config 5's CHAIN8 fp16 SUM over 8 x 128 MiB
// (operands at the collective's staging stride, block + 4352 B; 96 KiB LDS
// reservation: one 1024-thread workgroup per CU, as the library launches it),
// and the product's two-operand tile (reduce_tile, fp32 SUM, 256 MiB) beside
// it.  Each workgroup's thread 0 stamps the 100 MHz wall clock at its start and
// after its stores completed (s_waitcnt vmcnt(0)), with its XCD.  Per launch:
//   ramp   first start -> the R-th start (R = workgroups resident at once),
//   steady the bytes of workgroups that ENDED between the ramp and the last
//          start, over that window: the rate with every CU busy,
//   drain  last start -> last end,
//   loss   span - total bytes / steady rate, split into head (before the ramp
//          ends) and tail (after the last start) by the same rule,
// plus workgroup durations (mean, p10, p90) and per-XCD spans.
//
// Part 2, candidate shapes, HIP events over batches of back-to-back launches
// on rotating operand sets (> Infinity Cache), variants in shuffled order,
// every output compared bit for bit with the library launch's:
//   library       k_combine_multi<.., 8, .., U = 1, TH = 1024>, 96 KiB LDS
//   persist WxU   persistent workgroups (W per CU, 256 threads, U vectors per
//                 lane per operand), the next tile's 8 x U loads issued before
//                 the current tile's fold and store (software pipeline), tiles
//                 interleaved over the grid
// for CHAIN8 fp16 8 x 128 MiB (config 5) and TREE8 fp32 8 x 32 MiB (config 4).
//
// Part 3, write volume: the fold's eight reads with 0, 1 and 2 output streams.
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

struct Rec {
    unsigned long long t0, t1;
    unsigned int blk, xcc;
};

__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); }

template <class T, bool TREE>
__global__ __launch_bounds__(1024) void k_fold_traced(MultiArgs a, Rec *rec) {
    const unsigned long long t0 = wall_clock64();
    combine_multi_tile<OpSum, T, 8, TREE, 1, 1024>(a, blockIdx.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) rec[blockIdx.x] = Rec{t0, (unsigned long long)wall_clock64(), blockIdx.x, xcc_id()};
}

__global__ __launch_bounds__(kThreads) void k_tile_traced(const char *in, char *io, uint64_t vbytes, Rec *rec) {
    const unsigned long long t0 = wall_clock64();
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) rec[blockIdx.x] = Rec{t0, (unsigned long long)wall_clock64(), blockIdx.x, xcc_id()};
}

__global__ __launch_bounds__(kThreads) void k_tile(const char *in, char *io, uint64_t vbytes) {
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
}

// ---- persistent, software-pipelined fold ------------------------------------
template <class T, int P, int U>
__device__ __forceinline__ void fold_load(u32x4 (&v)[P][U], const MultiArgs &a, uint64_t blk) {
    constexpr uint32_t tile = kThreads * U * 16;
    const uint64_t base = blk * tile, left = a.vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (U * 1024) + (t & 63) * 16;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < P; ++j) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
            v[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r, wb + u * 1024, 0, kCachePolicyNT);
            if ((u * P + j + 1) % 4 == 0 && u * P + j + 1 < U * P) issue_gap();
        }
}

template <class T, int P, bool TREE, int U>
__device__ __forceinline__ void fold_store(const u32x4 (&v)[P][U], const MultiArgs &a, uint64_t blk) {
    constexpr uint32_t tile = kThreads * U * 16;
    const uint64_t base = blk * tile, left = a.vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (U * 1024) + (t & 63) * 16;
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        Pack16<T> pk[P];
#pragma unroll
        for (int j = 0; j < P; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, v[j][u]);
        Pack16<T> res;
#pragma unroll
        for (int k = 0; k < (int)(16 / sizeof(T)); ++k) {
            T e[P];
#pragma unroll
            for (int j = 0; j < P; ++j) e[j] = pk[j].e[k];
            res.e[k] = fold_fast<OpSum, T, P, TREE>(e);
        }
        store16(__builtin_bit_cast(u32x4, res), ro, wb + u * 1024, keep_tile(base, a.vbytes, a.keep));
    }
}

template <class T, bool TREE, int U>
__global__ __launch_bounds__(kThreads) void k_fold_persist(MultiArgs a, uint64_t ntiles) {
    u32x4 x[8][U], y[8][U];
    uint64_t blk = blockIdx.x;
    const uint64_t g = gridDim.x;
    if (blk < ntiles) fold_load<T, 8, U>(x, a, blk);
    while (blk < ntiles) {
        if (blk + g < ntiles) fold_load<T, 8, U>(y, a, blk + g);
        fold_store<T, 8, TREE, U>(x, a, blk);
        blk += g;
        if (blk >= ntiles) break;
        if (blk + g < ntiles) fold_load<T, 8, U>(x, a, blk + g);
        fold_store<T, 8, TREE, U>(y, a, blk);
        blk += g;
    }
}

// ---- write-volume probe: the product fold (1024 threads, U = 1) with NW output
// streams: 0 (the eight reads alone; a store only for an impossible result, so
// the loads stay live), 1 (the product), 2 (the result to out and to out2)
template <int NW>
__global__ __launch_bounds__(1024) void k_fold_nw(MultiArgs a, char *out2) {
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
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, wb, 0, kCachePolicyNT);
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
    const u32x4 v = __builtin_bit_cast(u32x4, res);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
    if (NW == 0) {
        if (__builtin_expect(v.x == 0xFFFFFFFFu && v.y == 0x01234567u, 0)) store16(v, ro, wb, false);
    } else {
        store16(v, ro, wb, false);
        if (NW == 2) {
            __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void *)(out2 + base), 0, nrec, 0x00020000);
            store16(v, r2, wb, false);
        }
    }
}

// ---- harness ----------------------------------------------------------------
__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed, int f16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = f16 ? (uint16_t)(x & 0xBFFF) : (uint16_t)((i & 1) ? ((x & 0x803F) | 0x3E00) : x);
    }
}

static double pctl(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(p * (double)(v.size() - 1))];
}

struct Trace {
    double span = 0, ramp = 0, drain = 0, steady = 0, loss = 0, head = 0, tail = 0, dmean = 0, dp10 = 0, dp90 = 0;
    double xspan[8] = {0};
    int n = 0;
};

// one launch's records -> Trace increments; bytes per workgroup `wgb`, R resident
static void analyse(std::vector<Rec> &v, double wgb, size_t R, double tick_us, Trace &tr) {
    unsigned long long t0 = ~0ull, t1 = 0;
    std::vector<double> st, dur;
    for (const Rec &r : v) {
        t0 = std::min(t0, r.t0);
        t1 = std::max(t1, r.t1);
    }
    for (const Rec &r : v) {
        st.push_back((double)(r.t0 - t0) * tick_us);
        dur.push_back((double)(r.t1 - r.t0) * tick_us);
    }
    std::vector<double> sorted = st;
    std::sort(sorted.begin(), sorted.end());
    const double span = (double)(t1 - t0) * tick_us;
    const double ramp = sorted[std::min(R, sorted.size()) - 1];
    const double last_start = sorted.back();
    double mid_bytes = 0, head_bytes = 0, tail_bytes = 0;
    for (const Rec &r : v) {
        const double e = (double)(r.t1 - t0) * tick_us;
        if (e <= ramp) head_bytes += wgb;
        else if (e <= last_start) mid_bytes += wgb;
        else tail_bytes += wgb;
    }
    const double rate = mid_bytes / std::max(1e-9, last_start - ramp);        // bytes per us
    tr.span += span;
    tr.ramp += ramp;
    tr.drain += span - last_start;
    tr.steady += rate * 1e6 / 8e12;
    tr.loss += span - (head_bytes + mid_bytes + tail_bytes) / rate;
    tr.head += ramp - head_bytes / rate;
    tr.tail += (span - last_start) - tail_bytes / rate;
    double m = 0;
    for (double d : dur) m += d;
    tr.dmean += m / dur.size();
    tr.dp10 += pctl(dur, 0.1);
    tr.dp90 += pctl(dur, 0.9);
    for (int x = 0; x < 8; ++x) {
        unsigned long long a = ~0ull, z = 0;
        for (const Rec &r : v)
            if ((int)(r.xcc & 7) == x) {
                a = std::min(a, r.t0);
                z = std::max(z, r.t1);
            }
        if (z) tr.xspan[x] += (double)(z - a) * tick_us;
    }
    ++tr.n;
}

static void report(const char *name, const Trace &t, double bytes, double ev_us) {
    const double n = t.n;
    printf("%s\n", name);
    printf("  event mean %.2f us (%.4f of 8 TB/s); traced span %.2f us\n", ev_us, bytes / (ev_us * 1e-6) / 8e12, t.span / n);
    printf("  ramp %.2f us, drain %.2f us; steady state %.4f of 8 TB/s\n", t.ramp / n, t.drain / n, t.steady / n);
    printf("  loss vs steady rate %.2f us = head %.2f + tail %.2f + (rest %.2f)\n", t.loss / n, t.head / n, t.tail / n,
           (t.loss - t.head - t.tail) / n);
    printf("  workgroup duration mean %.2f us, p10 %.2f, p90 %.2f\n", t.dmean / n, t.dp10 / n, t.dp90 / n);
    printf("  per XCD span (us):");
    for (int x = 0; x < 8; ++x) printf(" %.2f", t.xspan[x] / n);
    printf("\n");
}

struct Case {
    const char *name;
    uint64_t block;
    bool f16;
};

template <class T, bool TREE>
void launch_var(int v, const MultiArgs &a, int ncu, hipStream_t s) {
    const uint64_t n1 = (a.vbytes + 16383) / 16384;
    switch (v) {
    case 0:
        hipLaunchKernelGGL((k_combine_multi<OpSum, T, 8, TREE, 1, 1024>), dim3((unsigned)n1), dim3(1024), 96 << 10, s, a);
        break;
    case 1: {   // persist 2 x U1
        const uint64_t nt = (a.vbytes + 4095) / 4096;
        hipLaunchKernelGGL((k_fold_persist<T, TREE, 1>), dim3(2 * ncu), dim3(kThreads), 0, s, a, nt);
        break;
    }
    case 2: {   // persist 4 x U1
        const uint64_t nt = (a.vbytes + 4095) / 4096;
        hipLaunchKernelGGL((k_fold_persist<T, TREE, 1>), dim3(4 * ncu), dim3(kThreads), 0, s, a, nt);
        break;
    }
    case 3: {   // persist 2 x U2
        const uint64_t nt = (a.vbytes + 8191) / 8192;
        hipLaunchKernelGGL((k_fold_persist<T, TREE, 2>), dim3(2 * ncu), dim3(kThreads), 0, s, a, nt);
        break;
    }
    default: {  // persist 4 x U2
        const uint64_t nt = (a.vbytes + 8191) / 8192;
        hipLaunchKernelGGL((k_fold_persist<T, TREE, 2>), dim3(4 * ncu), dim3(kThreads), 0, s, a, nt);
        break;
    }
    }
}
const char *kVarNames[] = {"library (1024 x 1, 1 / CU)", "persist 2/CU x U1", "persist 4/CU x U1",
                           "persist 2/CU x U2", "persist 4/CU x U2"};
constexpr int kNV = 5;

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 20;
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, f16, 8, false, 1, 1024>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, float, 8, true, 1, 1024>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_fold_traced<f16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    int ncu = 0, freq_khz = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&freq_khz, hipDeviceAttributeWallClockRate, 0));
    const double tick_us = 1e3 / (double)freq_khz;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    // ---------------- part 1: traces -----------------------------------------
    {
        const uint64_t block = 128ull << 20, stride = block + 4352, setbytes = 8 * stride + block;
        const int nsets = 3;
        std::vector<char *> sets(nsets);
        for (auto &p : sets) {
            CK(hipMalloc(&p, setbytes));
            k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p, 1);
        }
        const unsigned groups = (unsigned)(block / 16384);
        Rec *drec;
        CK(hipMalloc(&drec, sizeof(Rec) * groups));
        std::vector<Rec> rec(groups);
        Trace tr;
        double ev = 0;
        int nev = 0;
        for (int it = 0; it < K + 3; ++it) {
            MultiArgs a{};
            char *b = sets[it % nsets];
            for (int j = 0; j < 8; ++j) a.in[j] = b + j * stride;
            a.out = b + 8 * stride;
            a.vbytes = block;
            a.keep = keep_for(block);
            CK(hipMemsetAsync(drec, 0, sizeof(Rec) * groups, s));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL((k_fold_traced<f16, false>), dim3(groups), dim3(1024), 96 << 10, s, a, drec);
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it < 3) continue;
            ev += ms * 1e3;
            ++nev;
            CK(hipMemcpy(rec.data(), drec, sizeof(Rec) * groups, hipMemcpyDeviceToHost));
            analyse(rec, 9.0 * 16384, (size_t)ncu, tick_us, tr);
        }
        report("CHAIN8 fp16 SUM 8 x 128 MiB, traced library fold (1024 threads, 1 workgroup / CU)", tr, 9.0 * block,
               ev / nev);
        CK(hipFree(drec));
        for (auto p : sets) CK(hipFree(p));
    }
    {
        const uint64_t bytes = 256ull << 20, foot = 1ull << 30;
        const int nwin = (int)(foot / bytes);
        char *in, *io;
        CK(hipMalloc(&in, foot));
        CK(hipMalloc(&io, foot));
        k_fill<<<4096, 256>>>((uint16_t *)in, foot / 2, 1, 0);
        k_fill<<<4096, 256>>>((uint16_t *)io, foot / 2, 2, 0);
        const unsigned groups = (unsigned)(bytes / kTileBytes);
        Rec *drec;
        CK(hipMalloc(&drec, sizeof(Rec) * groups));
        std::vector<Rec> rec(groups);
        // resident workgroups per CU of the plain tile kernel
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)k_tile_traced, kThreads, 0));
        Trace tr;
        double ev = 0;
        int nev = 0;
        for (int it = 0; it < K + 3; ++it) {
            const size_t off = (size_t)(it % nwin) * bytes;
            CK(hipMemsetAsync(drec, 0, sizeof(Rec) * groups, s));
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_tile_traced, dim3(groups), dim3(kThreads), 0, s, in + off, io + off, bytes, drec);
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it < 3) continue;
            ev += ms * 1e3;
            ++nev;
            CK(hipMemcpy(rec.data(), drec, sizeof(Rec) * groups, hipMemcpyDeviceToHost));
            analyse(rec, 3.0 * kTileBytes, (size_t)ncu * occ, tick_us, tr);
        }
        char name[160];
        snprintf(name, sizeof name, "two-operand tile fp32 SUM 256 MiB, traced (256 threads, %d resident / CU)", occ);
        report(name, tr, 3.0 * bytes, ev / nev);
        CK(hipFree(drec));
        CK(hipFree(in));
        CK(hipFree(io));
    }

    // ---------------- part 2: candidate shapes ---------------------------------
    const Case cases[] = {{"config5 CHAIN8 fp16 8 x 128 MiB", 128ull << 20, true},
                          {"config4 TREE8 fp32 8 x 32 MiB", 32ull << 20, false}};
    for (const Case &c : cases) {
        const uint64_t stride = c.block + 4352, setbytes = 8 * stride + c.block;
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
            if (c.f16) launch_var<f16, false>(v, args(k), ncu, s);
            else launch_var<float, true>(v, args(k), ncu, s);
        };
        std::vector<char> h0(c.block), h1(c.block);
        run(0, 0);
        CK(hipMemcpyAsync(h0.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        bool same = true;
        for (int v = 1; v < kNV; ++v) {
            CK(hipMemsetAsync(args(0).out, 0, c.block, s));
            run(0, v);
            CK(hipMemcpyAsync(h1.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            const bool eq = memcmp(h0.data(), h1.data(), c.block) == 0;
            if (!eq) printf("  variant %s differs\n", kVarNames[v]);
            same = same && eq;
        }
        std::vector<double> us[kNV];
        std::mt19937 rng(11);
        const int batch = 20;
        int k = 1;
        for (int r = 0; r < 11; ++r) {
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
        printf("%s (%d sets, 10 rounds x %d launches), outputs identical across variants: %s\n", c.name, nsets, batch,
               same ? "yes" : "NO");
        for (int v = 0; v < kNV; ++v) {
            std::sort(us[v].begin(), us[v].end());
            const double med = us[v][us[v].size() / 2];
            printf("  %-28s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f\n", kVarNames[v], med, us[v][0],
                   bytes / (med * 1e-6) / 8e12);
        }
        for (auto p : sets) CK(hipFree(p));
    }

    // ---------------- part 3: write volume ------------------------------------
    // the fold's eight reads with 0 / 1 / 2 output streams (nt stores), CHAIN8
    // fp16 over 8 x 128 MiB: if the mix, not the bytes, sets the rate, a second
    // write stream costs less than its bytes at the fold's rate
    {
        CK(hipFuncSetAttribute((const void *)k_fold_nw<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
        CK(hipFuncSetAttribute((const void *)k_fold_nw<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
        CK(hipFuncSetAttribute((const void *)k_fold_nw<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
        const uint64_t block = 128ull << 20, stride = block + 4352, setbytes = 8 * stride + 2 * block + 4352;
        const int nsets = 3;
        std::vector<char *> sets(nsets);
        for (auto &p : sets) {
            CK(hipMalloc(&p, setbytes));
            k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p, 1);
        }
        CK(hipDeviceSynchronize());
        const unsigned groups = (unsigned)(block / 16384);
        auto run = [&](int k, int nw) {
            MultiArgs a{};
            char *b = sets[k % nsets];
            for (int j = 0; j < 8; ++j) a.in[j] = b + j * stride;
            a.out = b + 8 * stride;
            a.vbytes = block;
            char *o2 = b + 8 * stride + block + 4352;
            if (nw == 0) hipLaunchKernelGGL(k_fold_nw<0>, dim3(groups), dim3(1024), 96 << 10, s, a, o2);
            else if (nw == 1) hipLaunchKernelGGL(k_fold_nw<1>, dim3(groups), dim3(1024), 96 << 10, s, a, o2);
            else hipLaunchKernelGGL(k_fold_nw<2>, dim3(groups), dim3(1024), 96 << 10, s, a, o2);
        };
        std::vector<double> us[3];
        std::mt19937 rng(5);
        int k = 0;
        const int batch = 20;
        for (int r = 0; r < 11; ++r) {
            int order[3] = {0, 1, 2};
            std::shuffle(order, order + 3, rng);
            for (int nw : order) {
                run(k++, nw);
                CK(hipEventRecord(e0, s));
                for (int b = 0; b < batch; ++b) run(k++, nw);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) us[nw].push_back(ms * 1e3 / batch);
            }
        }
        printf("write volume: CHAIN8 fp16 8 x 128 MiB reads + 0 / 1 / 2 nt output streams (1 workgroup / CU), "
               "10 rounds x %d launches\n", batch);
        double med[3];
        for (int nw = 0; nw < 3; ++nw) {
            std::sort(us[nw].begin(), us[nw].end());
            med[nw] = us[nw][us[nw].size() / 2];
            const double bytes = (8.0 + nw) * block;
            printf("  8R + %dW  median %8.2f us  frac of 8 TB/s %.4f\n", nw, med[nw], bytes / (med[nw] * 1e-6) / 8e12);
        }
        printf("  the first write stream costs %.2f us (%.2f us at the reads' rate), the second %.2f us\n",
               med[1] - med[0], med[0] / 8.0, med[2] - med[1]);
        for (auto p : sets) CK(hipFree(p));
    }
    return 0;
}
