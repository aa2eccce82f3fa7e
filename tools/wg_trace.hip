// wg_trace.hip -- first / last workgroup tracing of the product tile kernel
// (reduce_tile<OpSum,float>, csrc/hip/reduce_kernels.hpp) on MI355X.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpich-pip_amd/csrc/hip \
//         tools/wg_trace.hip -o tools/wg_trace
//   tools/wg_trace [MiB per operand, default 64] [launches, default 40]
//
// Each workgroup's thread 0 records the 100 MHz wall clock when the
// workgroup starts and after its stores have completed (s_waitcnt), plus the
// XCC / SE / CU it ran on.  Launches rotate over windows of a 2 GiB (in, inout)
// footprint, so no launch finds its operands in the 256 MB MALL.  Per launch:
// the HIP-event duration, and from the records the start ramp (time until
// 50 / 90 / 100 % of workgroups had started), the end tail (time from 50 / 90 %
// of workgroups finished to the last), and per-XCD spans.  The instrumented
// kernel is timed next to the plain one so the records' cost is visible.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#include "reduce_kernels.hpp"

using namespace mpir_hip;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Rec {
    unsigned long long t0, t1;
    unsigned int hw, xcc;      // k_dyn: hw = tiles this workgroup processed
};

__global__ __launch_bounds__(kThreads) void k_plain(const char *in, char *io, uint64_t vbytes, uint64_t keep) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    reduce_tile<OpSum, float>(in, io, base, vbytes, keep);
}

// remap: 0..7 = tile (b & ~7) | ((b + remap) & 7); 8 = rotate the residue
// every 8 workgroups (each XCD walks all residues); 9 = swap 64 KiB halves
__device__ __forceinline__ unsigned remap_tile(unsigned b, int remap) {
    if (remap < 8) return (b & ~7u) | ((b + (unsigned)remap) & 7u);
    if (remap == 8) return (b & ~7u) | ((b + (b >> 3)) & 7u);
    return b ^ 4u;
}

// remap 10: XCD x = b % 8 takes a contiguous range of n_even (even x) or
// n_odd (odd x) tiles; workgroups past their XCD's share exit at once
__global__ __launch_bounds__(kThreads) void k_traced(const char *in, char *io, uint64_t vbytes, uint64_t keep,
                                                     Rec *rec, int remap, unsigned n_even, unsigned n_odd) {
    const unsigned long long t0 = wall_clock64();
    uint64_t tile;
    if (remap == 11) {
        // periods of P rounds: odd XCDs sit out the last d rounds of each
        // (n_even = P, n_odd = d); tiles stay interleaved at 16 KiB
        const unsigned P = n_even, d = n_odd;
        const unsigned x = blockIdx.x & 7u, J = blockIdx.x >> 3, per = J / P, j = J % P;
        if ((x & 1u) && j >= P - d) return;
        const unsigned idx = j < P - d ? j * 8u + x : (P - d) * 8u + (j - (P - d)) * 4u + (x >> 1);
        tile = (uint64_t)per * (8u * P - 4u * d) + idx;
        if (tile * kTileBytes >= vbytes) return;
    } else if (remap == 10) {
        const unsigned x = blockIdx.x & 7u, j = blockIdx.x >> 3;
        if (j >= ((x & 1u) ? n_odd : n_even)) return;
        tile = (uint64_t)(x >> 1) * (n_even + n_odd) + ((x & 1u) ? n_even : 0u) + j;
    } else {
        tile = remap_tile(blockIdx.x, remap);
    }
    const uint64_t base = tile * kTileBytes;
    if (base >= vbytes) return;
    reduce_tile<OpSum, float>(in, io, base, vbytes, keep);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        Rec r;
        r.t0 = t0;
        r.t1 = wall_clock64();
        r.hw = blockIdx.x;
        r.xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID, 16 bits
        rec[blockIdx.x] = r;
    }
}

// persistent workgroups, tiles handed out by a global ticket counter (one
// vector atomic per tile, the next ticket fetched while the current tile is in
// flight); a workgroup on a faster XCD simply takes more tiles
template <bool TRACE>
__global__ __launch_bounds__(kThreads) void k_dyn(const char *in, char *io, uint64_t vbytes, uint64_t keep,
                                                  unsigned *ctr, Rec *rec) {
    __shared__ unsigned next;
    const unsigned long long t0 = wall_clock64();
    const unsigned ntiles = (unsigned)(vbytes / kTileBytes);
    if (threadIdx.x == 0) next = atomicAdd(ctr, 1u);
    __syncthreads();
    unsigned tile = next;
    unsigned done = 0;
    while (tile < ntiles) {
        __syncthreads();
        if (threadIdx.x == 0) next = atomicAdd(ctr, 1u);
        reduce_tile<OpSum, float>(in, io, (uint64_t)tile * kTileBytes, vbytes, keep);
        __syncthreads();
        tile = next;
        ++done;
    }
    if (TRACE) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            Rec r;
            r.t0 = t0;
            r.t1 = wall_clock64();
            r.hw = done;
            r.xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
            rec[blockIdx.x] = r;
        }
    }
}

// the product tile body with U vectors per lane (reduce_tile is U = 4)
template <int U>
__device__ __forceinline__ void tile_u(const char *in, char *io, uint64_t base, uint64_t vbytes, uint64_t keepb) {
    constexpr uint32_t TB = kThreads * U * 16;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < TB ? left : TB);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (U * 1024) + (t & 63) * 16;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
        if (u + 1 < U) issue_gap();
    }
    const bool keep = keep_tile(base, vbytes, keepb);
#pragma unroll
    for (int u = 0; u < U; ++u) store16(combine16<OpSum, float>(a[u], b[u]), rio, wb + u * 1024, keep);
}

// the last `tail` bytes in smaller tiles (US vectors per lane), dispatched last
template <int US>
__global__ __launch_bounds__(kThreads) void k_tailsmall(const char *in, char *io, uint64_t vbytes, uint64_t keep,
                                                        uint64_t b1, unsigned n1) {
    if (blockIdx.x < n1) {
        tile_u<4>(in, io, (uint64_t)blockIdx.x * kTileBytes, vbytes, keep);
    } else {
        const uint64_t base = b1 + (uint64_t)(blockIdx.x - n1) * (kThreads * US * 16);
        if (base < vbytes) tile_u<US>(in, io, base, vbytes, keep);
    }
}

static double pct(std::vector<unsigned long long> &v, double p) {
    size_t i = (size_t)(p * (double)(v.size() - 1));
    return (double)v[i];
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? strtoul(argv[1], nullptr, 10) : 64;
    const int K = argc > 2 ? atoi(argv[2]) : 40;
    const size_t bytes = mib << 20;
    const size_t foot = 1ull << 30;                 // per operand side: 2 GiB total
    const int nwin = (int)std::max<size_t>(1, foot / bytes);
    char *in, *io;
    CK(hipMalloc(&in, foot));
    CK(hipMalloc(&io, foot));
    CK(hipMemset(in, 0, foot));
    CK(hipMemset(io, 0, foot));
    const unsigned groups = (unsigned)(bytes / kTileBytes);
    Rec *drec;
    CK(hipMalloc(&drec, sizeof(Rec) * groups * 2));
    unsigned *ctr;
    CK(hipMalloc(&ctr, 4096));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int pgrid_mult = getenv("WG_PER_CU") ? atoi(getenv("WG_PER_CU")) : 8;
    const unsigned pgroups = (unsigned)std::min<size_t>(groups, (size_t)ncu * pgrid_mult);
    std::vector<Rec> rec(groups * 2), last;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int freq_khz = 0;
    CK(hipDeviceGetAttribute(&freq_khz, hipDeviceAttributeWallClockRate, 0));
    const double tick_us = 1e3 / (double)freq_khz;
    const uint64_t keep = 64ull << 20;
    printf("fp32 SUM, %zu MiB per operand, %u workgroups x %d threads, %d windows, wall clock %d kHz\n", mib, groups,
           kThreads, nwin, freq_khz);

    if (getenv("WG_TAIL")) {
        // interleaved A/B of the product kernel and tail-small variants, HIP events
        struct V { const char *name; int us; int den; };
        const V vs[] = {{"product", 0, 0}, {"tail 1/16 in 4 KiB", 1, 16}, {"tail 1/8 in 4 KiB", 1, 8},
                        {"tail 1/16 in 8 KiB", 2, 16}, {"tail 1/32 in 4 KiB", 1, 32}};
        const int NV = sizeof(vs) / sizeof(vs[0]);
        std::vector<std::vector<float>> d(NV);
        for (int it = 0; it < K + 3; ++it) {
            for (int v = 0; v < NV; ++v) {
                const size_t off = (size_t)((it * NV + v) % nwin) * bytes;
                const uint64_t tailb = vs[v].den ? (bytes / vs[v].den) : 0;
                const uint64_t b1 = bytes - tailb;
                const unsigned n1 = (unsigned)(b1 / kTileBytes);
                CK(hipEventRecord(e0, s));
                if (vs[v].us == 0)
                    hipLaunchKernelGGL(k_plain, dim3(groups), dim3(kThreads), 0, s, in + off, io + off, (uint64_t)bytes, keep);
                else {
                    const unsigned n2 = (unsigned)(tailb / (kThreads * vs[v].us * 16));
                    if (vs[v].us == 1)
                        hipLaunchKernelGGL(k_tailsmall<1>, dim3(n1 + n2), dim3(kThreads), 0, s, in + off, io + off,
                                           (uint64_t)bytes, keep, b1, n1);
                    else
                        hipLaunchKernelGGL(k_tailsmall<2>, dim3(n1 + n2), dim3(kThreads), 0, s, in + off, io + off,
                                           (uint64_t)bytes, keep, b1, n1);
                }
                CK(hipEventRecord(e1, s));
                CK(hipStreamSynchronize(s));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 3) d[v].push_back(ms * 1e3f);
            }
        }
        for (int v = 0; v < NV; ++v) {
            std::sort(d[v].begin(), d[v].end());
            double mean = 0;
            for (float x : d[v]) mean += x;
            mean /= d[v].size();
            printf("%-22s event mean %7.2f us  median %7.2f  p10 %7.2f  (%.4f of 8 TB/s)\n", vs[v].name, mean,
                   d[v][d[v].size() / 2], d[v][d[v].size() / 10], 3.0 * bytes / (mean * 1e-6) / 8e12);
        }
        return 0;
    }
    const char *vname[4] = {"plain", "traced", "dyn", "dyn-traced"};
    const int nvar = getenv("WG_DYN") ? 4 : 2;
    const int remap = getenv("WG_REMAP") ? atoi(getenv("WG_REMAP")) : 0;
    const int wodd = getenv("WG_WODD") ? atoi(getenv("WG_WODD")) : 1000;
    unsigned n_even = 0, n_odd = 0, tgroups = groups;
    if (remap == 10) {
        // 4 n_even + 4 n_odd >= groups, n_odd ~ n_even * wodd / 1000
        n_even = (unsigned)((double)groups / (4.0 * (1.0 + wodd / 1000.0)) + 0.999);
        n_odd = (groups + 3) / 4 > n_even ? (groups + 3) / 4 - n_even : 0;
        while (4ull * (n_even + n_odd) < groups) ++n_odd;
        tgroups = 8 * std::max(n_even, n_odd);
    } else if (remap == 11) {
        n_even = getenv("WG_P") ? atoi(getenv("WG_P")) : 32;      // P
        n_odd = getenv("WG_D") ? atoi(getenv("WG_D")) : 1;        // d
        const unsigned per_tiles = 8 * n_even - 4 * n_odd;
        tgroups = ((groups + per_tiles - 1) / per_tiles) * 8 * n_even;
    }
    printf("remap %d (odd share %d/1000: n_even %u n_odd %u, grid %u)\n", remap, wodd, n_even, n_odd, tgroups);
    for (int variant = 0; variant < nvar; ++variant) {
        const bool tr = variant == 1 || variant == 3;
        const unsigned ng = variant >= 2 ? pgroups : (variant == 1 ? tgroups : groups);
        std::vector<float> dur;
        double r50 = 0, r90 = 0, r100 = 0, e50 = 0, e90 = 0, span = 0, first = 0, busy = 0;
        double xspan[8] = {0}, xmin_end[8] = {0}, xtiles[8] = {0};
        int traced = 0;
        unsigned long long xcc_mismatch = 0;
        for (int it = 0; it < K + 5; ++it) {
            const size_t off = (size_t)(it % nwin) * bytes;
            if (variant >= 2) CK(hipMemsetAsync(ctr, 0, 4, s));
            if (tr) CK(hipMemsetAsync(drec, 0, sizeof(Rec) * ng, s));
            CK(hipEventRecord(e0, s));
            if (variant == 0)
                hipLaunchKernelGGL(k_plain, dim3(groups), dim3(kThreads), 0, s, in + off, io + off, (uint64_t)bytes, keep);
            else if (variant == 1)
                hipLaunchKernelGGL(k_traced, dim3(tgroups), dim3(kThreads), 0, s, in + off, io + off, (uint64_t)bytes,
                                   keep, drec, remap, n_even, n_odd);
            else if (variant == 2)
                hipLaunchKernelGGL(k_dyn<false>, dim3(pgroups), dim3(kThreads), 0, s, in + off, io + off,
                                   (uint64_t)bytes, keep, ctr, drec);
            else
                hipLaunchKernelGGL(k_dyn<true>, dim3(pgroups), dim3(kThreads), 0, s, in + off, io + off,
                                   (uint64_t)bytes, keep, ctr, drec);
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it < 5) continue;
            dur.push_back(ms * 1e3f);
            if (tr) {
                CK(hipMemcpy(rec.data(), drec, sizeof(Rec) * ng, hipMemcpyDeviceToHost));
                last.clear();
                for (unsigned g = 0; g < ng; ++g)
                    if (rec[g].t0) last.push_back(rec[g]);
                const std::vector<Rec> &v = last;
                const size_t nv = v.size();
                std::vector<unsigned long long> st(nv), en(nv);
                unsigned long long t0 = ~0ull, t1 = 0;
                for (size_t g = 0; g < nv; ++g) {
                    st[g] = v[g].t0;
                    en[g] = v[g].t1;
                    t0 = std::min(t0, v[g].t0);
                    t1 = std::max(t1, v[g].t1);
                    if (variant == 1 && (v[g].hw & 7u) != (v[g].xcc & 7u)) ++xcc_mismatch;
                }
                std::sort(st.begin(), st.end());
                std::sort(en.begin(), en.end());
                r50 += (pct(st, 0.5) - t0) * tick_us;
                r90 += (pct(st, 0.9) - t0) * tick_us;
                r100 += (pct(st, 1.0) - t0) * tick_us;
                e50 += (t1 - pct(en, 0.5)) * tick_us;
                e90 += (t1 - pct(en, 0.9)) * tick_us;
                span += (t1 - t0) * tick_us;
                first += (pct(en, 0.0) - t0) * tick_us;
                double b = 0;
                for (size_t g = 0; g < nv; ++g) b += (double)(v[g].t1 - v[g].t0) * tick_us;
                if (variant == 3)
                    for (size_t g = 0; g < nv; ++g) xtiles[v[g].xcc & 7] += v[g].hw;
                busy += b / nv;
                for (int x = 0; x < 8; ++x) {
                    unsigned long long a = ~0ull, z = 0;
                    for (size_t g = 0; g < nv; ++g)
                        if ((int)(v[g].xcc & 7) == x) {
                            a = std::min(a, v[g].t0);
                            z = std::max(z, v[g].t1);
                        }
                    if (z) {
                        xspan[x] += (z - a) * tick_us;
                        xmin_end[x] += (t1 - z) * tick_us;
                    }
                }
                ++traced;
            }
        }
        std::sort(dur.begin(), dur.end());
        double mean = 0;
        for (float d : dur) mean += d;
        mean /= dur.size();
        printf("%-10s %5u WGs event mean %7.2f us  median %7.2f  p10 %7.2f  p90 %7.2f  (%.4f of 8 TB/s)\n",
               vname[variant], ng, mean, dur[dur.size() / 2], dur[dur.size() / 10],
               dur[dur.size() * 9 / 10], 3.0 * bytes / (mean * 1e-6) / 8e12);
        if (tr && traced) {
            const double n = traced;
            printf("  first start -> last end %7.2f us; workgroup duration mean %6.2f us; first workgroup done at %6.2f us\n",
                   span / n, busy / n, first / n);
            printf("  starts: 50%% by %6.2f us, 90%% by %6.2f, all by %6.2f\n", r50 / n, r90 / n, r100 / n);
            printf("  ends:   last end - 50%% end %6.2f us, - 90%% end %6.2f\n", e50 / n, e90 / n);
            if (variant == 1) printf("  workgroups not on XCD blockIdx %% 8: %llu\n", xcc_mismatch);
            printf("  per XCD span (us):");
            for (int x = 0; x < 8; ++x) printf(" %6.2f", xspan[x] / n);
            printf("\n  per XCD finishes before the last (us):");
            for (int x = 0; x < 8; ++x) printf(" %5.2f", xmin_end[x] / n);
            printf("\n");
            if (variant == 3) {
                printf("  tiles per XCD:");
                for (int x = 0; x < 8; ++x) printf(" %7.0f", xtiles[x] / n);
                printf("\n");
            }
        }
    }
    // one launch's start / end histogram, 1 us bins
    {
        std::vector<int> hs(400, 0), he(400, 0);
        unsigned long long t0 = ~0ull;
        for (const Rec &r : last) t0 = std::min(t0, r.t0);
        for (const Rec &r : last) {
            int a = (int)((r.t0 - t0) * tick_us), z = (int)((r.t1 - t0) * tick_us);
            if (a < 400) hs[a]++;
            if (z < 400) he[z]++;
        }
        printf("last traced launch, per 1 us bin: us:started/finished\n ");
        for (int i = 0; i < 400; ++i)
            if (hs[i] || he[i]) printf(" %d:%d/%d", i, hs[i], he[i]);
        printf("\n");
    }
    return 0;
}
