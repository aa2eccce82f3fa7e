// tail_xcd_trace.hip -- where do the headline loop's isolated slow launches
// lose their time?  (after the UTCL counters came out equal.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpich-pip_amd/csrc/hip \
//         tools/tail_xcd_trace.hip -o tools/tail_xcd_trace
//   tools/tail_xcd_trace [launches, default 600]
//
// The product tile body (reduce_tile<OpSum,float>, 256 MiB fp32 per operand,
// 16,384 workgroups) over 4 rotating operand pairs, back to back on one
// stream; every workgroup's thread 0 records the 100 MHz wall clock at its start
// and after its stores completed, and its XCC id.  Per launch: span (first
// start to last end), per-XCD last end, and the longest gap in which no
// workgroup of an XCD finished.  Launches slower than the median span + 4 us
// are compared with the rest: is one XCD late (a per-XCD stall), or all of them
// (a chip-wide stall), and when in the launch does the stall sit?
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
    unsigned int blk, xcc;
};

__device__ __forceinline__ unsigned long long wall() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(kThreads) void k_traced(const char *in, char *io, uint64_t vbytes, Rec *rec) {
    const unsigned long long t0 = wall();
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        Rec r;
        r.t0 = t0;
        r.t1 = wall();
        r.blk = blockIdx.x;
        r.xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
        rec[blockIdx.x] = r;
    }
}

int main(int argc, char **argv) {
    const int launches = argc > 1 ? atoi(argv[1]) : 600;
    const uint64_t bytes = 256ull << 20;
    const unsigned groups = (unsigned)(bytes / kTileBytes);
    const int npairs = 4;
    char *buf[2 * npairs];
    for (auto &b : buf) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 0, bytes));
    }
    Rec *rec;
    CK(hipMalloc(&rec, sizeof(Rec) * groups * (size_t)launches));
    CK(hipDeviceSynchronize());
    for (int i = 0; i < 20; ++i)
        k_traced<<<groups, kThreads>>>(buf[2 * (i % npairs)], buf[2 * (i % npairs) + 1], bytes, rec);
    CK(hipDeviceSynchronize());
    for (int i = 0; i < launches; ++i)
        k_traced<<<groups, kThreads>>>(buf[2 * (i % npairs)], buf[2 * (i % npairs) + 1], bytes,
                                       rec + (size_t)i * groups);
    CK(hipDeviceSynchronize());
    std::vector<Rec> h((size_t)groups * launches);
    CK(hipMemcpy(h.data(), rec, sizeof(Rec) * h.size(), hipMemcpyDeviceToHost));

    struct L {
        double span, start_spread, xlate[8], xgap[8], gap_at;
        int late_x;
    };
    std::vector<L> ls(launches);
    for (int i = 0; i < launches; ++i) {
        const Rec *r = &h[(size_t)i * groups];
        unsigned long long s0 = ~0ull, e1 = 0;
        unsigned long long xe[8] = {}, xs[8];
        for (int x = 0; x < 8; ++x) xs[x] = ~0ull;
        std::vector<unsigned long long> ends[8];
        for (unsigned g = 0; g < groups; ++g) {
            s0 = std::min(s0, r[g].t0);
            e1 = std::max(e1, r[g].t1);
            const int x = r[g].xcc & 7;
            xe[x] = std::max(xe[x], r[g].t1);
            xs[x] = std::min(xs[x], r[g].t0);
            ends[x].push_back(r[g].t1);
        }
        L &l = ls[i];
        l.span = (e1 - s0) * 0.01;
        unsigned long long xs_max = 0;
        for (int x = 0; x < 8; ++x) xs_max = std::max(xs_max, xs[x]);
        l.start_spread = (xs_max - s0) * 0.01;
        std::vector<unsigned long long> xes(xe, xe + 8);
        std::sort(xes.begin(), xes.end());
        const double med_end = (xes[3] + xes[4]) * 0.5;
        l.late_x = 0;
        double g_best = 0;
        for (int x = 0; x < 8; ++x) {
            l.xlate[x] = (xe[x] - med_end) * 0.01;
            if (l.xlate[x] > l.xlate[l.late_x]) l.late_x = x;
            std::sort(ends[x].begin(), ends[x].end());
            double gmax = 0, gat = 0;
            for (size_t k = 1; k < ends[x].size(); ++k) {
                const double gap = (ends[x][k] - ends[x][k - 1]) * 0.01;
                if (gap > gmax) {
                    gmax = gap;
                    gat = (ends[x][k - 1] - s0) * 0.01;
                }
            }
            l.xgap[x] = gmax;
            if (gmax > g_best) {
                g_best = gmax;
                l.gap_at = gat;
            }
        }
    }
    std::vector<double> spans;
    for (auto &l : ls) spans.push_back(l.span);
    std::sort(spans.begin(), spans.end());
    const double med = spans[spans.size() / 2];
    int nslow = 0;
    double fast_gap = 0, slow_gap = 0, fast_late = 0, slow_late = 0, fast_ss = 0, slow_ss = 0;
    int nfast = 0;
    printf("launches %d, median span %.2f us, p90 %.2f, max %.2f\n", launches, med, spans[spans.size() * 9 / 10],
           spans.back());
    for (int i = 0; i < launches; ++i) {
        const L &l = ls[i];
        double mg = 0;
        for (int x = 0; x < 8; ++x) mg = std::max(mg, l.xgap[x]);
        if (l.span > med + 4.0) {
            ++nslow;
            slow_gap += mg;
            slow_late += l.xlate[l.late_x];
            slow_ss += l.start_spread;
            printf("slow launch %3d: span %.2f (+%.2f)  start spread %.2f  latest XCD %d +%.2f us past the median "
                   "XCD end  per-XCD late [", i, l.span, l.span - med, l.start_spread, l.late_x, l.xlate[l.late_x]);
            for (int x = 0; x < 8; ++x) printf("%s%.1f", x ? " " : "", l.xlate[x]);
            printf("]  longest no-completion gap %.2f us at +%.1f us\n", mg, l.gap_at);
        } else if (l.span <= med) {
            ++nfast;
            fast_gap += mg;
            fast_late += l.xlate[l.late_x];
            fast_ss += l.start_spread;
        }
    }
    printf("fast (<= median) %d: mean longest gap %.2f us, latest XCD +%.2f us, start spread %.2f us\n", nfast,
           fast_gap / std::max(nfast, 1), fast_late / std::max(nfast, 1), fast_ss / std::max(nfast, 1));
    printf("slow (> median + 4 us) %d: mean longest gap %.2f us, latest XCD +%.2f us, start spread %.2f us\n", nslow,
           slow_gap / std::max(nslow, 1), slow_late / std::max(nslow, 1), slow_ss / std::max(nslow, 1));
    return 0;
}
