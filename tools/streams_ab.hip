// streams_ab.hip -- HBM efficiency against the number of concurrent streams,
// to explain the fused combine's ~0.75 (configs 4-5) against the two-operand
// kernel's ~0.83.  Every kernel has the fused kernel's shape (1024 threads,
// one 16 B vector per lane per operand, a 16 KiB tile per operand per
// workgroup) and folds with XOR (no floating point):
//   k_rw<P, IL>   P operand tiles read, one written (P + 1 streams)
//   k_ro<P, IL>   P read, nothing but one word per workgroup written
// IL = 0: operand j at base + j * (block + skew)  (the staging layout)
// IL = 1: the P tiles of one output tile adjacent (tile t of operand j at
//         (t * P + j) * 16 KiB): one read stream whatever P is
// Operand sets rotate (NSETS, default so that >= 2 GiB), so nothing is found in
// the Infinity Cache.  Run under rocprofv3 --kernel-trace; tools/streams_ab.sh
// turns the trace into fractions of 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Impich-pip_amd/csrc/hip -o tools/streams_ab tools/streams_ab.hip
//   tools/streams_ab [MiB per operand = 32] [rounds = 20] [skew = 4352]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int TH = 1024;
constexpr uint32_t TILE = TH * 16;   // 16 KiB per operand per workgroup

struct Args {
    const char *in[16];
    char *out;
    uint32_t *sink;
    uint64_t vbytes;   // bytes per operand
};

template <int P, int IL>
__device__ __forceinline__ u32x4 fold(const Args &a, uint64_t base, int off) {
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const char *p = IL ? a.in[0] + (base * P + (uint64_t)j * TILE) : a.in[j] + base;
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, TILE, 0x00020000);
        acc ^= __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
    }
    return acc;
}

template <int P, int IL>
__global__ __launch_bounds__(TH) void k_rw(Args a) {
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    if (base >= a.vbytes) return;
    const int off = (int)threadIdx.x * 16;
    const u32x4 v = fold<P, IL>(a, base, off);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, TILE, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 2);
}

// the result written over operand 0's tile (in place, as MPI_Reduce_local
// writes inoutbuf): P reads + 1 write, the write to rows just read
template <int P>
__global__ __launch_bounds__(TH) void k_rwip(Args a) {
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    if (base >= a.vbytes) return;
    const int off = (int)threadIdx.x * 16;
    const u32x4 v = fold<P, 0>(a, base, off);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[0] + base), 0, TILE, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 2);
}

template <int P, int IL>
__global__ __launch_bounds__(TH) void k_ro(Args a) {
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    if (base >= a.vbytes) return;
    const int off = (int)threadIdx.x * 16;
    const u32x4 v = fold<P, IL>(a, base, off);
    const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
    if (x == 0x9e3779b9u) a.sink[blockIdx.x & 1023] = x;   // practically never: keeps the loads
}

// K consecutive tiles per workgroup: all K x P loads first, then the K tile
// stores back to back (fewer, larger write bursts per workgroup); `policy`
// is the store's cache-policy bits (2 = nt, 16 = sc1)
template <int P, int K, int POL>
__global__ __launch_bounds__(TH) void k_rwk(Args a) {
    const uint64_t base0 = (uint64_t)blockIdx.x * TILE * K;
    if (base0 >= a.vbytes) return;
    const int off = (int)threadIdx.x * 16;
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = fold<P, 0>(a, base0 + (uint64_t)k * TILE, off);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base0 + (uint64_t)k * TILE), 0, TILE, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v[k], ro, off, 0, POL);
    }
}

typedef void (*kfn)(Args);
struct Var { std::string name; kfn k; int P; int IL; int K = 1; };

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 32;
    const int rounds = argc > 2 ? atoi(argv[2]) : 20;
    const size_t skew = argc > 3 ? strtoull(argv[3], 0, 10) : 4352;
    const size_t bytes = mib << 20;
    constexpr int PM = 8;
    const int NS = getenv("NSETS") ? std::max(2, atoi(getenv("NSETS")))
                                   : (int)std::max<size_t>(2, (2048 + (PM + 1) * mib - 1) / ((PM + 1) * mib));
    // set s: PM operands at a (block + skew) stride, then the interleaved copy, then the output
    const size_t set_bytes = PM * (bytes + skew) + PM * bytes + bytes + 3 * 4096;
    char *big = nullptr;
    CK(hipMalloc(&big, set_bytes * NS));
    CK(hipMemset(big, 0x5a, set_bytes * NS));
    uint32_t *sink = nullptr;
    CK(hipMalloc(&sink, 4096 * 4));
    std::vector<Args> sep(NS), il(NS);
    for (int s = 0; s < NS; ++s) {
        char *b = big + (size_t)s * set_bytes;
        for (int j = 0; j < 16; ++j) sep[s].in[j] = j < PM ? b + (size_t)j * (bytes + skew) : nullptr;
        char *ilb = b + PM * (bytes + skew) + 4096;
        char *out = ilb + PM * bytes + 4096;
        for (int j = 0; j < 16; ++j) il[s].in[j] = j == 0 ? ilb : nullptr;
        sep[s].out = il[s].out = out;
        sep[s].sink = il[s].sink = sink;
        sep[s].vbytes = il[s].vbytes = bytes;
    }
    std::vector<Var> vs = {
        {"rw P1", k_rw<1, 0>, 1, 0}, {"rw P2", k_rw<2, 0>, 2, 0}, {"rw P4", k_rw<4, 0>, 4, 0},
        {"rw P8", k_rw<8, 0>, 8, 0}, {"rw P8 interleaved", k_rw<8, 1>, 8, 1}, {"rw P4 interleaved", k_rw<4, 1>, 4, 1},
        {"ro P2", k_ro<2, 0>, 2, 0}, {"ro P4", k_ro<4, 0>, 4, 0}, {"ro P8", k_ro<8, 0>, 8, 0},
        {"ro P8 interleaved", k_ro<8, 1>, 8, 1},
        {"rwk P8 K2", k_rwk<8, 2, 2>, 8, 0, 2}, {"rwk P8 K4", k_rwk<8, 4, 2>, 8, 0, 4},
        {"rwk P8 K1 sc1", k_rwk<8, 1, 16>, 8, 0, 1}, {"rwk P8 K2 sc1", k_rwk<8, 2, 16>, 8, 0, 2},
        {"rwk P2 K2", k_rwk<2, 2, 2>, 2, 0, 2},
        {"rwk P1 sc1", k_rwk<1, 1, 16>, 1, 0, 1}, {"rwk P2 sc1", k_rwk<2, 1, 16>, 2, 0, 1},
        {"rwk P4 sc1", k_rwk<4, 1, 16>, 4, 0, 1},
        {"rwip P1", k_rwip<1>, 1, 0}, {"rwip P2", k_rwip<2>, 2, 0}, {"rwip P4", k_rwip<4>, 4, 0},
        {"rwip P8", k_rwip<8>, 8, 0},
    };
    if (getenv("ONLY_RW")) {   // the rw / rwip / ro strided variants only
        std::vector<Var> keep;
        for (auto &v : vs)
            if (!v.IL && v.K == 1 && v.name.find("sc1") == std::string::npos) keep.push_back(v);
        vs = keep;
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::vector<int> order(vs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    uint32_t rs = 99;
    int slot = 0;
    const unsigned grid = (unsigned)((bytes + TILE - 1) / TILE);
    for (int r = -2; r < rounds; ++r) {
        for (size_t i = order.size() - 1; i > 0; --i) {
            rs = rs * 1664525u + 1013904223u;
            std::swap(order[i], order[(rs >> 8) % (i + 1)]);
        }
        for (int vi : order) {
            const int s = slot++ % NS;
            hipLaunchKernelGGL(vs[vi].k, dim3((grid + vs[vi].K - 1) / vs[vi].K), dim3(TH), 0, st, vs[vi].IL ? il[s] : sep[s]);
            CK(hipGetLastError());
            CK(hipStreamSynchronize(st));
        }
    }
    printf("%zu MiB per operand, skew %zu B, %d sets, %d rounds\n", mib, skew, NS, rounds);
    // BATCH=1: each variant timed over `rounds` back-to-back launches (sets
    // rotating) between two events, so stores an sc1 policy leaves dirty in the
    // Infinity Cache are paid by the batch, not by whichever kernel runs next
    if (getenv("BATCH")) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int pass = 0; pass < 2; ++pass) {
            for (size_t vi = 0; vi < vs.size(); ++vi) {
                const Var &v = vs[vi];
                const unsigned g = (grid + v.K - 1) / v.K;
                for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(v.k, dim3(g), dim3(TH), 0, st, v.IL ? il[w % NS] : sep[w % NS]);
                CK(hipEventRecord(e0, st));
                for (int r = 0; r < rounds; ++r)
                    hipLaunchKernelGGL(v.k, dim3(g), dim3(TH), 0, st, v.IL ? il[r % NS] : sep[r % NS]);
                CK(hipEventRecord(e1, st));
                CK(hipStreamSynchronize(st));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / rounds;
                const bool ro = v.name.rfind("ro", 0) == 0;
                const double alg = (double)(v.P + (ro ? 0 : 1)) * bytes;
                if (pass) printf("batch %-20s %8.2f us per launch  frac %.3f\n", v.name.c_str(), us, alg / us / 8e6);
            }
        }
    }
    return 0;
}
