// fused_write_ab.hip -- round 4: does where (and how fast) the fused combine's one
// write stream lands decide its ~0.75?  DESIGN.md §(f) found the eight reads alone
// at 0.82-0.84 and the eight reads + one write at 0.75, in place over operand 0 or
// not, with the channels balanced; the write latency rose from 778 to 1181 cycles.
// Two hypotheses the earlier A/Bs did not separate:
//   (1) DRAM row locality of the writes: the results land in rows that no read has
//       open.  Variants put the output tile in place over the operand read last,
//       or interleave the nine tiles of one output (eight inputs + the output)
//       contiguously, so every write is next to the reads it follows;
//   (2) read pressure starving the writes: half the workgroups per CU (an LDS
//       reservation), half the reads in flight.
// Every kernel has the product's P = 8 shape (1024 threads, one 16 B vector per
// lane per operand, 16 KiB tile per operand per workgroup, nt loads and stores)
// and folds with XOR.  Timing: HIP events around batches of back-to-back launches
// over rotating operand sets (> Infinity Cache), variant order shuffled each round.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/fused_write_ab tools/fused_write_ab.hip
//   tools/fused_write_ab [MiB per operand = 128] [rounds = 8]
//   SWEEP=1 tools/fused_write_ab ...   workgroup size x workgroups per CU sweep (k_occ)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int TH = 1024;
constexpr uint32_t TILE = TH * 16;
constexpr int P = 8;

struct Args {
    char *base;         // the set's 9 regions of vbytes (or 9 interleaved tiles per output tile)
    uint64_t vbytes;    // bytes per operand
    uint64_t skew;      // region stride = vbytes + skew
};

__device__ __forceinline__ u32x4 ld(const char *p, int off) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, TILE, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
}
__device__ __forceinline__ void st(char *p, int off, u32x4 v) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, TILE, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 2);
}

// MODE 0: staging layout, separate output (region 8)            -- the product's case
// MODE 1: staging layout, result over operand 7's tile (read last)
// MODE 2: interleaved: output tile t's 8 inputs and its output contiguous
//         ((t * 9 + j) * TILE), output in slot 8
// MODE 3: interleaved, result over slot 7 (in place, last read)
// MODE 4: staging layout, 8 reads, no write (one word per workgroup)
template <int MODE>
__global__ __launch_bounds__(TH) void k_fold(Args a, uint32_t *sink) {
    extern __shared__ char lds_cap[];          // dynamic LDS: only caps workgroups per CU
    const uint64_t t = blockIdx.x;
    const uint64_t base = t * TILE;
    if (base >= a.vbytes) return;
    const int off = (int)threadIdx.x * 16;
    const uint64_t stride = a.vbytes + a.skew;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const char *p = (MODE == 2 || MODE == 3) ? a.base + (t * 9 + j) * TILE : a.base + j * stride + base;
        acc ^= ld(p, off);
    }
    if (MODE == 4) {
        if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = (uint32_t)t;
        if (threadIdx.x == 0 && lds_cap[0] == 1) sink[1] = 1;
        return;
    }
    char *o = MODE == 0 ? a.base + 8 * stride + base
            : MODE == 1 ? a.base + 7 * stride + base
            : MODE == 2 ? a.base + (t * 9 + 8) * TILE
                        : a.base + (t * 9 + 7) * TILE;
    st(o, off, acc);
}

// occupancy sweep: TH threads per workgroup, one 16 B vector per lane per
// operand (TH * 16 B tile per operand), PP operands, separate output; the
// launch's dynamic LDS caps the workgroups per CU
template <int TH_, int PP>
__global__ __launch_bounds__(TH_) void k_occ(Args a, uint32_t *sink) {
    extern __shared__ char lds_cap[];
    constexpr uint32_t T = TH_ * 16;
    const uint64_t base = (uint64_t)blockIdx.x * T;
    if (base >= a.vbytes) return;
    const int off = (int)threadIdx.x * 16;
    const uint64_t stride = a.vbytes + a.skew;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < PP; ++j) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.base + j * stride + base), 0, T, 0x00020000);
        acc ^= __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
    }
    __amdgpu_buffer_rsrc_t o = __builtin_amdgcn_make_buffer_rsrc((void *)(a.base + 8 * stride + base), 0, T, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc, o, off, 0, 2);
    (void)sink;
}

__global__ void k_fill(uint32_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = x;
    }
}

struct Var {
    const char *name;
    void (*k)(Args, uint32_t *);
    size_t lds;
    int writes;
    int th = TH;
    int p = P;
};

int main(int argc, char **argv) {
    const uint64_t mib = argc > 1 ? atoi(argv[1]) : 128;
    const int rounds = argc > 2 ? atoi(argv[2]) : 8;
    const uint64_t vbytes = mib << 20, skew = 4352;
    const uint64_t setbytes = 9 * (vbytes + skew);
    const int nsets = (int)std::max<uint64_t>(2, (3ull << 30) / setbytes + 1);
    std::vector<char *> sets(nsets);
    for (auto &s : sets) {
        CK(hipMalloc(&s, setbytes));
        k_fill<<<4096, 256>>>((uint32_t *)s, setbytes / 4, (uint32_t)(uintptr_t)s);
    }
    uint32_t *sink;
    CK(hipMalloc(&sink, 64));
    CK(hipDeviceSynchronize());
    const Var vars[] = {
        {"separate_out", k_fold<0>, 0, 1},
        {"inplace_last", k_fold<1>, 0, 1},
        {"interleaved9_out", k_fold<2>, 0, 1},
        {"interleaved9_inplace_last", k_fold<3>, 0, 1},
        {"separate_out_1wg_per_cu", k_fold<0>, 96 << 10, 1},
        {"read_only8", k_fold<4>, 0, 0},
        {"read_only8_1wg_per_cu", k_fold<4>, 96 << 10, 0},
    };
    const Var sweep[] = {
        // P = 8, in flight per CU = workgroups x TH x 128 B
        {"p8_t1024_x2(256K)", k_occ<1024, 8>, 0, 1, 1024, 8},
        {"p8_t1024_x1(128K)", k_occ<1024, 8>, 96 << 10, 1, 1024, 8},
        {"p8_t512_x4(256K)", k_occ<512, 8>, 0, 1, 512, 8},
        {"p8_t512_x3(192K)", k_occ<512, 8>, 48 << 10, 1, 512, 8},
        {"p8_t512_x2(128K)", k_occ<512, 8>, 64 << 10, 1, 512, 8},
        {"p8_t512_x1(64K)", k_occ<512, 8>, 96 << 10, 1, 512, 8},
        {"p8_t256_x6(96K)", k_occ<256, 8>, 26 << 10, 1, 256, 8},
        {"p8_t256_x5(80K)", k_occ<256, 8>, 32 << 10, 1, 256, 8},
        {"p8_t256_x4(64K)", k_occ<256, 8>, 40 << 10, 1, 256, 8},
        // P = 4
        {"p4_t1024_x2(128K)", k_occ<1024, 4>, 0, 1, 1024, 4},
        {"p4_t1024_x1(64K)", k_occ<1024, 4>, 96 << 10, 1, 1024, 4},
        {"p4_t512_x3(96K)", k_occ<512, 4>, 48 << 10, 1, 512, 4},
    };
    const bool do_sweep = getenv("SWEEP") != nullptr;
    const Var *vv = do_sweep ? sweep : vars;
    const int nvv = do_sweep ? (int)(sizeof(sweep) / sizeof(sweep[0])) : (int)(sizeof(vars) / sizeof(vars[0]));
    const int nv = nvv;
    for (int i = 0; i < nv; ++i)
        if (vv[i].lds) CK(hipFuncSetAttribute((const void *)vv[i].k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)vv[i].lds));
    const int batch = 24;
    std::vector<std::vector<double>> us(nv);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::mt19937 rng(7);
    std::vector<int> order(nv);
    for (int i = 0; i < nv; ++i) order[i] = i;
    int si = 0;
    for (int r = 0; r < rounds + 1; ++r) {
        std::shuffle(order.begin(), order.end(), rng);
        for (int v : order) {
            const unsigned grid = (unsigned)(vbytes / (vv[v].th * 16));
            for (int b = 0; b < 2; ++b) hipLaunchKernelGGL(vv[v].k, dim3(grid), dim3(vv[v].th), vv[v].lds, 0,
                                                         Args{sets[si++ % nsets], vbytes, skew}, sink);
            CK(hipEventRecord(e0));
            for (int b = 0; b < batch; ++b) hipLaunchKernelGGL(vv[v].k, dim3(grid), dim3(vv[v].th), vv[v].lds, 0,
                                                             Args{sets[si++ % nsets], vbytes, skew}, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) us[v].push_back(ms * 1e3 / batch);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("fused_write_ab: P = 8, %llu MiB per operand, skew %llu B, %d sets, %d rounds x %d back-to-back launches\n",
           (unsigned long long)mib, (unsigned long long)skew, nsets, rounds, batch);
    for (int v = 0; v < nv; ++v) {
        auto x = us[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        const double bytes = (double)vbytes * (vv[v].p + vv[v].writes);
        printf("%-28s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f (min-time %.4f)\n", vv[v].name, med, x[0],
               bytes / (med * 1e-6) / 8e12, bytes / (x[0] * 1e-6) / 8e12);
    }
    return 0;
}
