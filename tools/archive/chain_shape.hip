// chain_shape.hip -- workgroup shape and LDS cap of the fused CHAIN folds of
// 3, 5, 6 and 7 operands (round 5: the library runs P = 5-7 in P = 8's shape,
// 1024 threads x 1 vector under a 96 KiB cap = one workgroup per CU, and P = 3
// in P = 4's, 256 threads x 4 vectors under a 53 KiB cap = three per CU).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/archive/chain_shape tools/archive/chain_shape.hip
//   tools/archive/chain_shape [rounds = 9] [chain | chainslab | chainskew | p2slab | p4slab | tree | p8 | slab | slabskew]
//
// fp16 SUM CHAIN over p blocks of 1 GiB / p (config 5's sendbuf at p ranks),
// two operand sets alternated, HIP events over batches of 10 back-to-back
// launches, shapes shuffled per round, first round dropped; every shape's
// output compared bit for bit with the library shape's.
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

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = (uint16_t)(x & 0xBFFF);
    }
}

struct Shape {
    const char *name;
    int th, u, lds;
};

template <class T, int P, bool TREE, int U, int TH>
void launch(const MultiArgs &a, int lds) {
    const uint64_t tile = (uint64_t)TH * U * 16;
    hipLaunchKernelGGL((k_combine_multi<OpSum, T, P, TREE, U, TH>), dim3((unsigned)(a.vbytes / tile)), dim3(TH),
                       lds, 0, a);
}

// T / TREE / total: CHAIN fp16 over 1 GiB (config 5's sendbuf) by default;
// TREE fp32 over `total` bytes for config 4's reduce-scatter blocks
template <int P, class T = f16, bool TREE = false>
void run(int rounds, uint64_t total = 1ull << 30, uint64_t slab_skew = 0) {
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, T, P, TREE, 1, 1024>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, T, P, TREE, 4, kThreads>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    const Shape shapes[] = {{"1024 x 1, 96 KiB cap (1 / CU)", 1024, 1, 96 << 10}, {"1024 x 1, no cap (2 / CU)", 1024, 1, 0},
                            {"256 x 4, 53 KiB cap (3 / CU)", 256, 4, 53 << 10}, {"256 x 4, 40 KiB cap (4 / CU)", 256, 4, 40 << 10},
                            {"256 x 4, no cap", 256, 4, 0}};
    constexpr int NS = 5;
    // the library: P = 5-8 in 1024 x 1, P = 3-4 in 256 x 4 capped, P = 2 uncapped
    const int lib = P >= 5 ? 0 : (P == 2 ? 4 : 2);
    const uint64_t block = (total / P) / 65536 * 65536;              // bytes, a multiple of both tiles
    // operand sets rotated over at least 1.5 GiB (past the 256 MB Infinity Cache)
    // slab_skew != 0: each set is one allocation holding the P blocks at stride
    // block + slab_skew and the output after them, as the collectives' staging
    // slots (coll_hip.c stage_stride); else one allocation per block
    const int nsets = std::max<int>(2, (int)((3ull << 29) / ((P + 1) * block) + 1));
    std::vector<char *> bufs(nsets * (P + 1)), slabs;
    if (slab_skew) {
        for (int set = 0; set < nsets; ++set) {
            char *b;
            CK(hipMalloc(&b, (P + 1) * (block + slab_skew)));
            slabs.push_back(b);
            for (int j = 0; j <= P; ++j) bufs[set * (P + 1) + j] = b + j * (block + slab_skew);
        }
    } else {
        for (auto &b : bufs) CK(hipMalloc(&b, block));
    }
    for (int i = 0; i < nsets * (P + 1); ++i) k_fill<<<2048, 256>>>((uint16_t *)bufs[i], block / 2, 0x99u + 13u * i);
    CK(hipDeviceSynchronize());
    auto args = [&](int set) {
        MultiArgs a{};
        for (int j = 0; j < P; ++j) a.in[j] = bufs[set * (P + 1) + j];
        a.out = bufs[set * (P + 1) + P];
        a.vbytes = block;
        a.keep = keep_for(block);
        return a;
    };
    auto go = [&](int si, int set) {
        const Shape &s = shapes[si];
        if (s.th == 1024) launch<T, P, TREE, 1, 1024>(args(set), s.lds);
        else launch<T, P, TREE, 4, kThreads>(args(set), s.lds);
    };
    std::vector<char> want(block), got(block);
    int bad = 0;
    go(lib, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(want.data(), bufs[P], block, hipMemcpyDeviceToHost));
    for (int si = 0; si < NS; ++si) {
        if (si == lib) continue;
        CK(hipMemset(bufs[P], 0, block));
        go(si, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), bufs[P], block, hipMemcpyDeviceToHost));
        if (memcmp(got.data(), want.data(), block)) ++bad;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> us[NS];
    std::mt19937 rng(P);
    const int batch = 10;
    int k = 0;
    for (int r = 0; r < rounds; ++r) {
        int order[NS];
        for (int i = 0; i < NS; ++i) order[i] = i;
        std::shuffle(order, order + NS, rng);
        for (int si : order) {
            go(si, k++ % nsets);
            CK(hipEventRecord(e0, 0));
            for (int b = 0; b < batch; ++b) go(si, k++ % nsets);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) us[si].push_back(ms * 1e3 / batch);
        }
    }
    printf("%s%d %s, %d x %.1f MiB, %d sets%s: outputs %s\n", TREE ? "TREE" : "CHAIN", P, sizeof(T) == 2 ? "fp16" : "fp32",
           P, block / 1048576.0, nsets, slab_skew ? ", staging slab" : ", one allocation per block",
           bad ? "DIFFER" : "identical");
    for (int si = 0; si < NS; ++si) {
        std::sort(us[si].begin(), us[si].end());
        const double med = us[si][us[si].size() / 2];
        printf("  %-32s%s median %8.2f us  frac of 8 TB/s %.4f\n", shapes[si].name, si == lib ? " (library)" : "          ",
               med, (P + 1.0) * block / (med * 1e-6) / 8e12);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    if (slab_skew) for (auto b : slabs) CK(hipFree(b));
    else for (auto b : bufs) CK(hipFree(b));
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 9;
    const char *mode = argc > 2 ? argv[2] : "chain";
    if (!strcmp(mode, "p2slab")) {
        // config 4 / 5 at 2 ranks in the staging slab: TREE2 fp32 2 x 128 MiB, CHAIN2 fp16 2 x 512 MiB
        run<2, float, true>(rounds, 256ull << 20, 6400);
        run<2, f16, false>(rounds, 1ull << 30, 4352);
        // the other sizes of the same two shapes
        run<2, float, true>(rounds, 1ull << 30, 4352);
        run<2, f16, false>(rounds, 256ull << 20, 6400);
    } else if (!strcmp(mode, "p4slab")) {
        // config 4 / 5 at 4 ranks in the staging slab: TREE4 fp32 4 x 64 MiB, CHAIN4 fp16 4 x 256 MiB
        run<4, float, true>(rounds, 256ull << 20, 4352);
        run<4, f16, false>(rounds, 1ull << 30, 4352);
    } else if (!strcmp(mode, "chainskew")) {
        // the pairwise chain at 6 and 7 ranks (171 / 146 MiB slots) at both skews
        for (uint64_t skew : {4352ull, 6400ull}) {
            printf("== slab skew %llu B\n", (unsigned long long)skew);
            run<6>(rounds, 1ull << 30, skew);
            run<7>(rounds, 1ull << 30, skew);
        }
    } else if (!strcmp(mode, "slabskew")) {
        // config 4 / 5's P = 8 folds in the staging slab at several skews
        for (uint64_t skew : {4352ull, 6400ull, 2097152ull, 2097408ull}) {
            printf("== slab skew %llu B\n", (unsigned long long)skew);
            run<8, float, true>(rounds, 256ull << 20, skew);
            run<8, f16, false>(rounds, 1ull << 30, skew);
        }
    } else if (!strcmp(mode, "chainslab")) {
        // the pairwise chain's operands as the collective lays them: one staging slab
        run<3>(rounds, 1ull << 30, 4352);
        run<5>(rounds, 1ull << 30, 4352);
        run<6>(rounds, 1ull << 30, 4352);
        run<7>(rounds, 1ull << 30, 4352);
    } else if (!strcmp(mode, "chain")) {
        run<3>(rounds);
        run<5>(rounds);
        run<6>(rounds);
        run<7>(rounds);
        run<8>(rounds);     // config 5 at 8 ranks: the library's P = 8 shape against the others
    } else if (!strcmp(mode, "tree")) {
        // config 4's reduce-scatter folds: TREE8 fp32 over 8 x 32 MiB, TREE4 over 4 x 64 MiB
        run<8, float, true>(rounds, 256ull << 20);
        run<4, float, true>(rounds, 256ull << 20);
    } else {
        // P = 8 by block size: 32 / 64 / 128 MiB blocks, TREE fp32 and CHAIN fp16;
        // mode "slab": the blocks in one allocation at the staging stride
        const uint64_t skew = !strcmp(mode, "slab") ? 4352 : 0;
        for (uint64_t mib : {32, 64, 128}) {
            run<8, float, true>(rounds, 8 * (mib << 20), skew);
            run<8, f16, false>(rounds, 8 * (mib << 20), skew);
        }
    }
    return 0;
}
