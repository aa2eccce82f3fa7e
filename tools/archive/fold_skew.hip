// fold_skew.hip -- the fused folds' operand layout: the staging slots' skew.
// The collectives land received blocks in staging slots `stage_stride()` apart
// (coll_hip.c: block + 4352 B for blocks of 1 MiB or more, chosen in round 1
// from four skews).  Here the library's own fold kernel (k_combine_multi, 96 KiB
// LDS = one 1024-thread workgroup per CU, as launch_combine_pu launches it)
// runs over eight operands at stride block + skew for a wider set of skews, the
// output right after the eighth slot (as bench.py's config5_combine lays it).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/archive/fold_skew tools/archive/fold_skew.hip
//   tools/archive/fold_skew [rounds = 9]
//
// CHAIN8 fp16 and TREE8 fp32 over 8 blocks of 32-256 MiB (configs 5 and 4 at
// 8 ranks: 128 / 32 MiB), CHAIN4 / TREE4 at config 5 / 4's 4-rank sizes; sets
// rotated past the 256 MB Infinity Cache; HIP events over batches of 20
// back-to-back launches, skews shuffled per round, first round dropped; each
// skew's output compared bit for bit with skew 4352's on the same values.
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

__global__ void k_fill_block(uint16_t *p, uint64_t n, uint32_t seed, int f16) {
    // values depend on (seed, index in the block) only, so every layout folds the same numbers
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = f16 ? (uint16_t)(x & 0xBFFF) : (uint16_t)((i & 1) ? ((x & 0x803F) | 0x3E00) : x);
    }
}

const uint64_t kSkews[] = {256, 2304, 4352, 6400, 8448, 2097408};
constexpr int kNS = sizeof(kSkews) / sizeof(kSkews[0]);
constexpr int kLib = 2;                                 // 4352: stage_stride()'s

// the library's own launch (launch_combine_pu: P = 8 as 1024 x 1 with the
// 96 KiB cap, P = 4 as 256 x 4 with the 53 KiB cap)
template <class T, int P, bool TREE>
void launch_lib(const char *const *ins, char *out, uint64_t count) {
    constexpr int U = P >= 8 ? 1 : 4, TH = P >= 8 ? 1024 : kThreads;
    const void *v[kMaxOperands];
    for (int j = 0; j < P; ++j) v[j] = ins[j];
    CK((launch_combine_pu<OpSum, T, P, TREE, U, TH>(v, out, count, nullptr)));
}

template <class T, int P, bool TREE>
void run_case(const char *name, uint64_t block, int nsets, int rounds) {
    const uint64_t maxskew = kSkews[kNS - 1];
    const uint64_t setbytes = P * (block + maxskew) + block + 4096;
    std::vector<char *> sets(nsets);
    for (auto &p : sets) CK(hipMalloc(&p, setbytes));
    auto launch = [&](char *b, uint64_t skew) {
        const char *ins[P];
        for (int j = 0; j < P; ++j) ins[j] = b + j * (block + skew);
        launch_lib<T, P, TREE>(ins, b + P * (block + skew), block / sizeof(T));
    };
    // bit check: the same values at every skew give the same bytes
    std::vector<char> want(block), got(block);
    int bad = 0;
    auto fold_at = [&](int si, std::vector<char> &dst) {
        char *b = sets[0];
        for (int j = 0; j < P; ++j)
            k_fill_block<<<2048, 256>>>((uint16_t *)(b + j * (block + kSkews[si])), block / 2, 0x1234u + 77u * j,
                                        sizeof(T) == 2);
        launch(b, kSkews[si]);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(dst.data(), b + P * (block + kSkews[si]), block, hipMemcpyDeviceToHost));
    };
    fold_at(kLib, want);
    for (int si = 0; si < kNS; ++si)
        if (si != kLib) {
            fold_at(si, got);
            if (memcmp(got.data(), want.data(), block) != 0) ++bad;
        }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> us[kNS];
    std::mt19937 rng(11);
    int k = 0;
    const int batch = 20;
    for (int r = 0; r < rounds; ++r) {
        int order[kNS];
        for (int i = 0; i < kNS; ++i) order[i] = i;
        std::shuffle(order, order + kNS, rng);
        for (int si : order) {
            launch(sets[k++ % nsets], kSkews[si]);
            CK(hipEventRecord(e0, 0));
            for (int b = 0; b < batch; ++b) launch(sets[k++ % nsets], kSkews[si]);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) us[si].push_back(ms * 1e3 / batch);
        }
    }
    printf("%s: %d sets rotated, %d rounds x %d launches (first dropped); outputs %s\n", name, nsets, rounds, batch,
           bad ? "DIFFER" : "identical at every skew");
    for (int si = 0; si < kNS; ++si) {
        std::sort(us[si].begin(), us[si].end());
        const double med = us[si][us[si].size() / 2];
        printf("  skew %8llu B%s  median %8.2f us (min %8.2f, max %8.2f)  frac of 8 TB/s %.4f\n",
               (unsigned long long)kSkews[si], si == kLib ? " (library)" : "          ", med, us[si].front(),
               us[si].back(), (P + 1.0) * block / (med * 1e-6) / 8e12);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    for (auto p : sets) CK(hipFree(p));
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 9;
    const uint64_t M = 1ull << 20;
    run_case<f16, 8, false>("CHAIN8 fp16 8 x 128 MiB (config 5, 8 ranks)", 128 * M, 3, rounds);
    run_case<f16, 8, false>("CHAIN8 fp16 8 x 64 MiB", 64 * M, 5, rounds);
    run_case<f16, 8, false>("CHAIN8 fp16 8 x 256 MiB", 256 * M, 3, rounds);
    run_case<float, 8, true>("TREE8 fp32 8 x 32 MiB (config 4, 8 ranks)", 32 * M, 10, rounds);
    run_case<float, 8, true>("TREE8 fp32 8 x 64 MiB", 64 * M, 5, rounds);
    run_case<float, 8, true>("TREE8 fp32 8 x 128 MiB", 128 * M, 3, rounds);
    run_case<f16, 4, false>("CHAIN4 fp16 4 x 256 MiB (config 5, 4 ranks)", 256 * M, 3, rounds);
    run_case<float, 4, true>("TREE4 fp32 4 x 64 MiB (config 4, 4 ranks)", 64 * M, 6, rounds);
    return 0;
}
