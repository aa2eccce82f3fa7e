// mempool_race.hip -- does hipMallocAsync on one stream hand out memory that a
// hipFreeAsync on ANOTHER stream released while that stream's earlier work
// still reads it?  (The round-1 TREE combine fallback took its temporaries
// this way, one library stream per host thread, and MINLOC folds -- the pairs
// without a fused kernel, so the only users of that fallback -- came out
// corrupted when several threads ran at once; commit e7b5d60.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mempool_race.hip -o tools/mempool_race -lpthread
//   tools/mempool_race [iterations, default 300]
//
// T host threads, each with its own blocking stream, loop:
//   p = hipMallocAsync(4 MiB, s); fill(p, tag); delay kernel (~20 us, so the
//   free below is still pending on the GPU); copy(p -> own out); hipFreeAsync(p, s);
//   hipStreamSynchronize(s); check out == tag.
// Prints, per run: iterations, pointers handed to a thread while another
// thread's live block used the same address, and corrupted results.  Then the
// same loop with a per-thread hipMalloc'd buffer (what the product does now)
// as the control.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <atomic>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr size_t kN = (4u << 20) / 4;     // 4 MiB of uint32

__global__ void k_fill(unsigned *p, unsigned tag, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = tag;
}

__global__ void k_delay(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
}

__global__ void k_copy(const unsigned *p, unsigned *out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) out[i] = p[i];
}

std::mutex g_mu;
std::multiset<void *> g_live;
std::atomic<long> g_overlap{0}, g_bad{0};

static void worker(int tid, int iters, bool async_pool) {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    unsigned *out, *own = nullptr;
    CK(hipMalloc(&out, kN * 4));
    if (!async_pool) CK(hipMalloc(&own, kN * 4));
    std::vector<unsigned> host(kN);
    for (int it = 0; it < iters; ++it) {
        const unsigned tag = (unsigned)(tid << 24) | (unsigned)it;
        unsigned *p = own;
        if (async_pool) {
            CK(hipMallocAsync((void **)&p, kN * 4, s));
            std::lock_guard<std::mutex> lk(g_mu);
            if (g_live.count(p)) g_overlap++;
            g_live.insert(p);
        }
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, s, p, tag, kN);
        hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, 2000ull);   // 20 us at 100 MHz
        hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s, p, out, kN);
        if (async_pool) CK(hipFreeAsync(p, s));
        CK(hipStreamSynchronize(s));
        if (async_pool) {
            std::lock_guard<std::mutex> lk(g_mu);
            g_live.erase(g_live.find(p));
        }
        CK(hipMemcpy(host.data(), out, kN * 4, hipMemcpyDeviceToHost));
        size_t wrong = 0;
        for (size_t i = 0; i < kN; ++i) wrong += host[i] != tag;
        if (wrong) g_bad++;
    }
    CK(hipFree(out));
    if (own) CK(hipFree(own));
    CK(hipStreamDestroy(s));
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 300;
    for (int mode = 0; mode < 2; ++mode) {
        for (int T : {2, 4, 8}) {
            g_overlap = 0;
            g_bad = 0;
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back(worker, t, iters, mode == 0);
            for (auto &x : th) x.join();
            printf("%-32s threads %d iterations %d: address handed out while live elsewhere %ld, corrupted results %ld\n",
                   mode == 0 ? "hipMallocAsync/hipFreeAsync" : "per-thread hipMalloc (control)", T, iters,
                   g_overlap.load(), g_bad.load());
            fflush(stdout);
        }
    }
    return 0;
}
