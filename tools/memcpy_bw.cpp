// memcpy_bw.cpp -- host memcpy bandwidth pageable -> pinned (hipHostMalloc) and
// back with T threads, the CPU half of a bounce-buffer staging of pageable
// operands.   hipcc -O2 -o tools/memcpy_bw tools/memcpy_bw.cpp -lpthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t n = 256ull << 20;
    char *pg = (char *)aligned_alloc(4096, n);
    memset(pg, 1, n);
    char *pin;
    if (hipHostMalloc((void **)&pin, n, 0) != hipSuccess) return 2;
    memset(pin, 2, n);
    for (int T : {1, 2, 4, 8, 16}) {
        for (int dir = 0; dir < 2; ++dir) {
            double best = 1e9;
            for (int rep = 0; rep < 5; ++rep) {
                double t0 = now();
                std::vector<std::thread> th;
                for (int k = 0; k < T; ++k)
                    th.emplace_back([=] {
                        const size_t a = n / T * k, b = k == T - 1 ? n : n / T * (k + 1);
                        if (dir == 0) memcpy(pin + a, pg + a, b - a);
                        else memcpy(pg + a, pin + a, b - a);
                    });
                for (auto &x : th) x.join();
                best = std::min(best, now() - t0);
            }
            printf("T=%2d %s %.1f GB/s\n", T, dir ? "pinned->pageable" : "pageable->pinned", n / best / 1e9);
        }
    }
    return 0;
}
