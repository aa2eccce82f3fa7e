// concurrent_probe.cpp -- does a dispatch in flight on the queue shorten the
// ~4.3 us from doorbell to a new kernel running (DESIGN.md §Synchronous
// return)?  A one-wave `stamp` kernel writes a word to host memory when it
// runs; the host times doorbell -> word seen.  Cases (medians of K calls):
//   idle b0 / b1        nothing in flight; the stamp packet's barrier bit 0 / 1
//   keeper b0 / b1      a one-wave `keeper` kernel is already running on the
//                       same queue (the host waits until it has stamped its
//                       start); the stamp packet goes behind it, barrier 0 / 1;
//                       the host stops the keeper once the word is seen
//   other-queue b0      the keeper runs on a second queue
// Also reported: the stamp kernel's start minus the keeper's end on the GPU's
// 100 MHz clock (negative = the two ran concurrently) and the CP's own
// doorbell -> dispatch-start for the stamp packet.
//   bash tools/aql/build_concurrent.sh
//   HSA_ALLOCATE_QUEUE_DEV_MEM=1 tools/aql/concurrent_probe tools/aql/concurrent_kernels.co
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>

#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_; hsa_status_string(s_, &m_); \
    printf("HSA %s line %d: %s\n", #x, __LINE__, m_); exit(3);} } while (0)

static hsa_agent_t g_gpu, g_cpu;
static bool g_have_gpu = false, g_have_cpu = false;
static hsa_amd_memory_pool_t g_kern, g_fine;
static bool g_have_kern = false, g_have_fine = false;
static uint64_t g_freq = 0;

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) { g_cpu = a; g_have_cpu = true; }
    if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) { g_gpu = a; g_have_gpu = true; }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_pools(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t f = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &f);
    if ((f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_kern) { g_kern = p; g_have_kern = true; }
    if ((f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !g_have_fine) { g_fine = p; g_have_fine = true; }
    return HSA_STATUS_SUCCESS;
}

static uint64_t ts() {
    uint64_t t = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    return t;
}
static double us(uint64_t dt) { return (double)(int64_t)dt * 1e6 / (double)g_freq; }

static void post(hsa_queue_t *q, uint64_t ko, void *karg, hsa_signal_t sig, bool barrier) {
    const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    p->workgroup_size_x = 64;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->grid_size_x = 64;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->kernel_object = ko;
    p->kernarg_address = karg;
    p->completion_signal = sig;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    hsa_queue_store_write_index_relaxed(q, idx + 1);
    __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, idx);
}

// bounded waits: anything that never lands ends the run
static void wait_sig(hsa_signal_t s) {
    const uint64_t t0 = ts();
    while (hsa_signal_load_scacquire(s) != 0) {
        _mm_pause();
        if (us(ts() - t0) > 2e6) { printf("timeout waiting for a completion signal\n"); fflush(stdout); _exit(4); }
    }
}
template <class T> static void wait_word(volatile T *w, T v) {
    const uint64_t t0 = ts();
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != v) {
        _mm_pause();
        if (us(ts() - t0) > 2e6) { printf("timeout waiting for a word\n"); fflush(stdout); _exit(4); }
    }
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: %s concurrent_kernels.co\n", argv[0]); return 1; }
    setvbuf(stdout, nullptr, _IOLBF, 0);
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    hsa_amd_agent_iterate_memory_pools(g_cpu, find_pools, nullptr);
    if (!g_have_gpu || !g_have_kern || !g_have_fine) { printf("agents / pools not found\n"); return 1; }
    HK(hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &g_freq));
    FILE *f = fopen(argv[1], "rb");
    if (!f) { printf("cannot open %s\n", argv[1]); return 1; }
    std::vector<char> co;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) co.insert(co.end(), buf, buf + n);
    fclose(f);
    hsa_code_object_reader_t rd;
    hsa_executable_t exe;
    HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    HK(hsa_executable_load_agent_code_object(exe, g_gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(exe, nullptr));
    uint64_t ko_keep = 0, ko_stamp = 0;
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, "keeper.kd", &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko_keep));
    HK(hsa_executable_get_symbol_by_name(exe, "stamp.kd", &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko_stamp));

    // host words the kernels write / read (fine-grained, GPU-accessible)
    char *host = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_fine, 4096, 0, (void **)&host));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, host));
    memset(host, 0, 4096);
    volatile uint32_t *stop = (volatile uint32_t *)host;
    volatile uint32_t *flag = (volatile uint32_t *)(host + 64);
    volatile uint64_t *tk = (volatile uint64_t *)(host + 128);   // keeper start, end
    volatile uint64_t *tst = (volatile uint64_t *)(host + 192);  // stamp start
    const uint64_t max_ticks = 20000;                             // 200 us at 100 MHz
    struct KA { const void *stop; void *t; uint64_t max_ticks; };
    struct SA { void *flag; void *t; uint32_t seq; uint32_t pad; };
    KA *ka = nullptr;
    SA *sa = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_kern, 64, 0, (void **)&ka));
    HK(hsa_amd_memory_pool_allocate(g_kern, 64, 0, (void **)&sa));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, ka));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, sa));
    *ka = KA{(const void *)stop, (void *)tk, max_ticks};

    hsa_queue_t *q = nullptr, *q2 = nullptr;
    HK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    HK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q2));
    HK(hsa_amd_profiling_set_profiler_enabled(q, 1));
    hsa_signal_t sk, ss;
    HK(hsa_signal_create(0, 1, &g_gpu, &sk));
    HK(hsa_signal_create(0, 1, &g_gpu, &ss));
    printf("HSA_ALLOCATE_QUEUE_DEV_MEM=%s\n", getenv("HSA_ALLOCATE_QUEUE_DEV_MEM") ? getenv("HSA_ALLOCATE_QUEUE_DEV_MEM") : "(unset)");

    const int K = getenv("K") ? atoi(getenv("K")) : 300;
    struct Case { const char *name; int keeper; bool barrier; };   // keeper: 0 none, 1 same queue, 2 other queue
    const Case cases[] = {{"idle b0", 0, false}, {"idle b1", 0, true}, {"keeper b0", 1, false},
                          {"keeper b1", 1, true}, {"other-queue b0", 2, false}};
    uint32_t seq = 0;
    for (int round = 0; round < 2; ++round) {
        for (const Case &c : cases) {
            std::vector<double> d2w, d2cp, conc;
            int concurrent = 0;
            for (int k = 0; k < K + 10; ++k) {
                ++seq;
                *stop = 0;
                tk[0] = 0;
                tk[1] = 0;
                if (c.keeper) {
                    hsa_signal_store_relaxed(sk, 1);
                    post(c.keeper == 1 ? q : q2, ko_keep, ka, sk, true);
                    const uint64_t tw = ts();
                    while (__atomic_load_n(&tk[0], __ATOMIC_ACQUIRE) == 0) {
                        _mm_pause();
                        if (us(ts() - tw) > 2e6) { printf("keeper never started\n"); _exit(4); }
                    }
                    // 2 us more: the CP has long finished launching it
                    const uint64_t t2 = ts();
                    while (us(ts() - t2) < 2.0) _mm_pause();
                } else {
                    const uint64_t t2 = ts();
                    while (us(ts() - t2) < 8.0) _mm_pause();
                }
                *sa = SA{(void *)flag, (void *)tst, seq, 0};
                _mm_sfence();
                hsa_signal_store_relaxed(ss, 1);
                const uint64_t t0 = ts();
                post(q, ko_stamp, sa, ss, c.barrier);
                if (c.keeper == 1 && c.barrier) {
                    // the stamp waits for the keeper: stop it after 3 us so the
                    // case measures the serialised path, not the time limit
                    while (us(ts() - t0) < 3.0) _mm_pause();
                    *stop = 1;
                }
                wait_word<uint32_t>(flag, seq);
                const uint64_t t1 = ts();
                *stop = 1;
                wait_sig(ss);
                if (c.keeper) wait_sig(sk);
                hsa_amd_profiling_dispatch_time_t pt{};
                const bool okt = hsa_amd_profiling_get_dispatch_time(g_gpu, ss, &pt) == HSA_STATUS_SUCCESS;
                if (k < 10) continue;
                d2w.push_back(us(t1 - t0));
                if (okt) d2cp.push_back(us(pt.start - t0));
                if (c.keeper == 1) {
                    const double dt = ((double)(int64_t)(tst[0] - tk[1])) * 0.01;   // 100 MHz ticks -> us
                    conc.push_back(dt);
                    if (dt < 0) ++concurrent;
                }
            }
            printf("round %d %-15s doorbell->stamp seen %6.2f us  doorbell->CP start %6.2f us", round, c.name, med(d2w),
                   med(d2cp));
            if (c.keeper == 1) printf("  stamp start - keeper end %6.2f us (concurrent %d of %d)", med(conc), concurrent, K);
            printf("\n");
        }
    }
    return 0;
}
