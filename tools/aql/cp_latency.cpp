// cp_latency.cpp -- where the ~4 us between ringing the doorbell and the CP's
// dispatch start timestamp goes, for a one-workgroup dispatch of the product's
// own tile kernel (mpir_tile_SUM_MPIR_HIP_F32 from lib/libmpir_hip_tiles.hsaco).
//
//   g++ -O2 -std=c++17 -I/opt/rocm/include tools/aql/cp_latency.cpp -o tools/aql/cp_latency \
//       -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
//   [HSA_ALLOCATE_QUEUE_DEV_MEM=1] [KARG_VRAM=1] [IDLE_ONLY=1] [EXTRA_QUEUES=n] [HIP_INIT=1] [NO_PROFILE=1] tools/aql/cp_latency mpich-pip_amd/lib/libmpir_hip_tiles.hsaco
//
// Cases (medians over 300 calls, us; all on the system timestamp clock):
//   idle G      one dispatch, the host idles G us after the previous completion
//   pair        two dispatch packets published together, one doorbell: the
//               second's CP start minus the first's CP end
//   barrier+d   an empty barrier-AND packet rung first, the dispatch rung d us
//               later: its doorbell -> CP start
//   spinner     a one-wave kernel (tools/aql/spin_kernel.hip, argv[2]) already
//               running and polling a flag word; the call publishes its
//               dispatch behind it, rings, then sets the flag: flag -> CP start
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <dlfcn.h>
#include <immintrin.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unistd.h>
#include <vector>

#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_; hsa_status_string(s_, &m_); \
    printf("HSA %s line %d: %s\n", #x, __LINE__, m_); exit(3);} } while (0)

static hsa_agent_t g_gpu, g_cpu;
static bool g_have_gpu = false, g_have_cpu = false;
static hsa_amd_memory_pool_t g_vram, g_kern;
static bool g_have_vram = false, g_have_kern = false;
static uint64_t g_freq = 0;

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) { g_cpu = a; g_have_cpu = true; }
    if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) { g_gpu = a; g_have_gpu = true; }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_vram(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t f = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &f);
    if ((f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !g_have_vram) { g_vram = p; g_have_vram = true; }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kern(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t f = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &f);
    if ((f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_kern) { g_kern = p; g_have_kern = true; }
    return HSA_STATUS_SUCCESS;
}

static hsa_amd_memory_pool_t g_fine;
static bool g_have_fine = false;
static hsa_status_t find_fine(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t f = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &f);
    if ((f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !g_have_fine) { g_fine = p; g_have_fine = true; }
    return HSA_STATUS_SUCCESS;
}

static uint64_t ts() {
    uint64_t t = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    return t;
}
static double us(uint64_t dt) { return (double)(int64_t)dt * 1e6 / (double)g_freq; }
static void spin_us(double d) {
    const uint64_t t0 = ts();
    while (us(ts() - t0) < d) _mm_pause();
}

struct KArgs { const char *in; char *io; uint64_t vbytes; uint64_t keep; };

static hsa_queue_t *g_q;
static uint64_t g_ko;
static void *g_karg;

static void write_dispatch(uint64_t idx, hsa_signal_t sig, bool publish) {
    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)g_q->base_address + (idx & (g_q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    p->workgroup_size_x = 256;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->grid_size_x = 256;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->kernel_object = g_ko;
    p->kernarg_address = g_karg;
    p->completion_signal = sig;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    if (publish) __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
}
static void write_barrier(uint64_t idx) {
    hsa_barrier_and_packet_t *p = (hsa_barrier_and_packet_t *)g_q->base_address + (idx & (g_q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    const uint16_t header = (HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                            (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    __atomic_store_n((uint32_t *)p, (uint32_t)header, __ATOMIC_RELEASE);
}
static void write_barrier_dep(uint64_t idx, hsa_signal_t dep) {
    hsa_barrier_and_packet_t *p = (hsa_barrier_and_packet_t *)g_q->base_address + (idx & (g_q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    p->dep_signal[0] = dep;
    const uint16_t header = (HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                            (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    __atomic_store_n((uint32_t *)p, (uint32_t)header, __ATOMIC_RELEASE);
}
static void wait(hsa_signal_t s) {
    // bounded: a dispatch that never completes ends the run (2 s)
    const uint64_t t0 = ts();
    while (hsa_signal_load_scacquire(s) != 0) {
        _mm_pause();
        if (us(ts() - t0) > 2e6) {
            printf("timeout waiting for a completion signal\n");
            fflush(stdout);
            _exit(4);
        }
    }
}
static void times(hsa_signal_t s, uint64_t *a, uint64_t *b) {
    hsa_amd_profiling_dispatch_time_t t{};
    HK(hsa_amd_profiling_get_dispatch_time(g_gpu, s, &t));
    *a = t.start;
    *b = t.end;
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// HIP_INIT=1: bring the HIP runtime up in this process first (as the library's
// callers have it): hipInit, a 1 GiB hipMalloc, a hipMemset on the null stream
// and a synchronize, through dlopen so the tool keeps building without HIP.
static void hip_init() {
    void *h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) { printf("dlopen libamdhip64: %s\n", dlerror()); exit(3); }
    auto init = (int (*)(unsigned))dlsym(h, "hipInit");
    auto setdev = (int (*)(int))dlsym(h, "hipSetDevice");
    auto mal = (int (*)(void **, size_t))dlsym(h, "hipMalloc");
    auto mset = (int (*)(void *, int, size_t))dlsym(h, "hipMemset");
    auto sync = (int (*)())dlsym(h, "hipDeviceSynchronize");
    void *p = nullptr;
    if (!init || !setdev || !mal || !mset || !sync || init(0) || setdev(0) || mal(&p, 1ull << 30) ||
        mset(p, 0, 1ull << 30) || sync()) {
        printf("HIP bring-up failed\n");
        exit(3);
    }
    printf("HIP runtime up (1 GiB allocated and set)\n");
}

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: %s tiles.hsaco\n", argv[0]); return 1; }
    setvbuf(stdout, nullptr, _IOLBF, 0);
    if (getenv("HIP_INIT")) hip_init();
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    hsa_amd_agent_iterate_memory_pools(g_gpu, find_vram, nullptr);
    hsa_amd_agent_iterate_memory_pools(g_cpu, find_kern, nullptr);
    if (!g_have_gpu || !g_have_vram || !g_have_kern) { printf("agents / pools not found\n"); return 1; }
    HK(hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &g_freq));
    // code object
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
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, "mpir_tile_SUM_MPIR_HIP_F32.kd", &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &g_ko));
    // operands (16 KiB each, VRAM) and kernargs (kernarg pool, host memory)
    void *dev = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_vram, 1 << 16, 0, &dev));
    KArgs ka{(const char *)dev, (char *)dev + 32768, 16384, 0};
    if (getenv("KARG_VRAM")) {
        // KARG_VRAM=1: the kernargs in VRAM, as the library keeps its slots
        // (written once by a copy, so the first dispatch already sees them)
        HK(hsa_amd_memory_pool_allocate(g_vram, 4096, 0, &g_karg));
        char tmp[128] = {};
        memcpy(tmp, &ka, sizeof ka);
        HK(hsa_memory_copy(g_karg, tmp, sizeof tmp));
    } else {
        HK(hsa_amd_memory_pool_allocate(g_kern, 128, 0, &g_karg));
        HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, g_karg));
        memset(g_karg, 0, 128);
        memcpy(g_karg, &ka, sizeof ka);
    }
    printf("kernargs in %s\n", getenv("KARG_VRAM") ? "VRAM" : "the kernarg pool (host memory)");
    // QUEUE_SINGLE=1: a single-producer queue; QUEUE_SIZE: packets in the ring
    const uint32_t qsize = getenv("QUEUE_SIZE") ? (uint32_t)atoi(getenv("QUEUE_SIZE")) : 1024u;
    const hsa_queue_type32_t qtype = getenv("QUEUE_SINGLE") ? HSA_QUEUE_TYPE_SINGLE : HSA_QUEUE_TYPE_MULTI;
    printf("queue %s, %u packets\n", qtype == HSA_QUEUE_TYPE_SINGLE ? "single" : "multi", qsize);
    HK(hsa_queue_create(g_gpu, qsize, qtype, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &g_q));
    // NO_PROFILE=1: no CP timestamps (as the library's call queue runs); only
    // the host-clock doorbell -> host sees interval is then meaningful
    const bool prof = getenv("NO_PROFILE") == nullptr;
    if (prof) HK(hsa_amd_profiling_set_profiler_enabled(g_q, 1));
    if (const char *pr = getenv("QUEUE_PRIORITY")) {
        const hsa_amd_queue_priority_t qp = !strcmp(pr, "high") ? HSA_AMD_QUEUE_PRIORITY_HIGH
                                           : !strcmp(pr, "low") ? HSA_AMD_QUEUE_PRIORITY_LOW
                                                                : HSA_AMD_QUEUE_PRIORITY_NORMAL;
        HK(hsa_amd_queue_set_priority(g_q, qp));
        printf("queue priority %s\n", pr);
    }
    // EXTRA_QUEUES=n: n more (idle) queues on the GPU, each with one dispatch
    // run through it first, as other streams of the same process would leave them
    const int extra = getenv("EXTRA_QUEUES") ? atoi(getenv("EXTRA_QUEUES")) : 0;
    for (int i = 0; i < extra; ++i) {
        hsa_queue_t *q2;
        HK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q2));
        hsa_signal_t sx;
        HK(hsa_signal_create(1, 0, nullptr, &sx));
        hsa_queue_t *keep = g_q;
        g_q = q2;
        const uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
        write_dispatch(idx, sx, true);
        hsa_queue_store_write_index_relaxed(g_q, idx + 1);
        hsa_signal_store_screlease(g_q->doorbell_signal, idx);
        g_q = keep;
        const uint64_t t0 = ts();
        while (hsa_signal_load_scacquire(sx) != 0) {
            if (us(ts() - t0) > 2e6) { printf("extra queue dispatch timed out\n"); return 4; }
        }
        hsa_signal_destroy(sx);
    }
    if (extra) printf("%d extra queues\n", extra);
    hsa_signal_t s1, s2;
    HK(hsa_signal_create(0, 1, &g_gpu, &s1));
    HK(hsa_signal_create(0, 1, &g_gpu, &s2));
    printf("HSA_ALLOCATE_QUEUE_DEV_MEM=%s\n", getenv("HSA_ALLOCATE_QUEUE_DEV_MEM") ? getenv("HSA_ALLOCATE_QUEUE_DEV_MEM") : "(unset)");

    const int K = 300;
    // PRE_RING=1: only the "ring first, publish later" cases.  The slot's
    // header is INVALID when the doorbell rings; the host publishes the packet
    // d us later (the time the call's own validation would take), with or
    // without ringing again.  A CP that does not wait on an INVALID header
    // shows up as a timeout (wait() ends the run).
    if (getenv("PRE_RING")) {
        for (int again = 0; again < 2; ++again) {
            for (double d : {0.5, 1.0, 2.0, 3.0, 4.0, 6.0}) {
                std::vector<double> p2s, tot;
                for (int k = 0; k < K + 10; ++k) {
                    hsa_signal_store_relaxed(s1, 1);
                    const uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
                    hsa_kernel_dispatch_packet_t *p =
                        (hsa_kernel_dispatch_packet_t *)g_q->base_address + (idx & (g_q->size - 1));
                    __atomic_store_n((uint16_t *)p, (uint16_t)(HSA_PACKET_TYPE_INVALID << HSA_PACKET_HEADER_TYPE),
                                     __ATOMIC_RELEASE);
                    hsa_queue_store_write_index_relaxed(g_q, idx + 1);
                    const uint64_t tr = ts();
                    hsa_signal_store_screlease(g_q->doorbell_signal, idx);
                    spin_us(d);
                    write_dispatch(idx, s1, false);
                    const uint64_t tp = ts();
                    write_dispatch(idx, s1, true);
                    if (again) hsa_signal_store_screlease(g_q->doorbell_signal, idx);
                    wait(s1);
                    const uint64_t t1 = ts();
                    uint64_t a, b;
                    times(s1, &a, &b);
                    if (k < 10) continue;
                    p2s.push_back(us(a - tp));
                    tot.push_back(us(t1 - tr));
                }
                printf("pre-ring%s, publish %.1f us later: publish->CP start %5.2f; first ring->host sees %5.2f\n",
                       again ? " + ring again" : "", d, med(p2s), med(tot));
            }
        }
        return 0;
    }
    const bool spin_only = getenv("SPIN_ONLY") != nullptr;
    // idle G
    for (double G : {0.0, 5.0, 20.0, 100.0, 1000.0}) {
        if (spin_only) break;
        std::vector<double> d2s, s2e, e2h, tot;
        for (int k = 0; k < K + 10; ++k) {
            spin_us(G);
            hsa_signal_store_relaxed(s1, 1);
            const uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
            write_dispatch(idx, s1, true);
            hsa_queue_store_write_index_relaxed(g_q, idx + 1);
            const uint64_t t0 = ts();
            hsa_signal_store_screlease(g_q->doorbell_signal, idx);
            wait(s1);
            const uint64_t t1 = ts();
            uint64_t a = t0, b = t0;
            if (prof) times(s1, &a, &b);
            if (k < 10) continue;
            d2s.push_back(us(a - t0));
            s2e.push_back(us(b - a));
            e2h.push_back(us(t1 - b));
            tot.push_back(us(t1 - t0));
        }
        printf("idle %7.1f us: doorbell->CP start %5.2f  CP start->end %5.2f  CP end->host sees %5.2f  doorbell->host sees %5.2f\n",
               G, med(d2s), med(s2e), med(e2h), med(tot));
    }
    if (getenv("IDLE_ONLY")) return 0;
    // pair
    {
        std::vector<double> gap, d2s;
        for (int k = 0; k < K + 10; ++k) {
            hsa_signal_store_relaxed(s1, 1);
            hsa_signal_store_relaxed(s2, 1);
            const uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
            write_dispatch(idx, s1, true);
            write_dispatch(idx + 1, s2, true);
            hsa_queue_store_write_index_relaxed(g_q, idx + 2);
            const uint64_t t0 = ts();
            hsa_signal_store_screlease(g_q->doorbell_signal, idx + 1);
            wait(s2);
            uint64_t a1, b1, a2, b2;
            times(s1, &a1, &b1);
            times(s2, &a2, &b2);
            if (k < 10) continue;
            d2s.push_back(us(a1 - t0));
            gap.push_back(us(a2 - b1));
        }
        printf("pair: doorbell->first start %5.2f; second start - first end %5.2f\n", med(d2s), med(gap));
    }
    // barrier rung first, the dispatch d us later
    for (double d : {0.5, 1.0, 2.0, 4.0}) {
        std::vector<double> d2s, tot;
        for (int k = 0; k < K + 10; ++k) {
            hsa_signal_store_relaxed(s1, 1);
            uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
            const uint64_t tb = ts();
            write_barrier(idx);
            hsa_queue_store_write_index_relaxed(g_q, idx + 1);
            hsa_signal_store_screlease(g_q->doorbell_signal, idx);
            spin_us(d);
            idx = idx + 1;
            write_dispatch(idx, s1, true);
            hsa_queue_store_write_index_relaxed(g_q, idx + 1);
            const uint64_t t0 = ts();
            hsa_signal_store_screlease(g_q->doorbell_signal, idx);
            wait(s1);
            const uint64_t t1 = ts();
            uint64_t a, b;
            times(s1, &a, &b);
            if (k < 10) continue;
            d2s.push_back(us(a - t0));
            tot.push_back(us(t1 - tb));
        }
        printf("barrier then dispatch %.1f us later: doorbell->CP start %5.2f; barrier ring -> host sees %5.2f\n", d,
               med(d2s), med(tot));
    }
    // a barrier-AND waiting on a signal is posted (and rung) ahead of time; the
    // call publishes its dispatch behind it, then releases the signal
    {
        hsa_signal_t go;
        HK(hsa_signal_create(1, 1, &g_gpu, &go));
        for (double pre : {10.0, 50.0}) {
            std::vector<double> r2s, tot;
            for (int k = 0; k < K + 10; ++k) {
                hsa_signal_store_relaxed(go, 1);
                hsa_signal_store_relaxed(s1, 1);
                uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
                write_barrier_dep(idx, go);
                hsa_queue_store_write_index_relaxed(g_q, idx + 1);
                hsa_signal_store_screlease(g_q->doorbell_signal, idx);
                spin_us(pre);                           // the CP is now parked on the barrier
                const uint64_t t0 = ts();
                write_dispatch(idx + 1, s1, true);
                hsa_queue_store_write_index_relaxed(g_q, idx + 2);
                hsa_signal_store_screlease(g_q->doorbell_signal, idx + 1);
                const uint64_t tr = ts();
                hsa_signal_store_screlease(go, 0);
                wait(s1);
                const uint64_t t1 = ts();
                uint64_t a, b;
                times(s1, &a, &b);
                if (k < 10) continue;
                r2s.push_back(us(a - tr));
                tot.push_back(us(t1 - t0));
            }
            printf("parked barrier (%.0f us): release->CP start %5.2f; publish -> host sees %5.2f\n", pre, med(r2s),
                   med(tot));
        }
    }
    // spinner: needs the spin kernel's code object
    if (argc > 2) {
        hsa_amd_agent_iterate_memory_pools(g_cpu, find_fine, nullptr);
        FILE *f2 = fopen(argv[2], "rb");
        if (!f2 || !g_have_fine) { printf("no spin code object / fine-grained pool\n"); return 0; }
        std::vector<char> co2;
        while ((n = fread(buf, 1, sizeof buf, f2)) > 0) co2.insert(co2.end(), buf, buf + n);
        fclose(f2);
        hsa_code_object_reader_t rd2;
        hsa_executable_t exe2;
        HK(hsa_code_object_reader_create_from_memory(co2.data(), co2.size(), &rd2));
        HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe2));
        HK(hsa_executable_load_agent_code_object(exe2, g_gpu, rd2, nullptr, nullptr));
        HK(hsa_executable_freeze(exe2, nullptr));
        hsa_executable_symbol_t sym2;
        HK(hsa_executable_get_symbol_by_name(exe2, "spin_wait.kd", &g_gpu, &sym2));
        uint64_t ko_spin = 0;
        HK(hsa_executable_symbol_get_info(sym2, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko_spin));
        // flag in host fine-grained memory, or (SPIN_FLAG_VRAM=1) in VRAM written
        // through the BAR and pushed by an HDP flush; spinner kernargs in the kernarg pool
        const bool vram_flag = getenv("SPIN_FLAG_VRAM") != nullptr;
        uint32_t *flag = nullptr;
        volatile uint32_t *hdp = nullptr;
        if (vram_flag) {
            HK(hsa_amd_memory_pool_allocate(g_vram, 4096, 0, (void **)&flag));
            HK(hsa_amd_agents_allow_access(1, &g_cpu, nullptr, flag));
            hsa_amd_hdp_flush_t h{};
            HK(hsa_agent_get_info(g_gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &h));
            hdp = h.HDP_MEM_FLUSH_CNTL;
        } else {
            HK(hsa_amd_memory_pool_allocate(g_fine, 4096, 0, (void **)&flag));
            HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, flag));
        }
        printf("spinner flag in %s\n", vram_flag ? "VRAM (BAR write + HDP flush)" : "host fine-grained memory");
        void *karg2 = nullptr;
        HK(hsa_amd_memory_pool_allocate(g_kern, 64, 0, &karg2));
        HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, karg2));
        struct { const uint32_t *f; uint64_t max_ticks; } sa{flag, 100000ull};   // 1 ms at 100 MHz
        memcpy(karg2, &sa, sizeof sa);
        hsa_signal_t ss;
        HK(hsa_signal_create(0, 1, &g_gpu, &ss));
        for (double pre : {5.0, 20.0}) {
            std::vector<double> f2s, gap, tot;
            int timeouts = 0;
            for (int k = 0; k < K + 10; ++k) {
                __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
                if (hdp) { _mm_sfence(); *hdp = 1u; (void)*hdp; }
                hsa_signal_store_relaxed(ss, 1);
                hsa_signal_store_relaxed(s1, 1);
                uint64_t idx = hsa_queue_load_write_index_relaxed(g_q);
                {   // the spinner
                    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)g_q->base_address + (idx & (g_q->size - 1));
                    memset((char *)p + 4, 0, sizeof(*p) - 4);
                    p->workgroup_size_x = 64;
                    p->workgroup_size_y = 1;
                    p->workgroup_size_z = 1;
                    p->grid_size_x = 64;
                    p->grid_size_y = 1;
                    p->grid_size_z = 1;
                    p->kernel_object = ko_spin;
                    p->kernarg_address = karg2;
                    p->completion_signal = ss;
                    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
                    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
                    hsa_queue_store_write_index_relaxed(g_q, idx + 1);
                    __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
                    hsa_signal_store_screlease(g_q->doorbell_signal, idx);
                }
                spin_us(pre);                       // the spinner is running now
                const uint64_t t0 = ts();
                write_dispatch(idx + 1, s1, true);
                hsa_queue_store_write_index_relaxed(g_q, idx + 2);
                hsa_signal_store_screlease(g_q->doorbell_signal, idx + 1);
                const uint64_t tf = ts();
                __atomic_store_n(flag, 1u, __ATOMIC_RELEASE);
                if (hdp) { _mm_sfence(); *hdp = 1u; }
                wait(s1);
                const uint64_t t1 = ts();
                wait(ss);
                uint64_t a, b, sa0, sb0;
                times(s1, &a, &b);
                times(ss, &sa0, &sb0);
                if (k < 10) continue;
                if (us(sb0 - sa0) > 900.0) ++timeouts;
                f2s.push_back(us(a - tf));
                gap.push_back(us(a - sb0));
                tot.push_back(us(t1 - t0));
            }
            printf("spinner (%.0f us ahead): flag -> CP start %5.2f; spinner end -> CP start %5.2f; publish -> host sees %5.2f"
                   " (timeouts %d)\n", pre, med(f2s), med(gap), med(tot), timeouts);
        }
    }
    return 0;
}
