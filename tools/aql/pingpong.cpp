// pingpong.cpp -- host side of tools/aql/pingpong_kernel.hip: the round trip
// host -> resident waves -> host, against the command processor's doorbell
// path (tools/aql/cp_latency.cpp).  One dispatch of G workgroups stays resident
// for K commands; per command the host bumps the command word (host
// fine-grained memory, or VRAM through the BAR + HDP flush) and spins on the
// response word the last workgroup writes.
//   tools/aql/build_pingpong.sh && tools/aql/pingpong tools/aql/pingpong_kernel.co
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
static hsa_amd_memory_pool_t g_vram, g_kern, g_fine;
static bool g_have_vram = false, g_have_kern = false, g_have_fine = false;
static uint64_t g_freq = 0;

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) { g_cpu = a; g_have_cpu = true; }
    if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) { g_gpu = a; g_have_gpu = true; }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_pool(hsa_amd_memory_pool_t p, void *which) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t f = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &f);
    const long w = (long)which;
    if (w == 0 && (f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !g_have_vram) { g_vram = p; g_have_vram = true; }
    if (w == 1 && (f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_kern) { g_kern = p; g_have_kern = true; }
    if (w == 2 && (f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !g_have_fine) { g_fine = p; g_have_fine = true; }
    return HSA_STATUS_SUCCESS;
}
static uint64_t ts() {
    uint64_t t = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    return t;
}
static double us(uint64_t dt) { return (double)(int64_t)dt * 1e6 / (double)g_freq; }
static double pct(std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
}

struct Args { const uint32_t *cmd; uint32_t *ctr; uint32_t *resp; uint32_t iters; uint32_t fence; uint64_t max_ticks; uint32_t nwg; };

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: %s pingpong_kernel.co\n", argv[0]); return 1; }
    setvbuf(stdout, nullptr, _IOLBF, 0);
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    hsa_amd_agent_iterate_memory_pools(g_gpu, find_pool, (void *)0);
    hsa_amd_agent_iterate_memory_pools(g_cpu, find_pool, (void *)1);
    hsa_amd_agent_iterate_memory_pools(g_cpu, find_pool, (void *)2);
    if (!g_have_gpu || !g_have_vram || !g_have_kern || !g_have_fine) { printf("agents / pools not found\n"); return 1; }
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
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, "pingpong.kd", &g_gpu, &sym));
    uint64_t ko = 0;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko));
    uint32_t lds = 0;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &lds));

    hsa_queue_t *q = nullptr;
    HK(hsa_queue_create(g_gpu, 1024, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    hsa_amd_hdp_flush_t h{};
    HK(hsa_agent_get_info(g_gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &h));
    volatile uint32_t *hdp = h.HDP_MEM_FLUSH_CNTL;

    // command word: host fine-grained, or VRAM written through the BAR
    uint32_t *cmd_host = nullptr, *cmd_vram = nullptr, *resp = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_fine, 4096, 0, (void **)&cmd_host));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, cmd_host));
    HK(hsa_amd_memory_pool_allocate(g_vram, 4096, 0, (void **)&cmd_vram));
    HK(hsa_amd_agents_allow_access(1, &g_cpu, nullptr, cmd_vram));
    HK(hsa_amd_memory_pool_allocate(g_fine, 4096, 0, (void **)&resp));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, resp));
    uint32_t *ctr = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_vram, 4096, 0, (void **)&ctr));
    HK(hsa_amd_agents_allow_access(1, &g_cpu, nullptr, ctr));
    void *karg = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_kern, 64, 0, &karg));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, karg));
    hsa_signal_t done;
    HK(hsa_signal_create(1, 0, nullptr, &done));

    const uint32_t K = 400;
    for (int vram = 0; vram < 2; ++vram) {
        for (uint32_t G : {1u, 256u, 2048u}) {
            for (uint32_t fence : {0u, 1u, 2u}) {
                uint32_t *cmd = vram ? cmd_vram : cmd_host;
                __atomic_store_n(cmd, 0u, __ATOMIC_RELEASE);
                __atomic_store_n(ctr, 0u, __ATOMIC_RELEASE);
                __atomic_store_n(resp, 0u, __ATOMIC_RELEASE);
                _mm_sfence();
                *hdp = 1u;
                (void)*hdp;
                Args a{cmd, ctr, resp, K, fence, 20000000ull, G};   // 200 ms per wait at 100 MHz
                memcpy(karg, &a, sizeof a);
                hsa_signal_store_relaxed(done, 1);
                const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
                hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
                memset((char *)p + 4, 0, sizeof(*p) - 4);
                p->workgroup_size_x = 256;
                p->workgroup_size_y = 1;
                p->workgroup_size_z = 1;
                p->grid_size_x = 256 * G;
                p->grid_size_y = 1;
                p->grid_size_z = 1;
                p->group_segment_size = lds;
                p->kernel_object = ko;
                p->kernarg_address = karg;
                p->completion_signal = done;
                const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                        (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                        (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
                const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
                hsa_queue_store_write_index_relaxed(q, idx + 1);
                __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
                hsa_signal_store_screlease(q->doorbell_signal, idx);
                // let every workgroup become resident before the first command
                const uint64_t w0 = ts();
                while (us(ts() - w0) < 200.0) _mm_pause();
                std::vector<double> rt;
                bool lost = false;
                for (uint32_t k = 1; k <= K; ++k) {
                    const uint64_t t0 = ts();
                    __atomic_store_n(cmd, k, __ATOMIC_RELEASE);
                    if (vram) { _mm_sfence(); *hdp = 1u; }
                    while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != k) {
                        _mm_pause();
                        if (us(ts() - t0) > 100000.0) { lost = true; break; }
                    }
                    if (lost) break;
                    const uint64_t t1 = ts();
                    if (k > 20) rt.push_back(us(t1 - t0));
                    const uint64_t g0 = ts();                  // 5 us between commands
                    while (us(ts() - g0) < 5.0) _mm_pause();
                }
                if (lost) {
                    // end the kernel: a command beyond every wait
                    __atomic_store_n(cmd, 0xffffffffu, __ATOMIC_RELEASE);
                    _mm_sfence();
                    *hdp = 1u;
                }
                if (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, 3000000000ull, HSA_WAIT_STATE_BLOCKED) != 0) {
                    printf("resident kernel did not end\n");
                    _exit(4);
                }
                if (lost) { printf("cmd %s G %4u fence %u: response lost\n", vram ? "vram" : "host", G, fence); continue; }
                printf("cmd %s G %4u fence %u: round trip p10 %5.2f  p50 %5.2f  p90 %5.2f us\n", vram ? "vram" : "host",
                       G, fence, pct(rt, 0.1), pct(rt, 0.5), pct(rt, 0.9));
            }
        }
    }
    return 0;
}
