// aql2.cpp -- what a synchronous 256 MiB fp32 SUM call costs beyond its kernel
// body, and which dispatch / completion form removes it.
//
// Every variant runs K synchronous calls over 4 rotating 256 MiB pairs.  Per
// variant: the host wall time per call (mean), and from wall_clock64() stamps
// of every workgroup (a second pass) the GPU body (first start -> last end)
// and the GPU idle gap between one call's last workgroup and the next call's
// first one.
//   hip_flag_nt    hipLaunchKernel, hipStreamWriteValue32, spin   (the product)
//   hip_flag_hybF  the same, stores sc1 (write-through) in the last F of workgroups
//   hip_self       hipLaunchKernel of the self-completing kernel, spin on its word
//   aql_*          our own AQL queue: kernargs in VRAM written by the host (HDP
//                  flush before the doorbell), packet completion signal polled
//                  (sig_*) or the kernel's own word (self)
//   bash tools/aql/build2.sh; tools/aql/aql2 tools/aql/aql2_kernels.co [K]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "aql2_kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_; hsa_status_string(s_, &m_); printf("HSA %s line %d: %s\n", #x, __LINE__, m_); exit(3);} } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static hsa_agent_t g_gpu, g_cpu;
static uint32_t g_bdf;
static hsa_amd_memory_pool_t g_vram;
static bool g_have_cpu = false, g_have_vram = false;

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) { g_cpu = a; g_have_cpu = true; }
    if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t bdf = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        if (bdf == g_bdf) g_gpu = a;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_vram(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t f = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &f);
    if (f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) { g_vram = p; g_have_vram = true; return HSA_STATUS_INFO_BREAK; }
    return HSA_STATUS_SUCCESS;
}

struct Aql {
    hsa_queue_t *q = nullptr;
    hsa_signal_t sig{};
    char *karg = nullptr;          // VRAM ring, host-written
    int kslot = 0;
    volatile uint32_t *hdp = nullptr;
    uint16_t acq = HSA_FENCE_SCOPE_SYSTEM, rel = HSA_FENCE_SCOPE_SYSTEM;
    int barrier = 1;
    void dispatch(uint64_t ko, uint32_t groups, const void *args, size_t nargs, bool with_signal) {
        char *ka = karg + (size_t)(kslot++ & 63) * 256;
        memcpy(ka, args, nargs);
        _mm_sfence();
        if (hdp) { *hdp = 1u; (void)*hdp; }     // HDP flush: host writes to VRAM visible to the GPU
        if (with_signal) hsa_signal_store_relaxed(sig, 1);
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
        hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
        memset((char *)p + 4, 0, sizeof(*p) - 4);
        p->workgroup_size_x = 256; p->workgroup_size_y = 1; p->workgroup_size_z = 1;
        p->grid_size_x = groups * 256; p->grid_size_y = 1; p->grid_size_z = 1;
        p->kernel_object = ko;
        p->kernarg_address = ka;
        p->completion_signal = with_signal ? sig : hsa_signal_t{0};
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (barrier << HSA_PACKET_HEADER_BARRIER) |
                                (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, idx);
    }
    void wait() { while (hsa_signal_load_scacquire(sig) != 0) __builtin_ia32_pause(); }
};

struct KaNt { const char *in; char *io; uint64_t vbytes; uint64_t *ts; };
struct KaHyb { const char *in; char *io; uint64_t vbytes; uint64_t *ts; uint32_t sc1_from; };
struct KaSelfh { const char *in; char *io; uint64_t vbytes; uint64_t *ts; uint32_t *ctl; uint32_t *hflag; uint32_t seq;
                 uint32_t ngroups; uint32_t from; };
struct KaSelf { const char *in; char *io; uint64_t vbytes; uint64_t *ts; uint32_t *cnt; uint32_t nsh; uint32_t *hflag;
                uint32_t seq; uint32_t ngroups; };

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: aql2 code_object [K]\n"); return 1; }
    const int K = argc > 2 ? atoi(argv[2]) : 60;
    CK(hipSetDevice(0));
    int bus = 0, devn = 0, wclk = 0;
    CK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
    CK(hipDeviceGetAttribute(&devn, hipDeviceAttributePciDeviceId, 0));
    CK(hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0));   // kHz
    g_bdf = ((uint32_t)bus << 8) | ((uint32_t)devn << 3);
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    hsa_amd_agent_iterate_memory_pools(g_gpu, find_vram, nullptr);
    if (!g_have_vram || !g_have_cpu) { printf("no VRAM pool / CPU agent\n"); return 4; }
    hsa_amd_hdp_flush_t hdpf{};
    HK(hsa_agent_get_info(g_gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdpf));
    printf("wall clock %d kHz; HDP flush register %p\n", wclk, (void *)hdpf.HDP_MEM_FLUSH_CNTL);

    FILE *f = fopen(argv[1], "rb");
    if (!f) { printf("cannot open %s\n", argv[1]); return 1; }
    std::vector<char> co;
    { char buf[65536]; size_t n; while ((n = fread(buf, 1, sizeof buf, f)) > 0) co.insert(co.end(), buf, buf + n); }
    fclose(f);
    hsa_code_object_reader_t rd;
    HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    hsa_executable_t exe;
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    HK(hsa_executable_load_agent_code_object(exe, g_gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(exe, nullptr));
    auto kobj = [&](const char *name, size_t want) {
        hsa_executable_symbol_t sym;
        uint64_t ko = 0;
        uint32_t kas = 0;
        HK(hsa_executable_get_symbol_by_name(exe, name, &g_gpu, &sym));
        HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko));
        HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kas));
        printf("%s kernarg %u (host struct %zu)\n", name, kas, want);
        if (kas > want || kas + 8 < want) { printf("kernarg size mismatch\n"); exit(5); }
        return ko;
    };
    const uint64_t ko_probe = kobj("a2_probe.kd", 16);
    const uint64_t ko_nt = kobj("a2_nt.kd", sizeof(KaNt));
    const uint64_t ko_hyb = kobj("a2_hyb.kd", sizeof(KaHyb));
    const uint64_t ko_self = kobj("a2_self.kd", sizeof(KaSelf));
    const uint64_t ko_selfh = kobj("a2_selfh.kd", sizeof(KaSelfh));

    Aql aq;
    void *kp = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_vram, 64 * 256, 0, &kp));
    HK(hsa_amd_agents_allow_access(1, &g_cpu, nullptr, kp));
    aq.karg = (char *)kp;
    aq.hdp = hdpf.HDP_MEM_FLUSH_CNTL;
    HK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &aq.q));
    HK(hsa_signal_create(0, 0, nullptr, &aq.sig));

    // ---- kernarg visibility: values written through the BAR + HDP flush must
    // reach the kernel before any kernarg carries a pointer
    {
        hsa_executable_symbol_t sym;
        uint64_t paddr = 0;
        HK(hsa_executable_get_symbol_by_name(exe, "a2_probe_out", &g_gpu, &sym));
        HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_VARIABLE_ADDRESS, &paddr));
        for (int k = 0; k < 200; ++k) {
            uint64_t a[2] = {0x1234567800000000ull + k, ~(uint64_t)k};
            aq.dispatch(ko_probe, 1, a, sizeof a, true);
            aq.wait();
            uint64_t got[2] = {0, 0};
            HK(hsa_memory_copy(got, (void *)paddr, sizeof got));
            if (got[0] != a[0] || got[1] != a[1]) {
                printf("kernarg probe %d: got %llx %llx want %llx %llx -- stopping\n", k, (unsigned long long)got[0],
                       (unsigned long long)got[1], (unsigned long long)a[0], (unsigned long long)a[1]);
                return 7;
            }
        }
        printf("kernarg probe: 200 dispatches saw their VRAM kernargs\n");
        // host cost of the pieces of a dispatch
        const int N = 20000;
        double t0 = now();
        for (int k = 0; k < N; ++k) { *aq.hdp = 1u; (void)*aq.hdp; }
        double t1 = now();
        for (int k = 0; k < N; ++k) { *aq.hdp = 1u; }
        double t2 = now();
        uint64_t vals[4] = {1, 2, 3, 4};
        for (int k = 0; k < N; ++k) { memcpy(aq.karg + (k & 63) * 256, vals, 32); _mm_sfence(); }
        double t3 = now();
        printf("host: HDP flush + readback %.3f us, HDP flush write only %.3f us, 32 B kernarg BAR write + sfence %.3f us\n",
               (t1 - t0) / N * 1e6, (t2 - t1) / N * 1e6, (t3 - t2) / N * 1e6);
    }

    hipStream_t s;
    CK(hipStreamCreate(&s));
    volatile uint32_t *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    uint32_t seq = 0;
    uint32_t *cnt;
    CK(hipMalloc(&cnt, 64 * 1024));
    CK(hipMemset(cnt, 0, 64 * 1024));

    const uint64_t bytes = 256ull << 20;
    const uint64_t n = bytes / 4;
    const uint32_t grid = (uint32_t)(bytes / 16384);
    std::vector<char *> bufs(8);
    {
        std::vector<float> h(n);
        uint32_t x = 1;
        for (auto &v : h) { x = x * 1664525u + 1013904223u; v = (float)(x >> 8) / 16777216.0f * 2 - 1; }
        for (auto &b : bufs) { CK(hipMalloc(&b, bytes)); CK(hipMemcpy(b, h.data(), bytes, hipMemcpyHostToDevice)); }
    }
    uint64_t *ts;
    CK(hipMalloc(&ts, (size_t)K * grid * 16));
    CK(hipDeviceSynchronize());
    auto in = [&](int i) { return (const char *)bufs[2 * (i & 3)]; };
    auto io = [&](int i) { return bufs[2 * (i & 3) + 1]; };

    // ---- correctness: each AQL form == HIP a2_nt on the same operands
    {
        std::vector<char> want(bytes), got(bytes);
        char *o1, *o2;
        CK(hipMalloc(&o1, bytes));
        CK(hipMalloc(&o2, bytes));
        CK(hipMemcpy(o1, io(0), bytes, hipMemcpyDeviceToDevice));
        hipLaunchKernelGGL(a2_nt, dim3(grid), dim3(256), 0, s, in(0), o1, bytes, (uint64_t *)nullptr);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(want.data(), o1, bytes, hipMemcpyDeviceToHost));
        for (int v = 0; v < 3; ++v) {
            CK(hipMemcpy(o2, io(0), bytes, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
            if (v == 0) { KaNt a{in(0), o2, bytes, nullptr}; aq.dispatch(ko_nt, grid, &a, sizeof a, true); aq.wait(); }
            if (v == 1) { KaHyb a{in(0), o2, bytes, nullptr, grid - grid / 8}; aq.dispatch(ko_hyb, grid, &a, sizeof a, true); aq.wait(); }
            if (v == 2) {
                const uint32_t q = ++seq;
                KaSelf a{in(0), o2, bytes, nullptr, cnt, 64, (uint32_t *)flag, q, grid};
                aq.dispatch(ko_self, grid, &a, sizeof a, false);
                while (*flag != q) __builtin_ia32_pause();
            }
            CK(hipMemcpy(got.data(), o2, bytes, hipMemcpyDeviceToHost));
            printf("correctness aql variant %d: %s\n", v, memcmp(want.data(), got.data(), bytes) ? "MISMATCH" : "bit-identical");
        }
        CK(hipFree(o1));
        CK(hipFree(o2));
    }

    struct Var { std::string name; std::function<void(int, uint64_t *)> call; };
    std::vector<Var> vars;
    const char *only = getenv("AQL2_SWEEP");
    // (declared here: the sweep's stored lambdas capture it by reference)
    auto flagwait = [&]() {
        CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
        while (*flag != seq) __builtin_ia32_pause();
    };
    if (only) {
        // store-mix sweep, HIP launch + completion word
        for (int mib : {0, 32, 40, 48, 56, 64, 72, 80}) {
            const uint32_t from = grid - (uint32_t)(((uint64_t)mib << 20) / 16384);
            vars.push_back({"tail_sc1_" + std::to_string(mib) + "MiB", [&, from](int i, uint64_t *t) {
                hipLaunchKernelGGL(a2_hyb, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, from);
                flagwait();
            }});
        }
        for (auto mk : std::vector<std::pair<int, int>>{}) {
            vars.push_back({"mod_sc1_" + std::to_string(mk.second) + "of" + std::to_string(mk.first),
                            [&, mk](int i, uint64_t *t) {
                hipLaunchKernelGGL(a2_mod, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, (uint32_t)mk.first,
                                   (uint32_t)mk.second);
                flagwait();
            }});
        }
    }
    uint32_t *ctl;
    CK(hipMalloc(&ctl, A2_CTL_WORDS * 4));
    CK(hipMemset(ctl, 0, A2_CTL_WORDS * 4));
    int fallbacks = 0;
    auto selfwait = [&](uint32_t q, bool hip) {
        for (;;) {
            const uint32_t v = *flag;
            if (v == q) return;
            if (v == (q | 0x80000000u)) {
                ++fallbacks;
                if (hip) { CK(hipStreamSynchronize(s)); CK(hipMemsetAsync(ctl, 0, A2_CTL_WORDS * 4, s)); CK(hipStreamSynchronize(s)); }
                else { CK(hipDeviceSynchronize()); CK(hipMemset(ctl, 0, A2_CTL_WORDS * 4)); CK(hipDeviceSynchronize()); }
                return;
            }
            __builtin_ia32_pause();
        }
    };
    const char *selfh = getenv("AQL2_SELFH");
    {
        const int N = 20000;
        double t0 = now();
        for (int i = 0; i < N; ++i) (void)hipStreamQuery(nullptr);
        double t1 = now();
        for (int i = 0; i < N; ++i) (void)hipStreamQuery(s);
        double t2 = now();
        printf("host hipStreamQuery(null) %.3f us, hipStreamQuery(own idle stream) %.3f us\n", (t1 - t0) / N * 1e6,
               (t2 - t1) / N * 1e6);
    }
    if (selfh) {
        const uint32_t from64 = grid - (uint32_t)((64ull << 20) / 16384);
        vars.push_back({"hip_flag_nt", [&](int i, uint64_t *t) {
            hipLaunchKernelGGL(a2_nt, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t);
            CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
            while (*flag != seq) __builtin_ia32_pause();
        }});
        vars.push_back({"hip_flag_tail64M", [&](int i, uint64_t *t) {
            hipLaunchKernelGGL(a2_hyb, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, from64);
            CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
            while (*flag != seq) __builtin_ia32_pause();
        }});
        for (uint32_t from : std::vector<uint32_t>{}) {
            vars.push_back({"hip_selfh_from" + std::to_string(from), [&, from](int i, uint64_t *t) {
                const uint32_t q = ++seq;
                hipLaunchKernelGGL(a2_selfh, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, ctl, (uint32_t *)flag, q,
                                   grid, from);
                selfwait(q, true);
            }});
        }
        if (0) vars.push_back({"aql_selfh_agentacq_tail64M", [&](int i, uint64_t *t) {
            const uint32_t q = ++seq;
            aq.acq = HSA_FENCE_SCOPE_AGENT;
            KaSelfh a{in(i), io(i), bytes, t, ctl, (uint32_t *)flag, q, grid, from64};
            aq.dispatch(ko_selfh, grid, &a, sizeof a, false);
            aq.acq = HSA_FENCE_SCOPE_SYSTEM;
            selfwait(q, false);
        }});
        vars.push_back({"aql_sig_tail64M_agentacq_nullq", [&](int i, uint64_t *t) {
            // what the product would check first: is the legacy null stream idle?
            if (hipStreamQuery(nullptr) != hipSuccess) { printf("null stream busy\n"); }
            aq.acq = HSA_FENCE_SCOPE_AGENT;
            KaHyb a{in(i), io(i), bytes, t, from64};
            aq.dispatch(ko_hyb, grid, &a, sizeof a, true);
            aq.wait();
            aq.acq = HSA_FENCE_SCOPE_SYSTEM;
        }});
        vars.push_back({"aql_sig_tail64M_agentacq_agentrel", [&](int i, uint64_t *t) {
            aq.acq = HSA_FENCE_SCOPE_AGENT;
            aq.rel = HSA_FENCE_SCOPE_AGENT;
            KaHyb a{in(i), io(i), bytes, t, from64};
            aq.dispatch(ko_hyb, grid, &a, sizeof a, true);
            aq.wait();
            aq.acq = HSA_FENCE_SCOPE_SYSTEM;
            aq.rel = HSA_FENCE_SCOPE_SYSTEM;
        }});
        vars.push_back({"aql_sig_tail64M_agentacq_nobarrier", [&](int i, uint64_t *t) {
            aq.acq = HSA_FENCE_SCOPE_AGENT;
            aq.barrier = 0;
            KaHyb a{in(i), io(i), bytes, t, from64};
            aq.dispatch(ko_hyb, grid, &a, sizeof a, true);
            aq.wait();
            aq.acq = HSA_FENCE_SCOPE_SYSTEM;
            aq.barrier = 1;
        }});
        vars.push_back({"aql_sig_tail64M_agentacq", [&](int i, uint64_t *t) {
            aq.acq = HSA_FENCE_SCOPE_AGENT;
            KaHyb a{in(i), io(i), bytes, t, from64};
            aq.dispatch(ko_hyb, grid, &a, sizeof a, true);
            aq.wait();
            aq.acq = HSA_FENCE_SCOPE_SYSTEM;
        }});
    }
    const char *loopv = getenv("AQL2_LOOP");
    if (loopv) {
        const uint32_t from64 = grid - (uint32_t)((64ull << 20) / 16384);
        vars.push_back({"hip_flag_tile_tail64M", [&](int i, uint64_t *t) {
            hipLaunchKernelGGL(a2_hyb, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, from64);
            CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
            while (*flag != seq) __builtin_ia32_pause();
        }});
        for (uint32_t G : {1024u, 2048u, 4096u, 8192u, 16384u}) {
            for (uint32_t from : {grid, from64}) {
                vars.push_back({"hip_flag_loopG" + std::to_string(G) + (from == grid ? "_nt" : "_tail64M"),
                                [&, G, from](int i, uint64_t *t) {
                    hipLaunchKernelGGL(a2_loop, dim3(G), dim3(256), 0, s, in(i), io(i), bytes, t, G, grid, from);
                    CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
                    while (*flag != seq) __builtin_ia32_pause();
                }});
            }
        }
    }
    if (!only && !selfh && !loopv) {
    vars.push_back({"hip_flag_nt", [&](int i, uint64_t *t) {
        hipLaunchKernelGGL(a2_nt, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t);
        CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
        while (*flag != seq) __builtin_ia32_pause();
    }});
    for (int frac : {16, 8, 4}) {
        vars.push_back({"hip_flag_hyb1/" + std::to_string(frac), [&, frac](int i, uint64_t *t) {
            hipLaunchKernelGGL(a2_hyb, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, grid - grid / frac);
            CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
            while (*flag != seq) __builtin_ia32_pause();
        }});
    }
    vars.push_back({"hip_self", [&](int i, uint64_t *t) {
        const uint32_t q = ++seq;
        hipLaunchKernelGGL(a2_self, dim3(grid), dim3(256), 0, s, in(i), io(i), bytes, t, cnt, 64u, (uint32_t *)flag, q, grid);
        while (*flag != q) __builtin_ia32_pause();
    }});
    vars.push_back({"aql_sig_nt_sys", [&](int i, uint64_t *t) {
        aq.acq = HSA_FENCE_SCOPE_SYSTEM;
        KaNt a{in(i), io(i), bytes, t};
        aq.dispatch(ko_nt, grid, &a, sizeof a, true);
        aq.wait();
    }});
    vars.push_back({"aql_sig_nt_agentacq", [&](int i, uint64_t *t) {
        aq.acq = HSA_FENCE_SCOPE_AGENT;
        KaNt a{in(i), io(i), bytes, t};
        aq.dispatch(ko_nt, grid, &a, sizeof a, true);
        aq.wait();
        aq.acq = HSA_FENCE_SCOPE_SYSTEM;
    }});
    vars.push_back({"aql_sig_hyb1/8", [&](int i, uint64_t *t) {
        KaHyb a{in(i), io(i), bytes, t, grid - grid / 8};
        aq.dispatch(ko_hyb, grid, &a, sizeof a, true);
        aq.wait();
    }});
    vars.push_back({"aql_self", [&](int i, uint64_t *t) {
        const uint32_t q = ++seq;
        KaSelf a{in(i), io(i), bytes, t, cnt, 64, (uint32_t *)flag, q, grid};
        aq.dispatch(ko_self, grid, &a, sizeof a, false);
        while (*flag != q) __builtin_ia32_pause();
    }});

    }
    const double alg = 3.0 * bytes;
    std::vector<uint64_t> hts((size_t)K * grid * 2);
    for (int r = 0; r < 3; ++r) {
        for (auto &v : vars) {
            for (int i = 0; i < 5; ++i) v.call(i, nullptr);
            const double t0 = now();
            for (int i = 0; i < K; ++i) v.call(i, nullptr);
            const double t1 = now();
            CK(hipDeviceSynchronize());
            // second pass with per-workgroup stamps (slots of workgroups a
            // smaller grid does not have: start = max, end = 0)
            CK(hipMemset(ts, 0xff, (size_t)K * grid * 16));
            for (int i = 0; i < K; ++i) {
                hipLaunchKernelGGL(a2_ts_clear_ends, dim3((grid + 255) / 256), dim3(256), 0, s, ts + (size_t)i * grid * 2, grid);
            }
            CK(hipDeviceSynchronize());
            for (int i = 0; i < K; ++i) v.call(i, ts + (size_t)i * grid * 2);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hts.data(), ts, hts.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> body, gap;
            uint64_t prev_end = 0;
            for (int i = 0; i < K; ++i) {
                uint64_t st = ~0ull, en = 0;
                for (uint32_t b = 0; b < grid; ++b) {
                    st = std::min(st, hts[((size_t)i * grid + b) * 2]);
                    en = std::max(en, hts[((size_t)i * grid + b) * 2 + 1]);
                }
                body.push_back((double)(en - st) / wclk * 1e3);
                if (i) gap.push_back(((double)st - (double)prev_end) / wclk * 1e3);
                prev_end = en;
            }
            std::sort(body.begin(), body.end());
            std::sort(gap.begin(), gap.end());
            const double us = (t1 - t0) / K * 1e6;
            printf("r%d %-22s call %7.2f us (%.4f of 8 TB/s) | GPU body median %7.2f us | gap median %6.2f p10 %6.2f p90 %6.2f\n",
                   r, v.name.c_str(), us, alg / (us * 1e-6) / 8e12, body[K / 2], gap[gap.size() / 2], gap[gap.size() / 10],
                   gap[gap.size() * 9 / 10]);
            fflush(stdout);
        }
    }
    printf("self-completion fallbacks: %d\n", fallbacks);
    // correctness of the self-completing hybrid: result read on another stream right after the word
    if (selfh) {
        hipStream_t s2;
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        std::vector<float> a(n), b(n), got(n);
        const uint32_t from64 = grid - (uint32_t)((64ull << 20) / 16384);
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemcpy(a.data(), io(rep), bytes, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), in(rep), bytes, hipMemcpyDeviceToHost));
            CK(hipDeviceSynchronize());
            const uint32_t q = ++seq;
            hipLaunchKernelGGL(a2_selfh, dim3(grid), dim3(256), 0, s, in(rep), io(rep), bytes, (uint64_t *)nullptr, ctl,
                               (uint32_t *)flag, q, grid, rep == 2 ? 0u : from64);
            selfwait(q, true);
            CK(hipMemcpyAsync(got.data(), io(rep), bytes, hipMemcpyDeviceToHost, s2));
            CK(hipStreamSynchronize(s2));
            size_t bad = 0;
            for (uint64_t k = 0; k < n; ++k) bad += (got[k] != a[k] + b[k]);
            printf("selfh readback on another stream right after the word (rep %d): %zu mismatches\n", rep, bad);
            CK(hipStreamSynchronize(s));
        }
    }
    hsa_queue_destroy(aq.q);
    hsa_signal_destroy(aq.sig);
    return 0;
}
