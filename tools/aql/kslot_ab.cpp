// kslot_ab.cpp -- the direct dispatch's kernarg protocols, interleaved call by
// call in one process (so clock / thermal drift hits every variant alike):
// 256 MiB fp32 SUM, synchronous (doorbell -> completion signal), 4 rotating
// operand pairs, the product's tile kernel from two code objects -- round 2's
// (old: LeanArgs, no check) and the current one (KargSlot; mpir_tile_ reads it
// as it stands, mpir_ctile_ checks the nonce against its dispatch id):
//   old_hit        old kernel, cached slot: no host writes
//   old_miss       old kernel, args written + HDP flush + flush read back
//   new_hit        checked kernel, nonce words stamped + HDP flush
//   new_hit_nf     checked kernel, nonce words stamped, no flush
//   new_miss       checked kernel, args + nonce + HDP flush (the product's miss)
//   new_miss_nf    checked kernel, args + nonce, no flush
//   new_miss_late  new_miss with the args, nonce and flush written after the
//                  doorbell (the product since round 3's late-write change)
//   new_hit_rb     checked kernel, nonce + HDP flush + read back
//   new_nostamp    checked kernel, slot pre-stamped with the largest nonce: no
//                  host writes (isolates the checked prologue)
//   old_hit_touch  old kernel, cached slot, 16 B written into the same 128 B
//                  line (not the argument bytes), no flush (isolates the cost
//                  of a freshly host-written kernarg line)
//   plain_hit      unchecked kernel, cached slot: no host writes (the product's
//                  verified hit)
// Prints per variant the median / p10 / p90 host wall time per call and, from
// the CP's dispatch timestamps (the queue records them: KSLOT_TS=1, which adds
// the same ~0.4 us to every variant), the median kernel duration.
//   HSA_ALLOCATE_QUEUE_DEV_MEM=1 tools/aql/kslot_ab <old.hsaco | -> <new.hsaco> [calls per variant]
//   (bash tools/aql/build_kslot.sh)
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_; hsa_status_string(s_, &m_); printf("HSA %s line %d: %s\n", #x, __LINE__, m_); exit(3);} } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static hsa_agent_t g_gpu, g_cpu;
static uint32_t g_bdf;
static hsa_amd_memory_pool_t g_vram;
static bool g_have_cpu = false, g_have_vram = false, g_have_gpu = false;

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) { g_cpu = a; g_have_cpu = true; }
    if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) {
        uint32_t bdf = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        if ((bdf & ~7u) == g_bdf) { g_gpu = a; g_have_gpu = true; }
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

static uint64_t load_kernel(const char *path, const char *sym) {
    FILE *fp = fopen(path, "rb");
    if (!fp) { printf("cannot open %s\n", path); exit(4); }
    std::vector<char> co;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0) co.insert(co.end(), buf, buf + n);
    fclose(fp);
    hsa_code_object_reader_t rd;
    hsa_executable_t exe;
    HK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    HK(hsa_executable_load_agent_code_object(exe, g_gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(exe, nullptr));
    hsa_executable_symbol_t s;
    HK(hsa_executable_get_symbol_by_name(exe, sym, &g_gpu, &s));
    uint64_t ko = 0;
    HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko));
    return ko;
}

int main(int argc, char **argv) {
    if (argc < 3) { printf("usage: kslot_ab old.hsaco new.hsaco [calls]\n"); return 1; }
    const int calls = argc > 3 ? atoi(argv[3]) : 200;
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    g_bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    HK(hsa_init());
    hsa_iterate_agents(find_agents, nullptr);
    if (!g_have_gpu || !g_have_cpu) { printf("agents not found\n"); return 5; }
    hsa_amd_agent_iterate_memory_pools(g_gpu, find_vram, nullptr);
    hsa_amd_hdp_flush_t hdp{};
    HK(hsa_agent_get_info(g_gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp));
    volatile uint32_t *flush = hdp.HDP_MEM_FLUSH_CNTL;
    // "-" for old.hsaco: no round-2 code object, the old_* variants are skipped
    const bool have_old = strcmp(argv[1], "-") != 0;
    const uint64_t ko_old = have_old ? load_kernel(argv[1], "mpir_tile_SUM_MPIR_HIP_F32.kd") : 0;
    const uint64_t ko_new = load_kernel(argv[2], "mpir_ctile_SUM_MPIR_HIP_F32.kd");
    const uint64_t ko_plain = load_kernel(argv[2], "mpir_tile_SUM_MPIR_HIP_F32.kd");

    const size_t n = 64ull << 20, bytes = n * 4;
    char *bufs[8];
    for (auto &b : bufs) { CK(hipMalloc(&b, bytes)); CK(hipMemset(b, 0x3c, bytes)); }
    CK(hipDeviceSynchronize());
    void *kp = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_vram, 64 * 128, 0, &kp));
    HK(hsa_amd_agents_allow_access(1, &g_cpu, nullptr, kp));
    char *karg = static_cast<char *>(kp);
    void *ew = nullptr;
    CK(hipHostMalloc(&ew, 64, hipHostMallocCoherent | hipHostMallocMapped));
    memset(ew, 0, 64);
    hsa_queue_t *q = nullptr;
    HK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    const bool ts = getenv("KSLOT_TS") && atoi(getenv("KSLOT_TS"));
    if (ts) HK(hsa_amd_profiling_set_profiler_enabled(q, 1));
    uint64_t freq = 1;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq);
    hsa_signal_t sig;
    HK(hsa_signal_create(0, 1, &g_gpu, &sig));

    // slot s (0..31): pair s % 4; slots 0-3 "cached" (args written once), 4.. rewritten per call
    struct Lean { const char *in; char *io; uint64_t vbytes; uint64_t keep; };
    auto lean = [&](int pair) { return Lean{bufs[2 * pair + 1], bufs[2 * pair], bytes, 0}; };
    auto write_old = [&](char *slot, int pair) { Lean a = lean(pair); memcpy(slot, &a, sizeof a); };
    auto write_new_args = [&](char *slot, int pair) {
        uint64_t w[16] = {};
        Lean a = lean(pair);
        memcpy(w, &a, sizeof a);
        w[6] = (uint64_t)(uintptr_t)ew;
        uint64_t *ks = reinterpret_cast<uint64_t *>(slot);
        for (int i = 0; i < 6; ++i) { ks[i] = w[i]; ks[8 + i] = w[8 + i]; }
        ks[6] = w[6];
    };
    // cached old slots 0-3 and new slots 8-11, written once and flushed with read-back
    for (int p = 0; p < 4; ++p) {
        write_old(karg + p * 128, p);
        write_new_args(karg + (8 + p) * 128, p);
        write_new_args(karg + (12 + p) * 128, p);      // new_nostamp
        uint64_t *ks = reinterpret_cast<uint64_t *>(karg + (12 + p) * 128);
        ks[7] = ks[15] = ~0ull;
        write_old(karg + (32 + p) * 128, p);            // old_hit_touch
        write_new_args(karg + (36 + p) * 128, p);       // plain_hit
    }
    _mm_sfence();
    *flush = 1u;
    (void)*flush;

    enum { OLD_HIT, OLD_MISS, NEW_HIT, NEW_HIT_NF, NEW_MISS, NEW_MISS_NF, NEW_HIT_RB, NEW_NOSTAMP, OLD_HIT_TOUCH,
           PLAIN_HIT, NEW_MISS_LATE, NV };
    const char *names[NV] = {"old_hit", "old_miss", "new_hit", "new_hit_nf", "new_miss", "new_miss_nf", "new_hit_rb",
                             "new_nostamp", "old_hit_touch", "plain_hit", "new_miss_late"};
    std::vector<double> t[NV], kt[NV];
    const uint32_t groups = (uint32_t)(bytes / 16384);
    int call = 0;
    for (int it = 0; it < calls + 10; ++it) {
        for (int v = 0; v < NV; ++v, ++call) {
            if (!have_old && (v == OLD_HIT || v == OLD_MISS || v == OLD_HIT_TOUCH)) continue;
            const int pair = call % 4;
            const double t0 = now();
            const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
            char *slot;
            uint64_t ko;
            switch (v) {
            case OLD_HIT: slot = karg + pair * 128; ko = ko_old; break;
            case OLD_MISS:
                slot = karg + (4 + pair) * 128; ko = ko_old;
                write_old(slot, pair); _mm_sfence(); *flush = 1u; (void)*flush; break;
            case NEW_HIT: case NEW_HIT_NF: case NEW_HIT_RB: {
                slot = karg + (8 + pair) * 128; ko = ko_new;
                uint64_t *ks = reinterpret_cast<uint64_t *>(slot);
                ks[7] = idx + 1; ks[15] = idx + 1; _mm_sfence();
                if (v != NEW_HIT_NF) *flush = 1u;
                if (v == NEW_HIT_RB) (void)*flush;
                break;
            }
            case NEW_NOSTAMP: slot = karg + (12 + pair) * 128; ko = ko_new; break;
            case PLAIN_HIT: slot = karg + (36 + pair) * 128; ko = ko_plain; break;
            case NEW_MISS_LATE: slot = karg + (40 + (call % 16)) * 128; ko = ko_new; break;   // written below
            case OLD_HIT_TOUCH: {
                slot = karg + (32 + pair) * 128; ko = ko_old;
                uint64_t *ks = reinterpret_cast<uint64_t *>(slot);
                ks[8] = idx; ks[9] = idx; _mm_sfence();
                break;
            }
            default: {
                slot = karg + (16 + (call % 16)) * 128; ko = ko_new;
                write_new_args(slot, pair); _mm_sfence();
                uint64_t *ks = reinterpret_cast<uint64_t *>(slot);
                ks[7] = idx + 1; ks[15] = idx + 1; _mm_sfence();
                if (v == NEW_MISS) *flush = 1u;
                break;
            }
            }
            hsa_signal_store_relaxed(sig, 1);
            hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
            memset((char *)p + 4, 0, sizeof(*p) - 4);
            p->workgroup_size_x = 256; p->workgroup_size_y = 1; p->workgroup_size_z = 1;
            p->grid_size_x = groups * 256; p->grid_size_y = 1; p->grid_size_z = 1;
            p->kernel_object = ko;
            p->kernarg_address = slot;
            p->completion_signal = sig;
            const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                    (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                    (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
            hsa_queue_store_write_index_relaxed(q, idx + 1);
            _mm_sfence();
            __atomic_store_n((uint32_t *)p, (uint32_t)header | (1u << 16), __ATOMIC_RELEASE);
            hsa_signal_store_screlease(q->doorbell_signal, idx);
            if (v == NEW_MISS_LATE) {
                write_new_args(slot, pair); _mm_sfence();
                uint64_t *ks = reinterpret_cast<uint64_t *>(slot);
                ks[7] = idx + 1; ks[15] = idx + 1; _mm_sfence();
                *flush = 1u;
            }
            while (hsa_signal_load_scacquire(sig) != 0) _mm_pause();
            const double dt = now() - t0;
            if (it >= 10) t[v].push_back(dt * 1e6);
            if (it >= 10 && ts) {
                hsa_amd_profiling_dispatch_time_t pt{};
                if (hsa_amd_profiling_get_dispatch_time(g_gpu, sig, &pt) == HSA_STATUS_SUCCESS)
                    kt[v].push_back((double)(pt.end - pt.start) * 1e6 / (double)freq);
            }
        }
    }
    if (*(volatile uint32_t *)ew) printf("ERROR WORD SET\n");
    for (int v = 0; v < NV; ++v) {
        if (t[v].empty()) continue;
        std::sort(t[v].begin(), t[v].end());
        const size_t m = t[v].size();
        double mean = 0;
        for (double x : t[v]) mean += x;
        mean /= (double)m;
        printf("%-12s median %8.2f us  p10 %8.2f  p90 %8.2f  p99 %8.2f  max %8.2f  mean %8.2f  (%zu calls)", names[v],
               t[v][m / 2], t[v][m / 10], t[v][m * 9 / 10], t[v][m * 99 / 100], t[v][m - 1], mean, m);
        if (!kt[v].empty()) {
            std::sort(kt[v].begin(), kt[v].end());
            printf("  kernel median %8.2f us", kt[v][kt[v].size() / 2]);
        }
        printf("\n");
    }
    return 0;
}
