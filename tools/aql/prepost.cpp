// prepost.cpp -- synchronous 256 MiB / 64 MiB fp32 SUM calls two ways on one
// HSA queue (AQL ring in VRAM when HSA_ALLOCATE_QUEUE_DEV_MEM=1):
//   plain    the product's direct dispatch: packet + doorbell per call, wait on
//            the packet's completion signal (kernargs cached per operand pair);
//   prepost  each call writes its arguments and a sequence number into a VRAM
//            mailbox (BAR + HDP flush) for the gated kernel that the previous
//            call already queued (tools/aql/prepost_kernel.hip), queues the
//            NEXT call's gated kernel (so its dispatch overlaps this call's
//            kernel), then waits on this call's completion signal.
// Every call's result is checked (inbuf = 1.0f, inoutbuf counts the calls on
// its pair; sampled elements over the whole buffer) and every gate's decision
// is read back.  Modes alternate, 4 rounds each.
//   tools/aql/build_prepost.sh && HSA_ALLOCATE_QUEUE_DEV_MEM=1 tools/aql/prepost tools/aql/prepost_kernel.co
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_; hsa_status_string(s_, &m_); \
    printf("HSA %s line %d: %s\n", #x, __LINE__, m_); exit(3);} } while (0)

static hsa_agent_t g_gpu, g_cpu;
static bool g_have_gpu = false, g_have_cpu = false;
static hsa_amd_memory_pool_t g_vram, g_fine;
static bool g_have_vram = false, g_have_fine = false;
static uint64_t g_freq = 0;
static volatile uint32_t *g_hdp = nullptr;

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
    if (w == 2 && (f & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !g_have_fine) { g_fine = p; g_have_fine = true; }
    return HSA_STATUS_SUCCESS;
}
static uint64_t ts() {
    uint64_t t = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    return t;
}
static double us(uint64_t dt) { return (double)(int64_t)dt * 1e6 / (double)g_freq; }

static void *vram_alloc(size_t bytes) {
    void *p = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_vram, bytes, 0, &p));
    HK(hsa_amd_agents_allow_access(1, &g_cpu, nullptr, p));
    return p;
}
static void *fine_alloc(size_t bytes) {
    void *p = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_fine, bytes, 0, &p));
    HK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, p));
    memset(p, 0, bytes);
    return p;
}
static void hdp_flush(bool readback) {
    _mm_sfence();
    *g_hdp = 1u;
    if (readback) (void)*g_hdp;
}

struct Mail { uint64_t in, io, vbytes, keep; uint32_t seq; uint32_t pad[23]; };
struct PlainArgs { const void *in; void *io; uint64_t vbytes, keep; };
struct DirectArgs { const uint32_t *seqs; const Mail *mail; uint32_t k; uint32_t pad0; uint64_t ticks; uint32_t sleep;
                    uint32_t pad1; };
struct GateArgs { const Mail *mail; uint32_t *dec; uint32_t *outcome; uint32_t k; uint32_t pad0; uint64_t lead, follow;
                  uint32_t sleep; uint32_t pad1; };

static hsa_queue_t *q;
static uint64_t ko_plain, ko_gate, ko_direct;
static uint32_t ks_plain, ks_gate, ks_direct;

static void post(uint64_t ko, const void *karg, uint32_t grid_wg, hsa_signal_t sig) {
    hsa_signal_store_relaxed(sig, 1);
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
    p->workgroup_size_x = 256; p->workgroup_size_y = 1; p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = 256u * grid_wg; p->grid_size_y = 1; p->grid_size_z = 1;
    p->private_segment_size = 0;
    p->group_segment_size = 64;
    p->kernel_object = ko;
    p->kernarg_address = (void *)karg;
    p->reserved2 = 0;
    p->completion_signal = sig;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    _mm_sfence();
    __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, idx);
}
static bool wait_sig(hsa_signal_t s) {
    const uint64_t t0 = ts();
    while (hsa_signal_load_scacquire(s) > 0) {
        _mm_pause();
        if (us(ts() - t0) > 2e6) return false;
    }
    return true;
}

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: %s prepost_kernel.co [calls [sleep...]]\n", argv[0]); return 1; }
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int calls = argc > 2 ? atoi(argv[2]) : 200;
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    hsa_amd_agent_iterate_memory_pools(g_gpu, find_pool, (void *)0);
    hsa_amd_agent_iterate_memory_pools(g_cpu, find_pool, (void *)2);
    if (!g_have_gpu || !g_have_vram || !g_have_fine) { printf("agents / pools not found\n"); return 1; }
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
    auto sym = [&](const char *name, uint64_t *ko, uint32_t *kas) {
        hsa_executable_symbol_t s;
        HK(hsa_executable_get_symbol_by_name(exe, name, &g_gpu, &s));
        HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, ko));
        HK(hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, kas));
        uint32_t lds = 0, priv = 0;
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &lds);
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv);
        printf("%s: kernarg %u B, lds %u B, scratch %u B\n", name, *kas, lds, priv);
        if (lds > 64 || priv) { printf("unexpected LDS / scratch\n"); exit(1); }
    };
    sym("plain_tile.kd", &ko_plain, &ks_plain);
    sym("gated_tile.kd", &ko_gate, &ks_gate);
    sym("direct_gate_tile.kd", &ko_direct, &ks_direct);
    std::vector<uint32_t> sleeps;
    for (int a = 3; a < argc; ++a) sleeps.push_back((uint32_t)atoi(argv[a]));
    if (sleeps.empty()) sleeps = {0, 4};
    if (ks_plain > sizeof(PlainArgs) || ks_gate > sizeof(GateArgs) || ks_gate < 52 || ks_direct > sizeof(DirectArgs)) {
        printf("kernarg size mismatch: %u vs %zu, %u vs %zu\n", ks_plain, sizeof(PlainArgs), ks_gate, sizeof(GateArgs));
        return 1;
    }
    HK(hsa_queue_create(g_gpu, 256, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    hsa_amd_hdp_flush_t h{};
    HK(hsa_agent_get_info(g_gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &h));
    g_hdp = h.HDP_MEM_FLUSH_CNTL;

    const size_t MB = 1 << 20, big = 256 * MB;
    const int NP = 4;
    float *in[NP], *io[NP];
    for (int i = 0; i < NP; ++i) {
        in[i] = (float *)vram_alloc(big);
        io[i] = (float *)vram_alloc(big);
        HK(hsa_amd_memory_fill(in[i], 0x3f800000u, big / 4));
    }
    Mail *mail = (Mail *)vram_alloc(4096);
    uint32_t *dec = (uint32_t *)vram_alloc(4096);
    uint32_t *seqs = (uint32_t *)vram_alloc(4096);
    memset(seqs, 0, 4096);
    uint32_t *outcome = (uint32_t *)fine_alloc(64 * 128);
    memset(mail, 0, sizeof(Mail));
    memset(dec, 0, 4096);
    hdp_flush(true);
    // kernarg slots in VRAM: 64 windows for plain (cached), 64 ring slots for gates
    char *karg = (char *)vram_alloc(192 * 128);
    std::vector<hsa_signal_t> sig(64);
    for (auto &s : sig) HK(hsa_signal_create(1, 0, nullptr, &s));
    std::vector<hsa_signal_t> sigb(64);
    for (auto &s : sigb) HK(hsa_signal_create(1, 0, nullptr, &s));
    float *hostbuf = (float *)fine_alloc(4096);

    const uint64_t lead = 10000, follow = 1000000;   // 100 us, 10 ms at 100 MHz
    uint32_t gate_k = 0;                             // sequence numbers keep rising across runs

    for (int mib : {256, 64}) {
        const uint64_t vbytes = (uint64_t)mib * MB;
        const uint32_t grid = (uint32_t)(vbytes / 16384);
        const int nwin = NP * (int)(big / vbytes);          // 4 pairs at 256 MiB, 16 windows at 64 MiB
        for (int w = 0; w < nwin && w < 64; ++w) {
            const int p = w % NP, off = (w / NP) * (int)(vbytes / 4);
            PlainArgs a{in[p] + off, io[p] + off, vbytes, 0};
            memcpy(karg + w * 128, &a, sizeof a);
        }
        // split mode: the pre-posted gate covers the first wave of tiles (kFirst
        // workgroups, one per resident slot), a plain kernel posted at call time the rest
        const uint32_t kFirst = 2048;
        const uint64_t first_bytes = std::min<uint64_t>(vbytes, (uint64_t)kFirst * 16384);
        for (int w = 0; w < nwin && w < 64; ++w) {
            const int p = w % NP, off = (w / NP) * (int)(vbytes / 4);
            PlainArgs a{(char *)(in[p] + off) + first_bytes, (char *)(io[p] + off) + first_bytes, vbytes - first_bytes, 0};
            memcpy(karg + (128 + w) * 128, &a, sizeof a);
        }
        hdp_flush(true);
        struct Mode { int kind; uint32_t sleep; };
        std::vector<Mode> modes{{0, 0}};
        if (!getenv("PLAIN_ONLY"))
            for (uint32_t sl : sleeps) { modes.push_back({1, sl}); modes.push_back({2, sl}); modes.push_back({3, sl}); }
        static const char *kname[4] = {"plain", "gate", "direct", "split"};
        const int nrounds = getenv("ROUNDS") ? atoi(getenv("ROUNDS")) : 2;
        for (int round = 0; round < nrounds; ++round) {
            for (const Mode &md : modes) {
                const int mode = md.kind;
                for (int i = 0; i < NP; ++i) HK(hsa_amd_memory_fill(io[i], 0u, big / 4));
                std::vector<int> cnt(nwin, 0);
                std::vector<double> per;
                int fails = 0, lost = 0;
                uint64_t t_start = 0;
                const int warm = 20;
                auto arm = [&](uint32_t kk) {     // queue the gate kernel for call kk
                    char *slot = karg + (64 + (kk & 63)) * 128;
                    if (mode == 1) {
                        GateArgs g{mail, dec, outcome + (kk & 63) * 32, kk, 0, lead, follow, md.sleep, 0};
                        memcpy(slot, &g, sizeof g);
                        hdp_flush(true);
                        post(ko_gate, slot, grid, sig[kk & 63]);
                    } else {
                        DirectArgs g{seqs, mail, kk, 0, lead, md.sleep, 0};
                        memcpy(slot, &g, sizeof g);
                        hdp_flush(true);
                        post(ko_direct, slot, mode == 3 ? std::min(grid, kFirst) : grid, sig[kk & 63]);
                    }
                };
                if (mode != 0) arm(++gate_k);
                for (int c = 0; c < warm + calls; ++c) {
                    if (c == warm) t_start = ts();
                    const int w = c % nwin;
                    const uint64_t t0 = ts();
                    if (mode == 0) {
                        post(ko_plain, karg + w * 128, grid, sig[c & 63]);
                        if (!wait_sig(sig[c & 63])) { lost++; break; }
                    } else {
                        const uint32_t k = gate_k;
                        const int p = w % NP, off = (w / NP) * (int)(vbytes / 4);
                        mail->in = (uint64_t)(in[p] + off);
                        mail->io = (uint64_t)(io[p] + off);
                        mail->vbytes = mode == 3 ? first_bytes : vbytes;
                        mail->keep = 0;
                        _mm_sfence();
                        if (mode == 1) {
                            __atomic_store_n(&mail->seq, k, __ATOMIC_RELEASE);
                        } else {
                            for (int r = 0; r < 8; ++r) __atomic_store_n(seqs + r * 32, k, __ATOMIC_RELEASE);   // direct, split
                        }
                        hdp_flush(false);
                        const bool rest = mode == 3 && vbytes > first_bytes;
                        if (rest) post(ko_plain, karg + (128 + w) * 128, grid - kFirst, sigb[c & 63]);
                        arm(++gate_k);          // the next call's gate, queued behind this one
                        if (!wait_sig(sig[k & 63])) { lost++; break; }
                        if (rest && !wait_sig(sigb[c & 63])) { lost++; break; }
                        if (mode == 1) {
                            const uint32_t v = __atomic_load_n(outcome + (k & 63) * 32, __ATOMIC_ACQUIRE);
                            if (v != ((k << 1) | 1u)) fails++;
                        }
                    }
                    cnt[w]++;
                    if (c >= warm) per.push_back(us(ts() - t0));
                }
                const double tot = us(ts() - t_start);
                if (mode != 0) {       // the last armed gate expires on its own (lead timeout)
                    if (!wait_sig(sig[gate_k & 63])) lost++;
                    if (mode == 1) {
                        const uint32_t v = __atomic_load_n(outcome + (gate_k & 63) * 32, __ATOMIC_ACQUIRE);
                        if (v != (gate_k << 1)) printf("  last gate: outcome %#x, expected expired %#x\n", v, gate_k << 1);
                    }
                }
                if (lost) { printf("LOST a completion signal: stopping\n"); _exit(4); }
                // check: io window w holds cnt[w] in every sampled element
                int bad = 0;
                for (int w = 0; w < nwin; ++w) {
                    const int p = w % NP, off = (w / NP) * (int)(vbytes / 4);
                    for (int s = 0; s < 16; ++s) {
                        const size_t e = off + (size_t)s * (vbytes / 4 / 16) + (size_t)(s * 7919) % (vbytes / 4 / 16);
                        HK(hsa_memory_copy(hostbuf, io[p] + e, 4));
                        if (hostbuf[0] != (float)cnt[w]) bad++;
                    }
                }
                std::sort(per.begin(), per.end());
                const double alg = 3.0 * vbytes;
                printf("%3d MiB %-6s sleep %2u round %d: mean call %7.2f us (p10 %7.2f p50 %7.2f p90 %7.2f)  %7.1f GiB/s  "
                       "gate fails %d  bad samples %d\n", mib, kname[mode], md.sleep, round, tot / calls,
                       per[per.size() / 10], per[per.size() / 2], per[per.size() * 9 / 10],
                       alg * calls / (tot * 1e-6) / (1 << 30), fails, bad);
            }
        }
    }
    return 0;
}
