// direct_dispatch.hip -- synchronous device-resident MPI_Reduce_local without
// the HIP launch path: our own AQL queue, the tile kernel from a device-only
// code object (direct_tiles.hip -> lib/libmpir_hip_tiles.hsaco), kernargs in
// VRAM, and a wait on the dispatch packet's own completion signal.
//
// Why (tools/aql/aql2.cpp, profiles/r02/aql2_*.log): a synchronous HIP call
// is hipLaunchKernel + a completion word written by hipStreamWriteValue32,
// which is a second (blit) dispatch; the GPU then sits idle 8.8-8.9 us between
// one call's last workgroup and the next call's first.  A direct dispatch
// waits on the kernel packet's completion signal instead: 7.4-7.5 us, and the
// 256 MiB fp32 SUM call 126.2-126.4 us against 127.6-127.8 (same box, same
// kernel); with the kernarg cache below and the AQL rings in VRAM
// (HSA_ALLOCATE_QUEUE_DEV_MEM=1) the gap is 5.2-5.5 us, 4.3 us of it the CP
// noticing the doorbell (profiles/r02/sync_split_timeline.log, cp_latency.log).  An earlier attempt (round 1) lost because its kernargs sat in host
// memory (every workgroup read them over PCIe); here they are written through
// the BAR into VRAM and made visible with an HDP flush (the register ROCr
// exposes as HSA_AMD_AGENT_INFO_HDP_FLUSH; read back, as HIP does for its
// device kernargs), before the packet header is published.
//
// Scope and ordering (the HIP path is used whenever one does not hold):
//   * synchronous calls on the library's own stream (hip_stream NULL), both
//     operands on one device, any count and alignment: the kernel of
//     plan_reduce's launch plan (lean / full tile, shift, element-granular),
//     for every (op, element) pair the code object carries -- every op but
//     REPLACE on every class but the 32-byte ones;
//   * work the caller queued on the legacy null stream for these buffers stays
//     ordered before the reduction, as with the blocking HIP stream: when
//     hipStreamQuery(NULL) reports pending work (it keeps doing so for finished
//     work until the host synchronises, tools/direct_probe.py), the call first
//     synchronises with the null stream;
//   * the calling thread has no unfinished work on its own library stream.
// Packets carry an agent-scope acquire (what HIP uses between kernels; a
// system-scope acquire costs ~7 us of body, aql_sig_nt_sys) and a
// system-scope release, so the result is visible to every agent -- SDMA
// copies and the host included -- when the signal fires.  One queue per
// device (plus its timestamped twin for profiled calls), shared by the threads; a mutex orders packet publication (single
// producer at a time, doorbell monotonic); no barrier bit, so concurrent
// threads' kernels overlap; each thread waits on its own signal.
// MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip turns the path off.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/amd_hsa_signal.h>
#include <dlfcn.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <time.h>

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mpir_hip_reduce.h"
#include "kernel_table.hpp"

namespace mpir_hip {

namespace {

constexpr int kMaxDirectDev = 64;
constexpr uint32_t kKargSlots = 256, kKargSlotBytes = 128;
// Kernarg slots 0..kRingSlots-1 are a ring for one-off arguments; the rest are
// a direct-mapped cache: a call whose (kernel, arguments) match a cached slot
// dispatches with that slot as it stands -- no BAR write and no HDP flush
// (0.95 us of host time per dispatch with its read-back, tools/aql/aql2.cpp,
// profiles/r02/aql2_host_costs.log).  A reduction schedule that calls again on
// the same buffers, or a caller rotating a few buffer pairs, hits.  A cached
// slot is rewritten only when no dispatch that uses it is in flight.
constexpr uint32_t kRingSlots = 128, kCacheSlots = kKargSlots - kRingSlots;
constexpr uint32_t kQueueSize = 256;

// a plan's argument bytes (LeanArgs / TileArgs / ShiftArgs / ElemsArgs,
// reduce_kernels.hpp; their layouts do not depend on the element type)
constexpr uint32_t kMaxArgBytes = sizeof(ReducePlan::args);
static_assert(kMaxArgBytes <= kKargSlotBytes, "kernarg slot too small");
constexpr uint32_t kPlanArgBytes[kPlanKinds] = {sizeof(LeanArgs), sizeof(TileArgs<char>), sizeof(ShiftArgs<char>),
                                                sizeof(ElemsArgs), sizeof(ElemsArgs)};
const char *const kPlanPrefix[kPlanKinds] = {"mpir_tile_", "mpir_tilex_", "mpir_tiles_", "mpir_elems_", "mpir_elemsu_"};

struct CacheEntry {
    uint64_t ko = 0;
    uint32_t n = 0;                             // argument bytes
    alignas(8) unsigned char args[kMaxArgBytes] = {};
    std::atomic<int> inflight{0};
};

struct DevState {
    std::once_flag once;
    bool ok = false;
    int state = 0;          // 0 not tried, 1 ready, < 0 the init step that failed (MPIR_Hip_direct_state)
    hsa_agent_t agent{};
    hsa_queue_t *queue = nullptr;               // the calls' queue (no dispatch timestamps)
    hsa_queue_t *pqueue = nullptr;              // the same, timestamps on: calls while profiling is on
    std::once_flag ponce;                       // (created at the first profiled call)
    char *karg = nullptr;                       // kKargSlots x kKargSlotBytes, VRAM, host-written
    uint32_t kslot = 0;                         // next ring slot to try (under `publish`)
    std::atomic<int> ring_busy[kRingSlots] = {};  // a ring slot's dispatch is in flight
    CacheEntry cache[kCacheSlots];
    volatile uint32_t *hdp = nullptr;
    uint64_t kobj[kPlanKinds][MPIR_HIP_NOPS][MPIR_HIP_NELEMS] = {};   // by plan kind (kPlanPrefix)
    std::mutex publish;
    std::atomic<int> queue_error{0};
    // keep-alive (keepalive_us()): its queue and no-op kernargs; on a line of
    // their own, the monotonic time of the last call's end or keep-alive packet
    // and whether a call is in flight (a busy CP is not idle: no keep-alive
    // then).  Plain stores on the call path, no read-modify-write.
    hsa_queue_t *kqueue = nullptr;              // created when the keep-alive is first armed
    std::once_flag konce;
    std::atomic<bool> kready{false};
    char *kargs_noop = nullptr;
    alignas(64) std::atomic<uint64_t> last_packet_ns{0};
    std::atomic<uint64_t> last_call_ns{0};      // the keep-alive runs for a window after this
    std::atomic<int> call_busy{0};
    std::atomic<int> armed{0};                  // the caller has been seen to leave gaps
    char pad_[64 - 2 * sizeof(std::atomic<uint64_t>) - 2 * sizeof(std::atomic<int>)];
};

DevState g_dev[kMaxDirectDev];
std::atomic<uint64_t> g_direct_calls{0};
std::atomic<uint64_t> g_busy_skips{0};      // calls that first synchronised with a busy null stream
// MPIX_Reduce_local_profile: the CP's start / end timestamps of each direct
// dispatch (hsa_amd_profiling_get_dispatch_time, what rocprofv3 reads), so a
// benchmark can time the kernel the synchronous call really runs
std::atomic<int> g_profile{0};
thread_local uint64_t t_last_kernel_ns = 0;
// with profiling on, the last direct call's timeline on the system clock, ns
// from entering direct_reduce: doorbell rung, CP start, CP end, signal seen
thread_local uint64_t t_last_split[4] = {};

static inline uint64_t sys_ts() {
    uint64_t t = 0;
    hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &t);
    return t;
}
uint64_t g_ts_freq = 0;

// MPIR_CVAR_REDUCE_LOCAL_WAIT_MWAITX=1 (A/B, AMD hosts with MONITORX): wait for
// the completion signal's value line with MONITORX / MWAITX instead of a
// pause loop (tools/mwaitx_ab.sh)
bool use_mwaitx() {
    static const bool v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_WAIT_MWAITX");
        if (!e || atoi(e) == 0) return false;
        unsigned a, b, c, dd;
        __asm__ volatile("cpuid" : "=a"(a), "=b"(b), "=c"(c), "=d"(dd) : "a"(0x80000001u), "c"(0));
        return ((c >> 29) & 1u) != 0;   // CPUID Fn8000_0001 ECX[29] = MONITORX
    }();
    return v;
}

__attribute__((target("mwaitx"))) void wait_signal_mwaitx(hsa_signal_t sig) {
#if !defined(__HIP_DEVICE_COMPILE__)     // host code; the device pass never emits it
    volatile int64_t *v = &reinterpret_cast<amd_signal_t *>(sig.handle)->value;
    while (__atomic_load_n(v, __ATOMIC_ACQUIRE) != 0) {
        __builtin_ia32_monitorx((void *)v, 0, 0);
        if (__atomic_load_n(v, __ATOMIC_ACQUIRE) == 0) break;
        __builtin_ia32_mwaitx(0x2, 0, 20000);   // ECX bit 1: EBX timer, at most ~20000 TSC ticks
    }
#else
    (void)sig;
#endif
}

uint64_t mono_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// Keep-alive: after 50-100 us without a packet the command processor drops
// into a deeper idle state and the next doorbell takes ~10 us instead of ~5 to
// start the kernel (tools/idle_gap_probe.py: a 4 MiB call 9.6 us after a 50 us
// host gap, 14.9-15.5 us after 100 us-5 ms), which every combine step of a
// schedule that waits on the network would pay.  A kernel in flight on another
// queue does not prevent it (tools/idle_sleep_probe.py): it is the CP's
// doorbell handling that sleeps.  MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US = P
// (opt-in, e.g. 40; default 0 = off -- with it on, bench.py's back-to-back loop
// measured 0.763-0.786 against 0.79-0.80: profiles/r02/keepalive_default_bench.log): a call that arrives more than P + 10 us after the
// previous one ends arms the keep-alive, one that arrives within P us disarms
// it; while armed and within MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_MS (default 20)
// of the last call, a library thread puts an empty barrier-AND packet on the
// calls' own queue whenever no packet has gone for P us and no call is in
// flight.  Sparse callers then take ~10 us after any gap instead of ~15, with
// no slow outliers and no cost to back-to-back loops
// (tools/keepalive_same_ab.sh, profiles/r02/keepalive_same_ab.log).  On a queue
// of its own (_QUEUE=own) the packets made the hardware scheduler map one more
// active queue: calls that met them took ~18 us longer (tools/ka_probe.py,
// profiles/r02/ka_probe.log, keepalive_headline_ab.log, lazy_queues_ab.log).
// _KIND=kernel (one workgroup of the SUM tile kernel with nothing to do) and
// _QUEUE=same (the calls' queue) are the A/B's other variants, no better.
// Idle for longer than the window, the thread naps 1 ms at a time.
int keepalive_us() {
    static const int v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US");
        const int us = e ? atoi(e) : 0;
        return us > 0 && us <= 100000 ? us : 0;
    }();
    return v;
}
int keepalive_kernel() {
    static const int v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_KIND");
        return (e && !strcmp(e, "kernel")) ? 1 : 0;
    }();
    return v;
}
int keepalive_own_queue() {
    static const int v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_QUEUE");
        return (e && !strcmp(e, "own")) ? 1 : 0;
    }();
    return v;
}
uint64_t keepalive_active_ns() {
    static const uint64_t v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_MS");
        const long ms = e ? atol(e) : 20;
        return (uint64_t)(ms > 0 && ms <= 60000 ? ms : 20) * 1000000ull;
    }();
    return v;
}

int mode() {
    static const int m = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_DISPATCH");
        return (e && !strcmp(e, "hip")) ? 0 : 1;
    }();
    return m;
}

// Dispatch timestamps cost the synchronous call ~0.4 us at 256 MiB and ~0.9 us
// at 64 MiB (the CP writes start / end times per packet; alternated processes,
// tools/ts_ab.sh, profiles/r02/ts_ab.log), and switching them on for a live
// queue does not take effect (tools/ts_enable_probe.py).  So the calls' queue
// runs without them and a second queue, created with them on, takes the calls
// made while MPIR_Hip_direct_profile is on (the bench's roofline readout: the
// same kernel object, plan and arguments).
// MPIR_CVAR_REDUCE_LOCAL_DIRECT_TIMESTAMPS=1 turns them on for the calls' queue
// too (the round-2 behaviour, for A/Bs).
int timestamps() {
    static const int t = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_DIRECT_TIMESTAMPS");
        return e ? (atoi(e) != 0) : 0;
    }();
    return t;
}

// packet fence scopes (experiments: MPIR_CVAR_REDUCE_LOCAL_DIRECT_ACQUIRE /
// _RELEASE = none | agent | system); defaults agent acquire, system release
static int scope_env(const char *name, int dflt) {
    const char *e = getenv(name);
    if (!e) return dflt;
    if (!strcmp(e, "none")) return HSA_FENCE_SCOPE_NONE;
    if (!strcmp(e, "agent")) return HSA_FENCE_SCOPE_AGENT;
    if (!strcmp(e, "system")) return HSA_FENCE_SCOPE_SYSTEM;
    return dflt;
}
int acquire_scope() {
    static const int v = scope_env("MPIR_CVAR_REDUCE_LOCAL_DIRECT_ACQUIRE", HSA_FENCE_SCOPE_AGENT);
    return v;
}
int release_scope() {
    static const int v = scope_env("MPIR_CVAR_REDUCE_LOCAL_DIRECT_RELEASE", HSA_FENCE_SCOPE_SYSTEM);
    return v;
}

// MPIR_CVAR_REDUCE_LOCAL_DIRECT_SIGNAL: "memory" (default, 0) or "interrupt" (1)
int signal_kind() {
    static const int k = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_DIRECT_SIGNAL");
        return (e && !strcmp(e, "interrupt")) ? 1 : 0;
    }();
    return k;
}

struct Find {
    uint32_t bdf, domain;
    hsa_agent_t gpu{}, cpu{};
    bool have_gpu = false, have_cpu = false;
    hsa_amd_memory_pool_t vram{};
    bool have_vram = false;
};

hsa_status_t find_agent(hsa_agent_t a, void *p) {
    Find *f = static_cast<Find *>(p);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
        f->cpu = a;
        f->have_cpu = true;
    } else if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if (bdf == f->bdf && dom == f->domain) {
            f->gpu = a;
            f->have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t find_vram(hsa_amd_memory_pool_t p, void *arg) {
    Find *f = static_cast<Find *>(arg);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) {
        f->vram = p;
        f->have_vram = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

void queue_error_cb(hsa_status_t status, hsa_queue_t *q, void *data) {
    (void)q;
    DevState *d = static_cast<DevState *>(data);
    d->queue_error.store((int)status ? (int)status : -1);
    const char *msg = nullptr;
    hsa_status_string(status, &msg);
    fprintf(stderr, "mpir_hip: direct-dispatch queue error: %s\n", msg ? msg : "?");
}

// the code object sits next to this library
std::string tiles_path() {
    Dl_info info;
    if (!dladdr((void *)&tiles_path, &info) || !info.dli_fname) return "";
    std::string p = info.dli_fname;
    const size_t slash = p.rfind('/');
    p = (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) + "/libmpir_hip_tiles.hsaco";
    return p;
}

const char *op_name(int op) {
    switch (op) {
    case MPIR_HIP_OP_SUM: return "SUM";
    case MPIR_HIP_OP_PROD: return "PROD";
    case MPIR_HIP_OP_MAX: return "MAX";
    case MPIR_HIP_OP_MIN: return "MIN";
    case MPIR_HIP_OP_LAND: return "LAND";
    case MPIR_HIP_OP_LOR: return "LOR";
    case MPIR_HIP_OP_LXOR: return "LXOR";
    case MPIR_HIP_OP_BAND: return "BAND";
    case MPIR_HIP_OP_BOR: return "BOR";
    case MPIR_HIP_OP_BXOR: return "BXOR";
    case MPIR_HIP_OP_MAXLOC: return "MAXLOC";
    case MPIR_HIP_OP_MINLOC: return "MINLOC";
    default: return nullptr;
    }
}

const char *elem_name(int e) {
#define N(E) case E: return #E;
    switch (e) {
        N(MPIR_HIP_I8) N(MPIR_HIP_U8) N(MPIR_HIP_I16) N(MPIR_HIP_U16) N(MPIR_HIP_I32) N(MPIR_HIP_U32)
        N(MPIR_HIP_I64) N(MPIR_HIP_U64) N(MPIR_HIP_F16) N(MPIR_HIP_F32) N(MPIR_HIP_F64) N(MPIR_HIP_CF32)
        N(MPIR_HIP_CF64) N(MPIR_HIP_P2INT) N(MPIR_HIP_PFLOATINT) N(MPIR_HIP_PLONGINT) N(MPIR_HIP_PSHORTINT)
        N(MPIR_HIP_PDOUBLEINT) N(MPIR_HIP_F80)
    default: return nullptr;
    }
#undef N
}

void init_dev(int dev, DevState &d) {
    d.state = -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) { (void)hipGetLastError(); return; }
    Find f;
    f.bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    f.domain = (uint32_t)prop.pciDomainID;
    d.state = -2;
    if (hsa_init() != HSA_STATUS_SUCCESS) return;
    hsa_iterate_agents(find_agent, &f);
    d.state = -3;
    if (!f.have_gpu || !f.have_cpu) return;
    hsa_amd_agent_iterate_memory_pools(f.gpu, find_vram, &f);
    d.state = -4;
    if (!f.have_vram) return;
    d.state = -5;
    hsa_amd_hdp_flush_t hdp{};
    if (hsa_agent_get_info(f.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp) != HSA_STATUS_SUCCESS ||
        !hdp.HDP_MEM_FLUSH_CNTL)
        return;
    // code object
    d.state = -6;
    const std::string path = tiles_path();
    FILE *fp = path.empty() ? nullptr : fopen(path.c_str(), "rb");
    if (!fp) return;
    std::vector<char> co;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0) co.insert(co.end(), buf, buf + n);
    fclose(fp);
    d.state = -7;
    hsa_code_object_reader_t rd;
    hsa_executable_t exe;
    if (hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd) != HSA_STATUS_SUCCESS) return;
    if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_load_agent_code_object(exe, f.gpu, rd, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        hsa_executable_freeze(exe, nullptr) != HSA_STATUS_SUCCESS)
        return;     // (the reader and executable live as long as the process)
    d.state = -8;
    int found = 0;
    for (int op = 1; op < MPIR_HIP_NOPS; ++op) {
        for (int e = 1; e < MPIR_HIP_NELEMS; ++e) {
            if (!op_name(op) || !elem_name(e)) continue;
            // every plan kind, each with the argument size the host writes
            for (int kind = 0; kind < kPlanKinds; ++kind) {
                const std::string sym = std::string(kPlanPrefix[kind]) + op_name(op) + "_" + elem_name(e) + ".kd";
                hsa_executable_symbol_t s;
                uint64_t ko = 0;
                uint32_t kas = 0, lds = 1, priv = 1;
                if (hsa_executable_get_symbol_by_name(exe, sym.c_str(), &f.gpu, &s) != HSA_STATUS_SUCCESS) continue;
                // the packets carry no LDS or scratch: a kernel that needs either
                // (or reads arguments the host does not write) stays on the HIP path
                if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &ko) !=
                        HSA_STATUS_SUCCESS ||
                    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kas) !=
                        HSA_STATUS_SUCCESS ||
                    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &lds) !=
                        HSA_STATUS_SUCCESS ||
                    hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv) !=
                        HSA_STATUS_SUCCESS ||
                    kas != kPlanArgBytes[kind] || lds != 0 || priv != 0)
                    continue;
                d.kobj[kind][op][e] = ko;
                ++found;
            }
        }
    }
    if (!found) return;
    // kernargs in VRAM, host-writable
    d.state = -9;
    void *kp = nullptr;
    if (hsa_amd_memory_pool_allocate(f.vram, (size_t)kKargSlots * kKargSlotBytes, 0, &kp) != HSA_STATUS_SUCCESS) return;
    if (hsa_amd_agents_allow_access(1, &f.cpu, nullptr, kp) != HSA_STATUS_SUCCESS) {
        hsa_amd_memory_pool_free(kp);
        return;
    }
    d.state = -10;
    if (hsa_queue_create(f.gpu, kQueueSize, HSA_QUEUE_TYPE_MULTI, queue_error_cb, &d, UINT32_MAX, UINT32_MAX,
                         &d.queue) != HSA_STATUS_SUCCESS) {
        hsa_amd_memory_pool_free(kp);
        return;
    }
    d.agent = f.gpu;
    if (timestamps()) hsa_amd_profiling_set_profiler_enabled(d.queue, 1);
    // A/B only (tools/lazy_queues_ab.sh): idle queues that exist and are never used
    if (const char *xq = getenv("MPIR_CVAR_REDUCE_LOCAL_DIRECT_IDLE_QUEUES")) {
        for (int k = atoi(xq); k > 0 && k <= 8; --k) {
            hsa_queue_t *q = nullptr;
            (void)hsa_queue_create(f.gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q);
        }
    }
    if (!g_ts_freq) hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &g_ts_freq);
    d.karg = static_cast<char *>(kp);
    d.hdp = hdp.HDP_MEM_FLUSH_CNTL;
    if (keepalive_us()) {
        void *na = nullptr;
        if (hsa_amd_memory_pool_allocate(f.vram, 256, 0, &na) == HSA_STATUS_SUCCESS &&
            hsa_amd_agents_allow_access(1, &f.cpu, nullptr, na) == HSA_STATUS_SUCCESS) {
            memset(na, 0, 256);      // LeanArgs {in, io, vbytes = 0, keep}: every workgroup returns at once
            _mm_sfence();
            *d.hdp = 1u;
            (void)*d.hdp;
            d.kargs_noop = static_cast<char *>(na);
        }
    }
    d.ok = true;
    d.state = 1;
}

// Every extra queue is created only when first needed: an idle queue that
// merely exists costs the calls' queue ~1 % at 64 MiB (the CP has one more
// queue to serve; profiles/r02/keepalive_headline_ab.log, lazy_queues_ab.log).
hsa_queue_t *profiled_queue(DevState &d) {
    std::call_once(d.ponce, [&] {
        hsa_queue_t *q = nullptr;
        if (hsa_queue_create(d.agent, kQueueSize, HSA_QUEUE_TYPE_MULTI, queue_error_cb, &d, UINT32_MAX, UINT32_MAX,
                             &q) != HSA_STATUS_SUCCESS)
            return;
        // timestamps on from creation (see timestamps())
        hsa_amd_profiling_set_profiler_enabled(q, 1);
        d.pqueue = q;
    });
    return d.pqueue ? d.pqueue : d.queue;
}

bool keepalive_queue(DevState &d) {
    std::call_once(d.konce, [&] {
        if (!keepalive_own_queue()) {
            d.kqueue = d.queue;
        } else if (hsa_queue_create(d.agent, 64, HSA_QUEUE_TYPE_MULTI, queue_error_cb, &d, UINT32_MAX, UINT32_MAX,
                                    &d.kqueue) != HSA_STATUS_SUCCESS) {
            d.kqueue = nullptr;
        }
        d.kready.store(d.kqueue != nullptr);
    });
    return d.kready.load();
}

// ---- keep-alive thread (keepalive_us()) --------------------------------------
std::atomic<bool> g_keepalive_stop{false};
std::atomic<uint64_t> g_keepalive_packets{0}, g_keepalive_arms{0};
std::once_flag g_keepalive_once;

// one no-op packet on d.kqueue, no completion signal (under d.publish)
void keepalive_packet(DevState &d) {
    hsa_queue_t *q = d.kqueue;
    const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
    if (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) return;   // full: the CP is busy anyway
    const uint64_t ko = d.kobj[0][MPIR_HIP_OP_SUM][MPIR_HIP_F32];
    uint16_t header;
    uint16_t setup = 0;
    if (keepalive_kernel() && ko && d.kargs_noop) {
        hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
        memset((char *)p + 4, 0, sizeof(*p) - 4);
        p->workgroup_size_x = kThreads;
        p->workgroup_size_y = 1;
        p->workgroup_size_z = 1;
        p->grid_size_x = kThreads;
        p->grid_size_y = 1;
        p->grid_size_z = 1;
        p->kernel_object = ko;
        p->kernarg_address = d.kargs_noop;
        header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                 (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                 (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    } else {
        hsa_barrier_and_packet_t *p = (hsa_barrier_and_packet_t *)q->base_address + (idx & (q->size - 1));
        memset((char *)p + 4, 0, sizeof(*p) - 4);
        header = (HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                 (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                 (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    }
    hsa_queue_store_write_index_relaxed(q, idx + 1);
    _mm_sfence();
    __atomic_store_n((uint32_t *)((char *)q->base_address + (idx & (q->size - 1)) * 64),
                     (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, idx);
}

// Keep the thread off the caller's core: pin it to the highest-numbered CPU of
// its affinity mask other than the one the arming call ran on (a napping thread
// free to share the spinning caller's core cost it 2-6 %, ka_isolate.log).
void keepalive_pin(int caller_cpu) {
    if (getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOPIN")) return;   // A/B only
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) != 0) return;
    for (int c = CPU_SETSIZE - 1; c >= 0; --c) {
        if (c == caller_cpu || !CPU_ISSET(c, &set)) continue;
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(c, &one);
        (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
        return;
    }
}

void keepalive_loop(int caller_cpu) {
    keepalive_pin(caller_cpu);
    if (getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_EMPTY")) {   // A/B only: a thread that only naps
        const timespec ms = {0, 1000000};
        while (!g_keepalive_stop.load(std::memory_order_relaxed)) nanosleep(&ms, nullptr);
        return;
    }
    prctl(PR_SET_TIMERSLACK, 1000UL);     // 1 us: nanosleep wakes near the period
    // (no SCHED_IDLE: with it, the napping thread alone cost bench.py's
    // spinning caller 4-21 %, profiles/r02/ka_isolate.log)
    const uint64_t period = (uint64_t)keepalive_us() * 1000ull;
    // naps: half a period while some device idles inside its window (a packet
    // goes out at most 1.5 periods after the last one), a whole period while a
    // call is in flight (the CP is busy; fewer wake-ups for back-to-back
    // callers), 1 ms once every window has expired
    const timespec nap = {0, (long)(period / 2)}, busy_nap = {0, (long)period}, idle_nap = {0, 1000000};
    int state = 1;    // 0 nothing in its window, 1 idle in its window, 2 a call in flight
    while (!g_keepalive_stop.load(std::memory_order_relaxed)) {
        nanosleep(state == 0 ? &idle_nap : state == 2 ? &busy_nap : &nap, nullptr);
        const uint64_t t = mono_ns();
        bool active = false, busy = false;
        for (int i = 0; i < kMaxDirectDev; ++i) {
            DevState &d = g_dev[i];
            if (!d.ok || !d.kready.load(std::memory_order_acquire) || d.queue_error.load(std::memory_order_relaxed))
                continue;
            // (signed: a call may have stamped a time after this thread read the clock)
            const uint64_t lc = d.last_call_ns.load(std::memory_order_relaxed);
            if (!d.armed.load(std::memory_order_relaxed) || !lc || (int64_t)(t - lc) > (int64_t)keepalive_active_ns())
                continue;
            active = true;
            const uint64_t last = d.last_packet_ns.load(std::memory_order_relaxed);
            if (d.call_busy.load(std::memory_order_relaxed)) {
                busy = true;
                continue;
            }
            if ((int64_t)(t - last) < (int64_t)period) continue;
            std::lock_guard<std::mutex> lk(d.publish);
            if (g_keepalive_stop.load(std::memory_order_relaxed)) return;
            // re-check under the lock: a call that published meanwhile is in flight
            if (d.call_busy.load(std::memory_order_relaxed) ||
                (int64_t)(mono_ns() - d.last_packet_ns.load(std::memory_order_relaxed)) < (int64_t)period)
                continue;
            keepalive_packet(d);
            g_keepalive_packets.fetch_add(1, std::memory_order_relaxed);
            d.last_packet_ns.store(mono_ns(), std::memory_order_relaxed);
        }
        state = !active ? 0 : busy ? 2 : 1;
    }
}

// at exit, before the HIP / HSA runtimes tear down (registered after they
// initialised, so it runs first): no packet after this returns
void keepalive_stop() {
    g_keepalive_stop.store(true);
    if (getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_DEBUG"))
        fprintf(stderr, "mpir_hip keep-alive: %llu arms, %llu packets\n",
                (unsigned long long)g_keepalive_arms.load(), (unsigned long long)g_keepalive_packets.load());
    for (int i = 0; i < kMaxDirectDev; ++i) {
        if (!g_dev[i].ok) continue;
        std::lock_guard<std::mutex> lk(g_dev[i].publish);
    }
}

void keepalive_start() {
    if (getenv("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_NOTHREAD")) return;   // A/B only
    std::call_once(g_keepalive_once, [] {
        atexit(keepalive_stop);
        std::thread(keepalive_loop, sched_getcpu()).detach();
    });
}

}  // namespace

// Completion signals, one per (thread, device).  A thread's signals go back
// to a process-wide free list when it exits (no HSA call at thread exit) and
// the next new thread takes them, so threads that come and go reuse a bounded
// set.
std::mutex g_sig_mu;
std::vector<hsa_signal_t> g_sig_free[kMaxDirectDev];

struct DirectSignals {
    hsa_signal_t sig[kMaxDirectDev] = {};
    bool have[kMaxDirectDev] = {};
    bool get(int dev, hsa_signal_t *out) {
        if (!have[dev]) {
            {
                std::lock_guard<std::mutex> lk(g_sig_mu);
                if (!g_sig_free[dev].empty()) {
                    sig[dev] = g_sig_free[dev].back();
                    g_sig_free[dev].pop_back();
                    have[dev] = true;
                }
            }
            if (!have[dev]) {
                // The host polls the signal and never sleeps on it, so it needs no
                // interrupt event: naming the GPU as its only consumer makes ROCr
                // create a plain memory signal (MPIR_CVAR_REDUCE_LOCAL_DIRECT_SIGNAL
                // =interrupt keeps the default, event-backed kind)
                hsa_status_t st;
                if (signal_kind() == 0) st = hsa_signal_create(0, 1, &g_dev[dev].agent, &sig[dev]);
                else st = hsa_signal_create(0, 0, nullptr, &sig[dev]);
                if (st != HSA_STATUS_SUCCESS) return false;
                have[dev] = true;
            }
        }
        *out = sig[dev];
        return true;
    }
    ~DirectSignals() {
        std::lock_guard<std::mutex> lk(g_sig_mu);
        for (int i = 0; i < kMaxDirectDev; ++i)
            if (have[i]) g_sig_free[i].push_back(sig[i]);
    }
};
thread_local DirectSignals t_sig;

// 1: dispatched and completed (rc set); 0: not applicable, use the HIP path.
// `p` is plan_reduce's launch plan of the call (padding bytes zero).
int direct_reduce(int dev, int op, int elem, const ReducePlan &p, int *rc) {
    if (mode() == 0 || dev < 0 || dev >= kMaxDirectDev || op <= 0 || op >= MPIR_HIP_NOPS || elem <= 0 ||
        elem >= MPIR_HIP_NELEMS || p.kind < 0 || p.kind >= kPlanKinds || p.arg_bytes != kPlanArgBytes[p.kind])
        return 0;
    const bool prof = g_profile.load(std::memory_order_relaxed) != 0;
    const uint64_t th0 = prof ? sys_ts() : 0;
    uint64_t th1 = 0;
    DevState &d = g_dev[dev];
    std::call_once(d.once, [&] { init_dev(dev, d); });
    if (!d.ok || d.queue_error.load(std::memory_order_relaxed)) return 0;
    if (keepalive_us()) {
        // arm on a call after a gap, disarm on a back-to-back one
        const uint64_t lc = d.last_call_ns.load(std::memory_order_relaxed);
        if (lc) {
            const int64_t gap = (int64_t)(mono_ns() - lc);
            const int64_t p = (int64_t)keepalive_us() * 1000;
            if (gap > p + 10000) {
                if (!d.armed.load(std::memory_order_relaxed) && keepalive_queue(d)) {
                    d.armed.store(1, std::memory_order_relaxed);
                    g_keepalive_arms.fetch_add(1, std::memory_order_relaxed);
                    keepalive_start();
                }
            } else if (gap < p && d.armed.load(std::memory_order_relaxed)) {
                d.armed.store(0, std::memory_order_relaxed);
            }
        }
    }
    const uint64_t ko = d.kobj[p.kind][op][elem];
    // the packet's grid_size_x (workgroups x kThreads) is 32 bits
    if (!ko || p.groups == 0 || p.groups > (uint64_t)UINT32_MAX / kThreads) return 0;
    // Work queued on the legacy null stream stays ordered before us, as it is
    // for the HIP path's blocking library stream.  hipStreamQuery(nullptr)
    // keeps answering "not ready" after such work has finished until the host
    // synchronises with it (measured: tools/direct_probe.py), so a busy answer
    // is followed by that synchronisation -- the wait the synchronous call
    // would spend behind the same work on the HIP path anyway.
    if (hipStreamQuery(nullptr) != hipSuccess) {
        (void)hipGetLastError();
        g_busy_skips.fetch_add(1, std::memory_order_relaxed);
        if (hipStreamSynchronize(nullptr) != hipSuccess) {
            (void)hipGetLastError();
            return 0;
        }
    }
    hsa_signal_t sig;
    if (!t_sig.get(dev, &sig)) return 0;
    const uint32_t groups = (uint32_t)p.groups;
    const unsigned char *ka = p.args;
    const uint32_t kn = p.arg_bytes;
    hsa_signal_store_relaxed(sig, 1);
    CacheEntry *held = nullptr;
    int ring = -1;
    {
        std::lock_guard<std::mutex> lk(d.publish);
        uint64_t h = ko;
        for (uint32_t w = 0; w < kn / 8; ++w) {
            uint64_t x;
            memcpy(&x, ka + 8 * w, 8);
            h = (h ^ x) * 0x9E3779B97F4A7C15ull;
        }
        h ^= h >> 29;
        const uint32_t ci = (uint32_t)(h % kCacheSlots);
        CacheEntry &e = d.cache[ci];
        char *slot;
        const bool hit = e.ko == ko && e.n == kn && !memcmp(e.args, ka, kn);
        if (hit || e.inflight.load(std::memory_order_acquire) == 0) {
            slot = d.karg + (size_t)(kRingSlots + ci) * kKargSlotBytes;
            e.inflight.fetch_add(1, std::memory_order_acq_rel);
            held = &e;
            if (!hit) {
                e.ko = ko;
                e.n = kn;
                memcpy(e.args, ka, kn);
            }
        } else {
            // a ring slot no in-flight dispatch reads (workgroups load their
            // kernargs when they start, i.e. all through a long kernel's life)
            for (uint32_t k = 0; k < kRingSlots; ++k) {
                const uint32_t r = (d.kslot + k) % kRingSlots;
                if (d.ring_busy[r].load(std::memory_order_acquire) == 0) {
                    ring = (int)r;
                    break;
                }
            }
            if (ring < 0) return 0;     // every ring slot in flight: the HIP path takes this call
            d.kslot = (uint32_t)ring + 1;
            d.ring_busy[ring].store(1, std::memory_order_relaxed);
            slot = d.karg + (size_t)ring * kKargSlotBytes;
        }
        if (!hit) {
            memcpy(slot, ka, kn);
            _mm_sfence();
            *d.hdp = 1u;        // HDP flush: the BAR writes land in VRAM before the CP reads them
            (void)*d.hdp;
        }
        hsa_queue_t *q = prof ? profiled_queue(d) : d.queue;
        const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) _mm_pause();
        hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
        memset((char *)p + 4, 0, sizeof(*p) - 4);
        p->workgroup_size_x = kThreads;
        p->workgroup_size_y = 1;
        p->workgroup_size_z = 1;
        p->grid_size_x = groups * kThreads;
        p->grid_size_y = 1;
        p->grid_size_z = 1;
        p->kernel_object = ko;
        p->kernarg_address = slot;
        p->completion_signal = sig;
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (acquire_scope() << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (release_scope() << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        hsa_queue_store_write_index_relaxed(q, idx + 1);
        // the ring may be write-combined VRAM (HSA_ALLOCATE_QUEUE_DEV_MEM): the
        // packet body must be out of the WC buffers before its header is valid
        _mm_sfence();
        __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        if (prof) th1 = sys_ts();
        hsa_signal_store_screlease(q->doorbell_signal, idx);
        if (keepalive_us()) d.call_busy.store(1, std::memory_order_relaxed);
    }
    if (use_mwaitx() && !d.queue_error.load(std::memory_order_relaxed)) wait_signal_mwaitx(sig);
    for (uint64_t it = 1; hsa_signal_load_scacquire(sig) != 0; ++it) {
        if ((it & 0xFFFF) == 0 && d.queue_error.load(std::memory_order_relaxed)) {
            *rc = MPIR_HIP_ERUNTIME;
            return 1;       // (the entry stays held: a faulted queue is not used again)
        }
        _mm_pause();
    }
    if (held) held->inflight.fetch_sub(1, std::memory_order_acq_rel);
    if (ring >= 0) d.ring_busy[ring].store(0, std::memory_order_release);
    if (keepalive_us()) {
        // (with several threads calling, one's end may clear another's busy
        // flag: at worst a keep-alive packet goes out during a call, harmless)
        const uint64_t t = mono_ns();
        d.last_packet_ns.store(t, std::memory_order_relaxed);
        d.last_call_ns.store(t, std::memory_order_relaxed);
        d.call_busy.store(0, std::memory_order_relaxed);
    }
    if (prof) {
        const uint64_t th2 = sys_ts();
        hsa_amd_profiling_dispatch_time_t t{};
        const bool okt = hsa_amd_profiling_get_dispatch_time(d.agent, sig, &t) == HSA_STATUS_SUCCESS && g_ts_freq;
        const double ns = okt ? 1e9 / (double)g_ts_freq : 0.0;
        t_last_kernel_ns = okt ? (uint64_t)((double)(t.end - t.start) * ns) : 0;
        // the dispatch times are in the system domain, like HSA_SYSTEM_INFO_TIMESTAMP
        t_last_split[0] = (uint64_t)((double)(th1 - th0) * ns);
        t_last_split[1] = okt ? (uint64_t)((double)((int64_t)(t.start - th0)) * ns) : 0;
        t_last_split[2] = okt ? (uint64_t)((double)((int64_t)(t.end - th0)) * ns) : 0;
        t_last_split[3] = (uint64_t)((double)(th2 - th0) * ns);
    }
    g_direct_calls.fetch_add(1, std::memory_order_relaxed);
    *rc = MPIR_HIP_OK;
    return 1;
}

uint64_t direct_calls() { return g_direct_calls.load(std::memory_order_relaxed); }

void direct_profile(int on) { g_profile.store(on ? 1 : 0); }

uint64_t direct_last_kernel_ns() { return t_last_kernel_ns; }

void direct_last_split(uint64_t out[4]) {
    for (int i = 0; i < 4; ++i) out[i] = t_last_split[i];
}

int direct_state(int dev) {
    if (mode() == 0) return -20;
    if (dev < 0 || dev >= kMaxDirectDev) return -21;
    return g_dev[dev].state;
}

uint64_t direct_busy_skips() { return g_busy_skips.load(std::memory_order_relaxed); }

}  // namespace mpir_hip
