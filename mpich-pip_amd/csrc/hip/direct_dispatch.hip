// direct_dispatch.hip -- synchronous device-resident MPI_Reduce_local without
// the HIP launch path: our own AQL queue, the tile kernel from a device-only
// code object (direct_tiles.hip -> lib/libmpir_hip_tiles.hsaco), kernargs in
// VRAM, and a wait on the dispatch packet's own completion signal.
//
// Why (tools/aql/aql2.cpp, profiles/archive/r02/aql2_*.log): a synchronous HIP call
// is hipLaunchKernel + a completion word written by hipStreamWriteValue32,
// which is a second (blit) dispatch; the GPU then sits idle 8.8-8.9 us between
// one call's last workgroup and the next call's first.  A direct dispatch
// waits on the kernel packet's completion signal instead: 7.4-7.5 us, and the
// 256 MiB fp32 SUM call 126.2-126.4 us against 127.6-127.8 (same box, same
// kernel); with the kernarg cache below and the AQL rings in VRAM
// (HSA_ALLOCATE_QUEUE_DEV_MEM=1, the library's default: default_rings_in_vram)
// the gap is 5.2-5.5 us, 4.3 us of it the CP
// noticing the doorbell (profiles/archive/r02/sync_split_timeline.log,
// cp_latency.log).  An earlier attempt (round 1) lost because its kernargs sat
// in host memory (every workgroup read them over PCIe); here they sit in VRAM:
// a call that repeats its arguments dispatches a cached slot as it stands, and
// any other call writes its slot through the BAR before ringing the doorbell,
// with an HDP flush (the register ROCr exposes as HSA_AMD_AGENT_INFO_HDP_FLUSH)
// that is not read back, for a checked kernel that verifies the slot's nonce
// (kRingSlots below).
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
//     work until the host synchronises, tools/archive/direct_probe.py), the call first
//     synchronises with the null stream;
//   * the calling thread has no unfinished work on its own library stream.
// Packets carry an agent-scope acquire (what HIP uses between kernels; a
// system-scope acquire costs ~7 us of body, aql_sig_nt_sys) and a
// system-scope release, so the result is visible to every agent -- SDMA
// copies and the host included -- when the signal fires.  One queue per
// device (plus its timestamped twin for profiled calls), shared by the
// threads; a mutex orders packet publication (single producer at a time,
// doorbell monotonic); each thread waits on its own signal.  The CP runs a
// queue's dispatches one after another whatever the barrier bit
// (tools/aql/concurrent_probe.cpp, profiles/archive/r03/concurrent_probe.log), so
// concurrent callers on one device take turns, as they would for the HBM.
// MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip turns the path off.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/amd_hsa_signal.h>
#include <ctype.h>
#include <dirent.h>
#include <dlfcn.h>
#include <immintrin.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "mpir_hip_reduce.h"
#include "kernel_table.hpp"

namespace mpir_hip {

namespace {

#ifndef MPIR_TILES_HASH
#define MPIR_TILES_HASH "unknown"   // (the Makefile passes the code object's source hash)
#endif

constexpr int kMaxDirectDev = 64;
constexpr uint32_t kKargSlotBytes = sizeof(KargSlot);
static_assert(kKargSlotBytes == 128, "one kernarg slot per 128-byte L2 line");
// Kernarg slots, by region: [0, kRingSlots) a ring for one-off arguments;
// [kRingSlots, +kCacheSlots) a direct-mapped cache: a call whose (kernel,
// arguments) match a cached slot that a checked dispatch has read back
// complete dispatches the unchecked kernel with that slot as it stands, no
// host write at all; [kProfBase, +kRingSlots) the ring of the
// timestamped twin queue, whose dispatch ids count separately (a slot is only
// ever stamped by one queue's packets).  A reduction schedule that calls
// again on the same buffers, or a caller rotating a few buffer pairs, hits.  A
// cached slot's arguments are rewritten only when no dispatch that uses it
// is in flight.
//
// Every other call dispatches the checked kernel and writes its slot through
// the BAR before ringing the doorbell (KargSlot's layout, reduce_kernels.hpp):
// the argument words that change, an sfence, each half's nonce (the packet's
// queue index + 1), an sfence, then an HDP flush that is not read back.  Round
// 2 read the flush register back (1.7 us from entry to doorbell on a miss
// against 0.35 us on a hit, profiles/archive/r03/fresh_args_split_before_grid.log);
// without the read-back a miss runs 0.5-0.8 us behind a hit
// (tools/aql/kslot_ab.cpp, profiles/archive/r03/kslot_ab*.log).  Correctness does not
// rest on the timing: the checked kernels (direct_tiles.hip checked_args)
// re-read a slot whose halves carry a nonce older than their dispatch id + 1,
// so a workgroup never combines with stale arguments.  (Writing after the
// doorbell saves another 0.3-0.6 us but loses badly when the write is late:
// see direct_reduce.)
constexpr uint32_t kRingSlots = 128, kCacheSlots = 128, kProfBase = kRingSlots + kCacheSlots;
constexpr uint32_t kKargSlots = kProfBase + kRingSlots;
constexpr uint32_t kQueueSize = 256;

// Why a verified slot may be dispatched unchecked on any XCD.  The MI355X's 8
// XCDs each have their own L2, not coherent with the others
// (MI355X_MICROARCH.md), and the slot sits in coarse-grained VRAM, which an L2
// may cache.  A host write (BAR + HDP flush) updates HBM, not a line an XCD's
// L2 may still hold from an earlier dispatch through the slot.  The packet's
// agent-scope acquire is HIP's own kernel-to-kernel fence, but the ISA guide
// and the headers available here do not state that the command processor's
// acquire invalidates that line in every XCD's L2, so the library does not rely
// on it: a checked dispatch verifies the slot on every XCD before it counts as
// verified.  Workgroups are handed to the XCDs round-robin, so a grid of at
// least 8 reaches all of them; a checked dispatch of a smaller plan is padded
// to 8 workgroups (the extra ones read and check the slot -- re-reading past the
// caches if their XCD's line is stale -- and exit, direct_tiles.hip in_grid).
// After it, every XCD's L2 holds the fresh line or none, and the slot is only
// rewritten after its entry leaves the cache.  Cost: the seven padding
// workgroups of a one-workgroup miss (measured in DESIGN.md §Synchronous
// return); hits pay nothing.
#ifndef MPIR_DIRECT_MIN_CHECKED_GROUPS
#define MPIR_DIRECT_MIN_CHECKED_GROUPS 8    // (a build-time override for tools/small_miss_ab.sh only)
#endif
constexpr uint32_t kMinCheckedGroups = MPIR_DIRECT_MIN_CHECKED_GROUPS;

// a plan's argument bytes (LeanArgs / TileArgs / ShiftArgs / ElemsArgs,
// reduce_kernels.hpp; their layouts do not depend on the element type)
constexpr uint32_t kMaxArgBytes = sizeof(ReducePlan::args);
static_assert(kMaxArgBytes <= kSlotArgBytes, "kernarg slot too small");
constexpr uint32_t kPlanArgBytes[kPlanKinds] = {sizeof(LeanArgs), sizeof(TileArgs<char>), sizeof(ShiftArgs<char>),
                                                sizeof(ElemsArgs), sizeof(ElemsArgs)};
// per plan kind, the unchecked and the checked kernel (direct_tiles.hip)
const char *const kPlanPrefix[2][kPlanKinds] = {
    {"mpir_tile_", "mpir_tilex_", "mpir_tiles_", "mpir_elems_", "mpir_elemsu_"},
    {"mpir_ctile_", "mpir_ctilex_", "mpir_ctiles_", "mpir_celems_", "mpir_celemsu_"}};

struct CacheEntry {
    uint64_t ko = 0;                            // the unchecked kernel of the plan
    uint32_t n = 0;                             // argument bytes
    alignas(8) unsigned char args[kMaxArgBytes] = {};
    std::atomic<int> inflight{0};
    std::atomic<int> verified{0};               // a checked dispatch read this write complete
};

struct DevState {
    std::once_flag once;
    bool ok = false;
    std::atomic<int> state{0};  // 0 not tried, 1 ready, 2 ready with flushes read back (readback),
                            // < 0 the init step that failed (MPIR_Hip_direct_state)
    hsa_agent_t agent{};
    hsa_queue_t *queue = nullptr;               // the calls' queue (no dispatch timestamps)
    hsa_queue_t *pqueue = nullptr;              // the same, timestamps on: calls while profiling is on
    std::once_flag ponce;                       // (created at the first profiled call)
    char *karg = nullptr;                       // kKargSlots x kKargSlotBytes, VRAM, host-written
    volatile uint32_t *err = nullptr;           // host memory: a kernel found its arguments missing
    uint32_t kslot = 0, pslot = 0;              // next ring / profiled-ring slot to try (under `publish`)
    std::atomic<int> ring_busy[2 * kRingSlots] = {};  // a (profiled) ring slot's dispatch is in flight
    CacheEntry cache[kCacheSlots];
    volatile uint32_t *hdp = nullptr;
    uint64_t kobj[2][kPlanKinds][MPIR_HIP_NOPS][MPIR_HIP_NELEMS] = {};   // [checked][plan kind] (kPlanPrefix)
    uint64_t kprobe = 0;                        // mpir_probe_dispatch_id
    // a queue's dispatch ids are not its packet indices (an intercepting tool,
    // probe_ids): every written slot is made visible by a flush read back
    // before the doorbell, and only unchecked kernels run
    std::atomic<bool> readback{false};
    std::mutex publish;
    std::atomic<int> queue_error{0};
};

DevState g_dev[kMaxDirectDev];
std::atomic<uint64_t> g_direct_calls{0};
std::atomic<uint64_t> g_busy_skips{0};      // calls that first synchronised with a busy null stream
std::atomic<uint32_t> g_test_write_delay_us{0};   // MPIR_Hip_direct_test_write_delay_us (tests only)
std::atomic<bool> g_test_fail_probe{false};       // MPIR_Hip_direct_test_fail_probe (tests only)
std::atomic<uint64_t> g_kernarg_writes{0};  // kernarg-cache misses (BAR write + HDP flush)
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

int mode() {
    static const int m = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_DISPATCH");
        return (e && !strcmp(e, "hip")) ? 0 : 1;
    }();
    return m;
}

// The calls' queue records no dispatch timestamps: with them the CP's
// per-packet timestamp writes cost the synchronous call ~0.4 us at 256 MiB and
// ~0.9 us at 64 MiB (alternated processes, tools/archive/ts_ab.sh, profiles/archive/r02/ts_ab.log),
// and switching them on for a live queue does not take effect
// (tools/archive/ts_enable_probe.py).  A second queue, created with them on, takes the
// calls made while MPIR_Hip_direct_profile is on (the bench's roofline readout:
// the same kernel object, plan and arguments).
//
// Packet fences: agent-scope acquire (what HIP uses between kernels; a
// system-scope acquire costs ~7 us of kernel body, aql_sig_nt_sys) and
// system-scope release, so the result is visible to every agent -- SDMA copies
// and the host included -- when the signal fires.  Other scopes measured within
// 0.2 us (tools/archive/scope_ab.sh, profiles/archive/r02/scope_ab.log); none at release would
// leave results in one XCD's L2 and is not offered.
constexpr int kAcquireScope = HSA_FENCE_SCOPE_AGENT;
constexpr int kReleaseScope = HSA_FENCE_SCOPE_SYSTEM;

// HIP's device -> its HSA agent.  The device's UUID (hipDeviceProp_t::uuid,
// the 16 characters after "GPU-" of HSA_AMD_AGENT_INFO_UUID) identifies it when
// it matches exactly one agent; otherwise its PCI domain and bus / device
// numbers must match exactly one agent.  Compute-partitioned GPUs expose
// several agents with one bus / device number (the function bits, which HIP's
// properties do not carry, tell them apart): with no unique match the direct
// path is refused (MPIR_Hip_direct_state -3) rather than guessed.
struct Find {
    uint32_t bdf, domain;
    char uuid[16];
    bool have_uuid = false;
    hsa_agent_t bdf_gpu{}, uuid_gpu{}, cpu{};
    int bdf_matches = 0, uuid_matches = 0;
    bool have_cpu = false;
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
        char uuid[24] = {};
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if ((bdf & ~7u) == f->bdf && dom == f->domain) {
            f->bdf_gpu = a;
            ++f->bdf_matches;
        }
        if (f->have_uuid && hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_UUID, uuid) == HSA_STATUS_SUCCESS &&
            !strncmp(uuid, "GPU-", 4) && !memcmp(uuid + 4, f->uuid, sizeof f->uuid)) {
            f->uuid_gpu = a;
            ++f->uuid_matches;
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

// Write a kernel dispatch packet at `idx` (already reserved: the write index
// is stored here) and ring the doorbell.
void publish_packet(hsa_queue_t *q, uint64_t idx, uint64_t ko, void *slot, hsa_signal_t sig, uint32_t wg,
                    uint32_t groups) {
    hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    p->workgroup_size_x = (uint16_t)wg;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->grid_size_x = groups * wg;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->kernel_object = ko;
    p->kernarg_address = slot;
    p->completion_signal = sig;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (kAcquireScope << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (kReleaseScope << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    hsa_queue_store_write_index_relaxed(q, idx + 1);
    // the ring may be write-combined VRAM (HSA_ALLOCATE_QUEUE_DEV_MEM): the
    // packet body must be out of the WC buffers before its header is valid
    _mm_sfence();
    __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
}

// Whether queue `q` hands its kernels their packet's index as the dispatch id
// (the checked kernels' nonce, direct_tiles.hip): two probe dispatches through
// kernarg slot `slot`, each storing the id it was given.  A tool that
// intercepts the queue (rocprofv3 --kernel-trace measured: the ids run ahead
// of the indices) makes them differ; so does a queue the probe cannot run on.
bool probe_ids(DevState &d, hsa_queue_t *q, char *slot) {
    if (!d.kprobe) return false;
    hsa_signal_t s;
    if (hsa_signal_create(1, 0, nullptr, &s) != HSA_STATUS_SUCCESS) return false;
    volatile uint64_t *out = reinterpret_cast<volatile uint64_t *>((volatile char *)d.err + 16);
    bool match = true, done = true;
    for (int i = 0; i < 2 && match && done; ++i) {
        KargSlot ks{};
        ks.w[0] = (uint64_t)(uintptr_t)out;
        ks.w[6] = (uint64_t)(uintptr_t)d.err;
        memcpy(slot, &ks, sizeof ks);
        _mm_sfence();
        *d.hdp = 1u;
        (void)*d.hdp;
        *out = ~0ull;
        hsa_signal_store_relaxed(s, 1);
        const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) _mm_pause();
        publish_packet(q, idx, d.kprobe, slot, s, 64, 1);
        hsa_signal_store_screlease(q->doorbell_signal, idx);
        // 2 s: a probe that has not finished by then leaves its signal alive
        done = hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_EQ, 0, 2 * g_ts_freq, HSA_WAIT_STATE_ACTIVE) == 0;
        match = done && *out == idx;
    }
    if (done) hsa_signal_destroy(s);
    return match;
}

void init_dev(int dev, DevState &d) {
    d.state = -1;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) { (void)hipGetLastError(); return; }
    Find f;
    f.bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    f.domain = (uint32_t)prop.pciDomainID;
    memcpy(f.uuid, prop.uuid.bytes, sizeof f.uuid);
    for (char c : f.uuid) f.have_uuid |= c != 0;
    d.state = -2;
    if (hsa_init() != HSA_STATUS_SUCCESS) return;
    hsa_iterate_agents(find_agent, &f);
    d.state = -3;
    if (!f.have_cpu || (f.uuid_matches != 1 && f.bdf_matches != 1)) return;
    const hsa_agent_t gpu = f.uuid_matches == 1 ? f.uuid_gpu : f.bdf_gpu;
    hsa_amd_agent_iterate_memory_pools(gpu, find_vram, &f);
    d.state = -4;
    if (!f.have_vram) return;
    d.state = -5;
    hsa_amd_hdp_flush_t hdp{};
    if (hsa_agent_get_info(gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp) != HSA_STATUS_SUCCESS ||
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
    // built from the sources this library was built from (Makefile TILES_HASH,
    // direct_tiles.hip mpir_tiles_build_id): else the HIP path takes every call
    d.state = -12;
    {
        static const char tag[] = "mpir-tiles-build:" MPIR_TILES_HASH;
        const std::string bytes(co.begin(), co.end());
        if (bytes.find(tag) == std::string::npos) {
            fprintf(stderr, "mpir_hip: %s was not built from this library's sources (want %s); direct dispatch off\n",
                    path.c_str(), tag);
            return;
        }
    }
    d.state = -7;
    hsa_code_object_reader_t rd;
    hsa_executable_t exe;
    if (hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd) != HSA_STATUS_SUCCESS) return;
    if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_load_agent_code_object(exe, gpu, rd, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        hsa_executable_freeze(exe, nullptr) != HSA_STATUS_SUCCESS)
        return;     // (the reader and executable live as long as the process)
    d.state = -8;
    int found = 0;
    for (int op = 1; op < MPIR_HIP_NOPS; ++op) {
        for (int e = 1; e < MPIR_HIP_NELEMS; ++e) {
            if (!op_name(op) || !elem_name(e)) continue;
            // every plan kind, unchecked and checked, each taking one kernarg slot
            for (int kc = 0; kc < 2 * kPlanKinds; ++kc) {
                const int chk = kc / kPlanKinds, kind = kc % kPlanKinds;
                const std::string sym = std::string(kPlanPrefix[chk][kind]) + op_name(op) + "_" + elem_name(e) + ".kd";
                hsa_executable_symbol_t s;
                uint64_t ko = 0;
                uint32_t kas = 0, lds = 1, priv = 1;
                if (hsa_executable_get_symbol_by_name(exe, sym.c_str(), &gpu, &s) != HSA_STATUS_SUCCESS) continue;
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
                    kas != kKargSlotBytes || lds != 0 || priv != 0)
                    continue;
                d.kobj[chk][kind][op][e] = ko;
                ++found;
            }
        }
    }
    if (!found) return;
    {
        hsa_executable_symbol_t s;
        uint32_t kas = 0, lds = 1, priv = 1;
        if (hsa_executable_get_symbol_by_name(exe, "mpir_probe_dispatch_id.kd", &gpu, &s) == HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &d.kprobe) == HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kas) ==
                HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &lds) ==
                HSA_STATUS_SUCCESS &&
            hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv) ==
                HSA_STATUS_SUCCESS &&
            (kas != kKargSlotBytes || lds != 0 || priv != 0))
            d.kprobe = 0;
    }
    // kernargs in VRAM, host-writable
    d.state = -9;
    void *kp = nullptr;
    if (hsa_amd_memory_pool_allocate(f.vram, (size_t)kKargSlots * kKargSlotBytes, 0, &kp) != HSA_STATUS_SUCCESS) return;
    if (hsa_amd_agents_allow_access(1, &f.cpu, nullptr, kp) != HSA_STATUS_SUCCESS) {
        hsa_amd_memory_pool_free(kp);
        return;
    }
    d.state = -10;
    if (hsa_queue_create(gpu, kQueueSize, HSA_QUEUE_TYPE_MULTI, queue_error_cb, &d, UINT32_MAX, UINT32_MAX,
                         &d.queue) != HSA_STATUS_SUCCESS) {
        hsa_amd_memory_pool_free(kp);
        return;
    }
    d.agent = gpu;
    if (!g_ts_freq) hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &g_ts_freq);
    // the kernels' error word: fine-grained host memory the GPU can write
    d.state = -11;
    void *ew = nullptr;
    if (hipHostMalloc(&ew, 64, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        hsa_queue_destroy(d.queue);
        d.queue = nullptr;
        hsa_amd_memory_pool_free(kp);
        return;
    }
    d.err = static_cast<volatile uint32_t *>(ew);
    *d.err = 0;
    d.karg = static_cast<char *>(kp);
    d.hdp = hdp.HDP_MEM_FLUSH_CNTL;
    // the nonce protocol, or flushes read back when the queue's dispatch ids
    // are not its indices (probe_ids; ring slot 0, rewritten below)
    if (!probe_ids(d, d.queue, d.karg)) d.readback.store(true);
    // Every slot starts with the error word's address (the same in every later
    // write, so never stale) and nonce 0, below every dispatch id + 1; this
    // once, the flush is read back.
    {
        KargSlot init{};
        init.w[6] = (uint64_t)(uintptr_t)ew;
        for (uint32_t k = 0; k < kKargSlots; ++k) memcpy(d.karg + (size_t)k * kKargSlotBytes, &init, sizeof init);
        _mm_sfence();
        *d.hdp = 1u;
        (void)*d.hdp;
    }
    d.ok = true;
    d.state = d.readback.load() ? 2 : 1;
}

// The profiled queue is created only when first needed: an idle queue that
// merely exists costs the calls' queue ~1 % at 64 MiB (the CP has one more
// queue to serve; profiles/archive/r02/keepalive_headline_ab.log, lazy_queues_ab.log).
hsa_queue_t *profiled_queue(DevState &d) {
    std::call_once(d.ponce, [&] {
        hsa_queue_t *q = nullptr;
        if (hsa_queue_create(d.agent, kQueueSize, HSA_QUEUE_TYPE_MULTI, queue_error_cb, &d, UINT32_MAX, UINT32_MAX,
                             &q) != HSA_STATUS_SUCCESS)
            return;
        // timestamps on from creation (see kAcquireScope's comment above)
        hsa_amd_profiling_set_profiler_enabled(q, 1);
        // (its ring's first slot: no profiled dispatch exists yet)
        if (g_test_fail_probe.exchange(false) || !probe_ids(d, q, d.karg + (size_t)kProfBase * kKargSlotBytes)) {
            d.readback.store(true);
            d.state = 2;        // MPIR_Hip_direct_state: flushes read back from now on
        }
        d.pqueue = q;
    });
    return d.pqueue ? d.pqueue : d.queue;
}

// AQL rings in VRAM by default.  ROCm places every queue's ring in host memory
// unless HSA_ALLOCATE_QUEUE_DEV_MEM=1; with the ring in VRAM the CP fetches each
// dispatch packet locally, 1.4 us off every synchronous call
// (profiles/archive/r02/sync_ab_ring.log), and HIP's own queues gain the same.  The HSA
// runtime reads the variable once, when it starts, and hsa_queue_create takes no
// per-queue choice in this ROCm; so the library sets the default when it is
// loaded -- before main() for a program linked against it (libmpi in Option 1),
// before the first HIP call for one that loads it first -- and leaves any value
// the environment already holds (HSA_ALLOCATE_QUEUE_DEV_MEM=0 keeps ROCm's
// placement).  The other HSA clients of the process gain too: alternated fresh
// processes without this library (tools/ring_placement_ab.py,
// profiles/r04/ring_placement_ab.log) give a HIP launch + synchronize of 14.0
// against 16.9 us, and a one-rank RCCL all_reduce 16.7 against 18.7 us at 8 B
// and 16.0 against 14.3 TB/s at 256 MiB, with the rings in VRAM.
// It is set only while it can still act and be set safely: not once the HSA
// runtime has started (ROCr read it then), and not once the process has a
// second thread (setenv may move the environment array under another
// thread's getenv; glibc does not lock getenv).  A program linked against the
// library loads it before main(), single-threaded; one that dlopens it later
// into a threaded process keeps ROCm's placement unless the job sets the
// variable (mpiexec does).
int process_threads() {
    FILE *f = fopen("/proc/self/status", "r");
    if (!f) return -1;
    char line[256];
    int n = -1;
    while (fgets(line, sizeof line, f))
        if (!strncmp(line, "Threads:", 8)) {
            n = atoi(line + 8);
            break;
        }
    fclose(f);
    return n;
}

// 1 set now, 0 the environment holds a value, -1 the HSA runtime has started,
// -2 the process runs other threads and `threads_ok` is 0.
int rings_default(int threads_ok) {
    if (getenv("HSA_ALLOCATE_QUEUE_DEV_MEM")) return 0;
    uint16_t major = 0;
    if (hsa_system_get_info(HSA_SYSTEM_INFO_VERSION_MAJOR, &major) == HSA_STATUS_SUCCESS) return -1;
    if (!threads_ok && process_threads() != 1) return -2;
    setenv("HSA_ALLOCATE_QUEUE_DEV_MEM", "1", 0);
    return 1;
}

__attribute__((constructor)) void default_rings_in_vram() { (void)rings_default(0); }

}  // namespace

// The same default, asked for by a caller that knows its other threads leave
// the environment alone -- the Python package's load(): an interpreter that
// imported numpy or torch first already runs their (parked) pool threads, so
// the constructor above stood aside, and without this its queues keep ROCm's
// host-memory rings, ~0.7 us on every synchronous call (tools/aql/cp_floor.sh,
// profiles/r06/cp_floor_r06j.log).
extern "C" int MPIR_Hip_default_rings_in_vram(int threads_ok) { return rings_default(threads_ok); }

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
                // create a plain memory signal (an event-backed one measured the
                // same, profiles/archive/r02/sync_ab_ring.log)
                if (hsa_signal_create(0, 1, &g_dev[dev].agent, &sig[dev]) != HSA_STATUS_SUCCESS) return false;
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

namespace {
// A/B knob (tools/placement_ab.py; default off): MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE=n
// makes the completion signals of unprofiled direct calls amd_signal_t blocks
// (amd_hsa_signal.h: the layout the CP decrements) that the library allocates
// from the fine-grained pool of the n-th CPU agent (NUMA node n) and makes
// accessible to the GPU, instead of the HSA runtime's own signals, so where the
// signal lives can be chosen and measured.  No event mailbox: the caller polls.
int signal_node_knob() {
    static const int n = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_SIGNAL_NODE");
        return e && *e ? atoi(e) : -1;
    }();
    return n;
}
struct PoolFind {
    int want, seen = 0;
    hsa_agent_t cpu{};
    bool found = false;
    hsa_amd_memory_pool_t pool{};
    bool have_pool = false;
};
hsa_status_t find_nth_cpu(hsa_agent_t a, void *p) {
    PoolFind *f = static_cast<PoolFind *>(p);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
        if (f->seen++ == f->want) {
            f->cpu = a;
            f->found = true;
            return HSA_STATUS_INFO_BREAK;
        }
    }
    return HSA_STATUS_SUCCESS;
}
hsa_status_t find_fine_pool(hsa_amd_memory_pool_t p, void *arg) {
    PoolFind *f = static_cast<PoolFind *>(arg);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    bool alloc = false;
    if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && alloc) {
        f->pool = p;
        f->have_pool = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}
// this thread's placed signal for device dev (nullptr: not available)
thread_local amd_signal_t *t_placed_sig[kMaxDirectDev] = {};
thread_local bool t_placed_failed[kMaxDirectDev] = {};
amd_signal_t *placed_signal(int dev) {
    if (t_placed_sig[dev] || t_placed_failed[dev]) return t_placed_sig[dev];
    t_placed_failed[dev] = true;    // until the allocation below succeeds: tried once per thread
    PoolFind f;
    f.want = signal_node_knob();
    hsa_iterate_agents(find_nth_cpu, &f);
    if (!f.found) return nullptr;
    hsa_amd_agent_iterate_memory_pools(f.cpu, find_fine_pool, &f);
    if (!f.have_pool) return nullptr;
    void *mem = nullptr;
    if (hsa_amd_memory_pool_allocate(f.pool, 4096, 0, &mem) != HSA_STATUS_SUCCESS) return nullptr;
    if (hsa_amd_agents_allow_access(1, &g_dev[dev].agent, nullptr, mem) != HSA_STATUS_SUCCESS) {
        hsa_amd_memory_pool_free(mem);
        return nullptr;
    }
    amd_signal_t *sg = static_cast<amd_signal_t *>(mem);
    memset(sg, 0, sizeof *sg);
    sg->kind = AMD_SIGNAL_KIND_USER;
    sg->value = 0;
    t_placed_sig[dev] = sg;     // (kept for the thread's life: 4 KiB per thread and device, test knob only)
    t_placed_failed[dev] = false;
    return sg;
}
}  // namespace

// ---- placement: where the synchronous call's host side runs relative to the
// device.  The call's host-memory traffic is the doorbell write (MMIO to the
// device's BAR), the completion signal the CP writes and the host polls, and
// the error word read once per call; everything else (AQL ring, kernargs) sits
// in VRAM.
namespace {
// NUMA node of the page holding p (-1 if unknown): move_pages without target
// nodes only reports where each page lives
int page_node(const void *p) {
    void *pg = reinterpret_cast<void *>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)4095);
    int status = -1;
    if (syscall(SYS_move_pages, 0, 1UL, &pg, nullptr, &status, 0) == 0 && status >= 0) return status;
    // driver mappings (the runtime's signal pages) answer no page: the node
    // /proc/self/numa_maps gives their mapping (its "N<node>=<pages>" fields,
    // the node holding most of them)
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    uintptr_t vma = 0;
    bool found = false;
    char line[4096];
    if (FILE *m = fopen("/proc/self/maps", "r")) {
        while (!found && fgets(line, sizeof line, m)) {
            char *dash = nullptr;
            const uintptr_t lo = (uintptr_t)strtoull(line, &dash, 16);
            const uintptr_t hi = dash && *dash == '-' ? (uintptr_t)strtoull(dash + 1, nullptr, 16) : 0;
            if (lo <= a && a < hi) {
                vma = lo;
                found = true;
            }
        }
        fclose(m);
    }
    FILE *f = found ? fopen("/proc/self/numa_maps", "r") : nullptr;
    if (!f) return -1;
    int node = -1;
    while (fgets(line, sizeof line, f)) {
        if ((uintptr_t)strtoull(line, nullptr, 16) != vma) continue;
        long most = 0;
        for (char *t = strstr(line, " N"); t; t = strstr(t + 1, " N")) {
            int n = -1;
            long pages = 0;
            if (sscanf(t, " N%d=%ld", &n, &pages) == 2 && pages > most) {
                most = pages;
                node = n;
            }
        }
    }
    fclose(f);
    return node;
}
// NUMA node of a CPU: the nodeN entry of its sysfs directory
int cpu_node(int cpu) {
    if (cpu < 0) return -1;
    char path[64];
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d", cpu);
    DIR *d = opendir(path);
    if (!d) return -1;
    int node = -1;
    for (struct dirent *e; (e = readdir(d)) != nullptr;)
        if (!strncmp(e->d_name, "node", 4) && e->d_name[4] >= '0' && e->d_name[4] <= '9') {
            node = atoi(e->d_name + 4);
            break;
        }
    closedir(d);
    return node;
}
// NUMA node of HIP device dev's PCI function (-1: unknown or no NUMA)
int device_node(int dev) {
    char bus[64] = {};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    for (char *c = bus; *c; ++c) *c = (char)tolower((unsigned char)*c);
    char path[128];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    return node;
}
}  // namespace

// MPIR_CVAR_REDUCE_LOCAL_BIND=gpu-node (opt-in, default off): at its first
// direct call on a device, the calling thread binds itself to the CPUs of that
// device's NUMA node (within the CPUs it may already use) -- for programs whose
// launcher does not bind GPU ranks (Hydra binds nothing by default).  A caller
// near its GPU saves ~2 us per synchronous call (DESIGN.md §(d), "Where the
// caller runs").  A library changing its caller's affinity is a side effect, so
// it is only done when asked.
static void maybe_bind_near(int dev) {
    static const bool on = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_BIND");
        return e && !strcmp(e, "gpu-node");
    }();
    thread_local bool done = false;
    if (!on || done) return;
    done = true;
    const int node = device_node(dev);
    if (node < 0) return;
    char path[96];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE *f = fopen(path, "r");
    if (!f) return;
    cpu_set_t want, have;
    CPU_ZERO(&want);
    char buf[4096];
    if (fgets(buf, sizeof buf, f)) {
        for (char *t = strtok(buf, ",\n"); t; t = strtok(nullptr, ",\n")) {
            int a = -1, b = -1;
            if (sscanf(t, "%d-%d", &a, &b) == 2) {
                for (int c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, &want);
            } else if (sscanf(t, "%d", &a) == 1 && a >= 0 && a < CPU_SETSIZE) {
                CPU_SET(a, &want);
            }
        }
    }
    fclose(f);
    if (pthread_getaffinity_np(pthread_self(), sizeof have, &have) != 0) return;
    CPU_AND(&want, &want, &have);
    if (CPU_COUNT(&want) > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof want, &want);
}

// out: the calling thread's CPU, that CPU's NUMA node, device dev's NUMA node,
// the node of the page holding this thread's completion signal for dev (-1
// before its first direct call, or unknown), the node of the device's error
// word (-1 before the direct path initialised)
void direct_placement(int dev, int out[5]) {
    const int cpu = sched_getcpu();
    out[0] = cpu;
    out[1] = cpu_node(cpu);
    out[2] = dev >= 0 && dev < kMaxDirectDev ? device_node(dev) : -1;
    out[3] = dev >= 0 && dev < kMaxDirectDev && t_placed_sig[dev] ? page_node(t_placed_sig[dev])
             : dev >= 0 && dev < kMaxDirectDev && t_sig.have[dev]
                 ? page_node(reinterpret_cast<const void *>((uintptr_t)t_sig.sig[dev].handle))
                 : -1;
    out[4] = dev >= 0 && dev < kMaxDirectDev && g_dev[dev].err ? page_node((const void *)g_dev[dev].err) : -1;
}

// Where device dev's direct-path queue keeps its AQL ring: 1 in device memory,
// 0 in host memory, -1 no queue yet or not an HSA allocation (diagnostic; the
// bench records it per rank, DESIGN.md §(d) "Where the caller runs").
extern "C" int MPIR_Hip_direct_ring_location(int dev) {
    if (dev < 0 || dev >= kMaxDirectDev || !g_dev[dev].queue) return -1;
    hsa_amd_pointer_info_t info{};
    info.size = sizeof info;
    if (hsa_amd_pointer_info(g_dev[dev].queue->base_address, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        info.type != HSA_EXT_POINTER_TYPE_HSA)
        return -1;
    hsa_device_type_t t;
    if (hsa_agent_get_info(info.agentOwner, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return -1;
    return t == HSA_DEVICE_TYPE_GPU ? 1 : 0;
}

// How the caller waits for the completion signal (A/B knobs for
// tools/placement_ab.py; the defaults are the product's):
//   MPIR_CVAR_REDUCE_LOCAL_POLL_DELAY_US  spin on the clock, without reading
//       the signal, this long after the doorbell before polling it (0);
//   MPIR_CVAR_REDUCE_LOCAL_POLL_FLUSH=1   clflush the signal's line once the
//       call has seen it, so no CPU cache holds it when the CP next writes it (0).
struct PollCfg {
    uint64_t delay_ns = 0;
    bool flush = false;
};
const PollCfg &poll_cfg() {
    static const PollCfg c = [] {
        PollCfg v;
        if (const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_POLL_DELAY_US")) v.delay_ns = (uint64_t)atol(e) * 1000;
        if (const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_POLL_FLUSH")) v.flush = atoi(e) != 0;
        return v;
    }();
    return c;
}
static inline uint64_t mono_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// 1: dispatched and completed (rc set); 0: not applicable, use the HIP path.
// `p` is plan_reduce's launch plan of the call (padding bytes zero).
int direct_reduce(int dev, int op, int elem, const ReducePlan &p, int *rc) {
    if (mode() == 0 || dev < 0 || dev >= kMaxDirectDev || op <= 0 || op >= MPIR_HIP_NOPS || elem <= 0 ||
        elem >= MPIR_HIP_NELEMS || p.kind < 0 || p.kind >= kPlanKinds || p.arg_bytes != kPlanArgBytes[p.kind])
        return 0;
    maybe_bind_near(dev);
    const bool prof = g_profile.load(std::memory_order_relaxed) != 0;
    const uint64_t th0 = prof ? sys_ts() : 0;
    uint64_t th1 = 0;
    DevState &d = g_dev[dev];
    std::call_once(d.once, [&] { init_dev(dev, d); });
    if (!d.ok || d.queue_error.load(std::memory_order_relaxed)) return 0;
    const uint64_t ko = d.kobj[0][p.kind][op][elem], ko_checked = d.kobj[1][p.kind][op][elem];
    // the packet's grid_size_x (workgroups x kThreads) is 32 bits
    if (!ko || !ko_checked || p.groups == 0 || p.groups > (uint64_t)UINT32_MAX / kThreads) return 0;
    // Work queued on the legacy null stream stays ordered before us, as it is
    // for the HIP path's blocking library stream.  hipStreamQuery(nullptr)
    // keeps answering "not ready" after such work has finished until the host
    // synchronises with it (measured: tools/archive/direct_probe.py), so a busy answer
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
    amd_signal_t *psig = !prof && signal_node_knob() >= 0 ? placed_signal(dev) : nullptr;
    if (psig) sig.handle = (uint64_t)(uintptr_t)psig;
    else if (!t_sig.get(dev, &sig)) return 0;
    uint64_t t_rung = 0;
    const uint32_t groups = (uint32_t)p.groups;
    const unsigned char *ka = p.args;
    const uint32_t kn = p.arg_bytes;
    if (psig) __atomic_store_n(&psig->value, (int64_t)1, __ATOMIC_RELAXED);
    else hsa_signal_store_relaxed(sig, 1);
    CacheEntry *held = nullptr;
    int ring = -1;
    bool checked = true;
    {
        std::lock_guard<std::mutex> lk(d.publish);
        hsa_queue_t *q = prof ? profiled_queue(d) : d.queue;
        // read under the lock, after profiled_queue(): the first profiled call's
        // probe of the twin queue may just have switched the device to read-back
        // flushes, and this call must already follow that protocol
        const bool rb = d.readback.load(std::memory_order_relaxed);
        const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) _mm_pause();
        char *slot = nullptr;
        bool write_args = true;
        // a free slot of a ring (first slot `base` of d.karg, busy flags from `busy`)
        auto take_ring = [&](uint32_t base, uint32_t busy, uint32_t &next) -> bool {
            for (uint32_t k = 0; k < kRingSlots; ++k) {
                const uint32_t r = (next + k) % kRingSlots;
                if (d.ring_busy[busy + r].load(std::memory_order_acquire) == 0) {
                    ring = (int)(busy + r);
                    next = r + 1;
                    d.ring_busy[ring].store(1, std::memory_order_relaxed);
                    slot = d.karg + (size_t)(base + r) * kKargSlotBytes;
                    return true;
                }
            }
            return false;
        };
        if (prof) {
            if (!take_ring(kProfBase, kRingSlots, d.pslot)) return 0;
        } else {
            uint64_t h = ko;
            for (uint32_t w = 0; w < kn / 8; ++w) {
                uint64_t x;
                memcpy(&x, ka + 8 * w, 8);
                h = (h ^ x) * 0x9E3779B97F4A7C15ull;
            }
            h ^= h >> 29;
            const uint32_t ci = (uint32_t)(h % kCacheSlots);
            CacheEntry &e = d.cache[ci];
            const bool hit = e.ko == ko && e.n == kn && !memcmp(e.args, ka, kn);
            if (hit || e.inflight.load(std::memory_order_acquire) == 0) {
                slot = d.karg + (size_t)(kRingSlots + ci) * kKargSlotBytes;
                e.inflight.fetch_add(1, std::memory_order_acq_rel);
                held = &e;
                if (hit) {
                    write_args = false;
                    // read back complete by an earlier checked dispatch: as it stands
                    checked = !e.verified.load(std::memory_order_acquire);
                } else {
                    e.verified.store(0, std::memory_order_relaxed);
                    e.ko = ko;
                    e.n = kn;
                    memcpy(e.args, ka, kn);
                }
            } else if (!take_ring(0, 0, d.kslot)) {
                return 0;       // every ring slot in flight: the HIP path takes this call
            }
        }
        // the argument words that change, then each half's nonce (KargSlot);
        // the sfences order them on PCIe, so a half showing the nonce holds
        // its words
        uint64_t *ks = reinterpret_cast<uint64_t *>(slot);
        auto write_args_words = [&] {
            if (!write_args) return;
            uint64_t w[12] = {};
            memcpy(w, ka, kn);
            for (int i = 0; i < 6; ++i) {
                ks[i] = w[i];
                ks[8 + i] = w[6 + i];
            }
            _mm_sfence();
            g_kernarg_writes.fetch_add(1, std::memory_order_relaxed);
        };
        // The test hook moves the write behind the doorbell, held back
        // `late` us: what a write that loses the race to the CP would cost
        // (tools/late_write_probe.py; tests/test_direct_timeout_gpu.py)
        const uint32_t late = checked && !rb ? g_test_write_delay_us.load(std::memory_order_relaxed) : 0;
        if (checked && rb) {
            // dispatch ids are not our indices: the slot is visible before the
            // doorbell (flush read back) and the unchecked kernel runs
            write_args_words();
            *d.hdp = 1u;
            (void)*d.hdp;
        } else if (checked && !late) {
            // Before the doorbell: the argument words, then the nonce, then an
            // HDP flush that is not read back.  The CP's ~4 us from doorbell to
            // dispatch lands them long before any workgroup reads the slot; the
            // checked kernel's nonce guards the rare read that still finds an
            // older line (direct_tiles.hip checked_args).  Written after the
            // doorbell instead, a miss cost 0.3-0.6 us less per call but a
            // write that lost the race stalled every first-round workgroup in
            // L2 invalidations: +57 us for a write 2 us late, +180 us at 4 us
            // (profiles/archive/r03/late_write_probe.log), and fresh-argument loops
            // 3-6 % slow on some boxes.
            write_args_words();
            ks[7] = idx + 1;
            ks[15] = idx + 1;
            _mm_sfence();
            *d.hdp = 1u;
        }
        // a checked grid spans every XCD (kMinCheckedGroups): then each XCD's
        // L2 holds the fresh line, or none, when a later hit runs unchecked.
        // Read-back mode pads its misses too: their dispatch marks
        // the entry verified as well, and the unchecked kernels' extra
        // workgroups start past the region and exit
        publish_packet(q, idx, checked && !rb ? ko_checked : ko, slot, sig, kThreads,
                       checked && groups < kMinCheckedGroups ? kMinCheckedGroups : groups);
        if (prof) th1 = sys_ts();
        hsa_signal_store_screlease(q->doorbell_signal, idx);
        if (poll_cfg().delay_ns) t_rung = mono_ns();
        if (late) {
            const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(late);
            while (std::chrono::steady_clock::now() < t_end) _mm_pause();
            write_args_words();
            ks[7] = idx + 1;
            ks[15] = idx + 1;
            _mm_sfence();
            *d.hdp = 1u;
        }
    }
    if (t_rung)
        while (mono_ns() - t_rung < poll_cfg().delay_ns) _mm_pause();
    for (uint64_t it = 1; (psig ? __atomic_load_n(&psig->value, __ATOMIC_ACQUIRE) : hsa_signal_load_scacquire(sig)) != 0;
         ++it) {
        if ((it & 0xFFFF) == 0 && d.queue_error.load(std::memory_order_relaxed)) {
            *rc = MPIR_HIP_ERUNTIME;
            return 1;       // (the entry stays held: a faulted queue is not used again)
        }
        _mm_pause();
    }
    if (poll_cfg().flush) _mm_clflush(reinterpret_cast<const char *>((uintptr_t)sig.handle) + 8);
    if (__builtin_expect(*d.err != 0, 0)) {
        // a workgroup never saw its arguments land (direct_tiles.hip
        // checked_args) and combined nothing: this call fails, and the path is
        // closed (the slot stays held)
        d.queue_error.store(-2, std::memory_order_relaxed);
        *rc = MPIR_HIP_ERUNTIME;
        return 1;
    }
    if (held) {
        // every workgroup of a checked dispatch saw the write: later hits on the
        // entry may take the unchecked kernel
        if (checked) held->verified.store(1, std::memory_order_release);
        held->inflight.fetch_sub(1, std::memory_order_acq_rel);
    }
    if (ring >= 0) d.ring_busy[ring].store(0, std::memory_order_release);
    if (prof) {
        const uint64_t th2 = sys_ts();
        hsa_amd_profiling_dispatch_time_t t{};
        const bool okt = hsa_amd_profiling_get_dispatch_time(d.agent, sig, &t) == HSA_STATUS_SUCCESS && g_ts_freq;
        const double ns = okt ? 1e9 / (double)g_ts_freq : 0.0;
        t_last_kernel_ns = okt ? (uint64_t)((double)(t.end - t.start) * ns) : 0;
        // the dispatch times are in the system domain, like HSA_SYSTEM_INFO_TIMESTAMP
        t_last_split[0] = (uint64_t)((double)(th1 - th0) * ns);
        // (the CP's stamps come through the runtime's clock translation: one
        // may land before th0 -- stored as a two's-complement int64)
        t_last_split[1] = okt ? (uint64_t)(int64_t)((double)((int64_t)(t.start - th0)) * ns) : 0;
        t_last_split[2] = okt ? (uint64_t)(int64_t)((double)((int64_t)(t.end - th0)) * ns) : 0;
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

// Initialise device `dev`'s direct path now (HSA queue, the 3.4 MB code object,
// kernarg slots, the dispatch-id probe: 2-10 ms) instead of in its first call;
// for MPI_Init-time integration.  Returns direct_state().
int direct_prepare(int dev) {
    if (mode() == 0) return -20;
    if (dev < 0 || dev >= kMaxDirectDev) return -21;
    DevState &d = g_dev[dev];
    std::call_once(d.once, [&] { init_dev(dev, d); });
    return d.state;
}

int direct_state(int dev) {
    if (mode() == 0) return -20;
    if (dev < 0 || dev >= kMaxDirectDev) return -21;
    return g_dev[dev].state;
}

uint64_t direct_busy_skips() { return g_busy_skips.load(std::memory_order_relaxed); }

uint64_t direct_kernarg_writes() { return g_kernarg_writes.load(std::memory_order_relaxed); }

uint32_t direct_test_write_delay_us(uint32_t us) { return g_test_write_delay_us.exchange(us); }

// the next probe of a twin (profiled) queue reports a mismatch, as under a tool
// that intercepts the queue: the first profiled call must switch the device to
// read-back flushes and still complete (tests only)
void direct_test_fail_probe() { g_test_fail_probe.store(true); }

}  // namespace mpir_hip
