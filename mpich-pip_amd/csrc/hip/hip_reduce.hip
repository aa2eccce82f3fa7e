// hip_reduce.hip -- C-ABI shim: (op, element class) dispatch, pointer
// classification, per-thread streams, host-operand staging.
//
// Replaces the scalar loop body the reference runs inside each MPIR_<OP>
// (src/mpi/coll/op/op*.c via MPIR_OP_TYPE_REDUCE_CASE,
// src/include/mpir_op_util.h:48-55).  Declared in include/mpir_hip_reduce.h.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include "mpir_hip_reduce.h"
#include "kernel_table.hpp"

using namespace mpir_hip;

namespace {

// Kernel tables (kernel_table.hpp), filled by the registration units
// reg_*.hip at static-initialisation time; zero-initialised storage here.
}  // namespace

namespace mpir_hip {
int direct_reduce(int dev, int op, int elem, const ReducePlan &p, int *rc);  // direct_dispatch.hip
uint64_t direct_calls();
void direct_profile(int on);
uint64_t direct_last_kernel_ns();
int direct_state(int dev);
int direct_prepare(int dev);
void direct_last_split(uint64_t out[4]);
uint64_t direct_busy_skips();
uint64_t direct_kernarg_writes();
uint32_t direct_test_write_delay_us(uint32_t us);
void direct_test_fail_probe();
void direct_placement(int dev, int out[5]);
Entry g_table[MPIR_HIP_NOPS][MPIR_HIP_NELEMS];
multi_fn g_multi[MPIR_HIP_NOPS][MPIR_HIP_NELEMS][2][kMultiMaxP - 1];

// Results of at most this many bytes are stored sc1 (into the Infinity Cache)
// rather than nt: MPIR_CVAR_REDUCE_LOCAL_KEEP_MB (0 = every store nt), default
// 64 (reduce_kernels.hpp, kKeepBytes); MPIR_Hip_set_keep_bytes() changes it at
// run time (an MPI_T-style cvar write).
std::atomic<uint64_t> g_keep{[] {
    const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_KEEP_MB");
    if (!e) return kKeepBytes;
    const long mb = atol(e);
    return (uint64_t)(mb >= 0 && mb <= 4096 ? mb : 64) << 20;
}()};
uint64_t keep_bytes() { return g_keep.load(std::memory_order_relaxed); }

// ... and results of at most this many bytes are stored nt again: below it the
// sc1 stores cost the call more at the kernel's end than a next reader gains
// from finding the result in the Infinity Cache (tools/keep_small_ab.py,
// profiles/r06/keep_small_r06z.log: nt ahead by 0.3-1.0 us per call from 16 KiB
// to 16 MiB whether or not the next call re-reads the result; sc1 ahead by
// 0.6-1.7 us at 32-64 MiB when it does).  MPIR_CVAR_REDUCE_LOCAL_KEEP_MIN_MB,
// default 16; MPIR_Hip_set_keep_min_bytes() at run time.
std::atomic<uint64_t> g_keep_min{[] {
    const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_KEEP_MIN_MB");
    const long mb = e ? atol(e) : 16;
    return (uint64_t)(mb >= 0 && mb <= 4096 ? mb : 16) << 20;
}()};

uint64_t keep_for(uint64_t vbytes) {
    return vbytes > g_keep_min.load(std::memory_order_relaxed) && vbytes <= keep_bytes() ? vbytes : 0;
}

// MPIR_Hip_combine_set_flags: the calling thread's combine flags
thread_local int t_combine_flags = 0;
bool multi_uncapped() { return (t_combine_flags & MPIR_HIP_COMBINE_UNCAPPED) != 0; }
}  // namespace mpir_hip

namespace {

const size_t g_elem_size[MPIR_HIP_NELEMS] = {
    0, 1, 1, 2, 2, 4, 4, 8, 8, 2, 4, 8, 8, 16, 8, 8, 16, 8, 16, 16, 32, 32,
};
static_assert(sizeof(g_elem_size) / sizeof(g_elem_size[0]) == MPIR_HIP_NELEMS, "one size per element class");

// ------------------------------------------------------------ per-thread state
constexpr int kMaxDev = 64;
constexpr int kMaxStageSlots = 8;

// Staging of host (or other-device) operands: chunks of `stage_chunk()` bytes
// per operand flow through a three-stage pipeline -- H2D copies on stream
// "up", the kernel on "comp", the D2H copy-back on "down" -- over
// `stage_slots()` device scratch slots, so host->device and device->host
// transfers run at the same time (PCIe is full duplex).  Events order the
// stages of one chunk and stop a slot from being refilled before its
// copy-back has read it.  Defaults 16 MiB x 3 slots (tools/archive/stage_sweep.py,
// profiles/archive/r01s3_stage_sweep.log: pinned 71.8 GiB/s, pageable 66.3 with the
// bounce path below; 32 MiB chunks leave a longer tail of copy-outs).
// MPIR_CVAR_REDUCE_LOCAL_STAGE_CHUNK_MB / MPIR_CVAR_REDUCE_LOCAL_STAGE_SLOTS override.
// (function-local statics: initialised once, thread-safe)
uint64_t stage_chunk() {
    static const uint64_t v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_STAGE_CHUNK_MB");
        const long mb = e ? atol(e) : 0;
        return (uint64_t)(mb > 0 && mb <= 1024 ? mb : 16) << 20;
    }();
    return v;
}
int stage_slots() {
    static const int v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_STAGE_SLOTS");
        const int n = e ? atoi(e) : 0;
        return n >= 2 && n <= kMaxStageSlots ? n : 3;
    }();
    return v;
}

enum { S_MAIN = 0, S_UP = 1, S_COMP = 2, S_DOWN = 3, S_NSTREAMS = 4 };

struct DevCtx {
    hipStream_t stream[S_NSTREAMS] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_up[kMaxStageSlots] = {}, ev_comp[kMaxStageSlots] = {}, ev_free[kMaxStageSlots] = {};
    volatile uint32_t *flag = nullptr;   // pinned completion word (wait mode "flag")
    uint32_t seq = 0;
    bool main_pending = false;   // work enqueued on stream[S_MAIN] without a wait (stream variant)
    char *scratch = nullptr;     // staging slots x (in, inout) x chunk, or multi-operand temporaries
    size_t scratch_bytes = 0;
    char *bounce = nullptr;      // pinned host bounce slots x (in, inout) x chunk (pageable operands)
    size_t bounce_bytes = 0;
    char *zc = nullptr;          // pinned, device-mapped slot for small mixed-residency calls
    size_t zc_bytes = 0;
};

// HIP's verdict on host pages the HSA query does not know (classify below)
struct HostVerdict {
    uintptr_t page = ~(uintptr_t)0;
    int loc = 0;
    int dev = 0;
};
constexpr int kVerdicts = 16;

struct ThreadCtx {
    DevCtx dev[kMaxDev];
    char err[256] = {0};
    HostVerdict verdict[kVerdicts];
    ThreadCtx *next = nullptr;
};

// Per-thread contexts (streams, events, completion word, scratch) come from a
// process-wide pool: a thread takes one at its first call and hands it back
// when it exits, so an application that starts and ends many threads reuses
// a bounded set of HIP streams instead of leaking one set per thread.  A
// handed-back context keeps its streams (work still queued on them stays in
// order for the next owner); thread exit makes no HIP call, so it is safe at
// process teardown too.
std::mutex g_pool_mu;
ThreadCtx *g_pool = nullptr;
int g_ctx_created = 0;

struct CtxHolder {
    ThreadCtx *c = nullptr;
    ThreadCtx &get() {
        if (!c) {
            std::lock_guard<std::mutex> lk(g_pool_mu);
            if (g_pool) {
                c = g_pool;
                g_pool = c->next;
                c->next = nullptr;
                c->err[0] = 0;
                for (HostVerdict &v : c->verdict) v = HostVerdict();    // a new thread's own verdicts
            } else {
                c = new ThreadCtx();
                ++g_ctx_created;
            }
        }
        return *c;
    }
    ~CtxHolder() {
        if (!c) return;
        std::lock_guard<std::mutex> lk(g_pool_mu);
        c->next = g_pool;
        g_pool = c;
        c = nullptr;
    }
};

thread_local CtxHolder t_holder;
inline ThreadCtx &ctx() { return t_holder.get(); }

int set_err(hipError_t e, const char *what) {
    snprintf(ctx().err, sizeof(ctx().err), "%s: %s", what, hipGetErrorString(e));
    return MPIR_HIP_ERUNTIME;
}

#define HIPCHK(call) do { hipError_t e_ = (call); if (e_ != hipSuccess) return set_err(e_, #call); } while (0)

int get_stream(int dev, int slot, hipStream_t *out) {
    DevCtx &d = ctx().dev[dev];
    if (!d.stream[slot]) {
        // Blocking stream (not hipStreamNonBlocking): it orders after work the
        // caller queued on the legacy null stream for these buffers.
        HIPCHK(hipStreamCreate(&d.stream[slot]));
    }
    *out = d.stream[slot];
    return MPIR_HIP_OK;
}

int get_stage_events(int dev, int nslots) {
    DevCtx &d = ctx().dev[dev];
    for (int k = 0; k < nslots; ++k) {
        if (!d.ev_up[k]) HIPCHK(hipEventCreateWithFlags(&d.ev_up[k], hipEventDisableTiming));
        if (!d.ev_comp[k]) HIPCHK(hipEventCreateWithFlags(&d.ev_comp[k], hipEventDisableTiming));
        if (!d.ev_free[k]) HIPCHK(hipEventCreateWithFlags(&d.ev_free[k], hipEventDisableTiming));
    }
    return MPIR_HIP_OK;
}

int get_scratch(int dev, size_t bytes, char **out) {
    DevCtx &d = ctx().dev[dev];
    if (d.scratch_bytes < bytes) {
        // stream-ordered users of the old scratch may still be in flight
        if (d.scratch) HIPCHK(hipDeviceSynchronize());
        if (d.scratch) HIPCHK(hipFree(d.scratch));
        d.scratch = nullptr;
        d.scratch_bytes = 0;
        HIPCHK(hipMalloc(&d.scratch, bytes));
        d.scratch_bytes = bytes;
    }
    *out = d.scratch;
    return MPIR_HIP_OK;
}

int get_bounce(int dev, size_t bytes, char **out) {
    DevCtx &d = ctx().dev[dev];
    if (d.bounce_bytes < bytes) {
        if (d.bounce) HIPCHK(hipDeviceSynchronize());   // in-flight copies may still read it
        if (d.bounce) HIPCHK(hipHostFree(d.bounce));
        d.bounce = nullptr;
        d.bounce_bytes = 0;
        HIPCHK(hipHostMalloc(&d.bounce, bytes, hipHostMallocDefault));
        d.bounce_bytes = bytes;
    }
    *out = d.bounce;
    return MPIR_HIP_OK;
}

// Host copies of the bounce path, split over a small process-wide pool of
// worker threads: one thread moves 31-33 GB/s between pageable and pinned
// memory on the MI355X host, four 83-86 GB/s (tools/memcpy_bw.cpp,
// profiles/archive/r01s3_memcpy_bw.log) -- more than the ~51 GB/s a PCIe Gen5 x16
// upload takes; the host combine uses every thread (copy_pool() below).
// MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS (1 = the calling thread alone).  The pool is never torn down: its idle workers end
// with the process, so exit never waits on them.
class CopyPool {
  public:
    // `cpus`: the workers may run on these CPUs only (a NUMA node's pool: the
    // scheduler still balances them over the node); empty: the process's mask
    CopyPool(int nthreads, int copy_parts, std::vector<int> cpus = {})
        : n_(nthreads), copy_n_(std::min(nthreads, copy_parts)), pid_(getpid()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int c : cpus) CPU_SET(c, &set);
        for (int i = 1; i < n_; ++i)
            std::thread([this, set, pin = !cpus.empty()] {
                if (pin) (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
                work();
            }).detach();
    }
    int threads() const { return n_; }
    // fn(ctx, k) for every k < nparts, the parts handed out one at a time to
    // the calling thread and the workers alike, so a slower thread (remote
    // memory, a throttled or preempted CPU) simply takes fewer; returns when
    // all are done.  One job at a time: a caller that finds the workers busy
    // with another thread's job runs its parts alone rather than waiting, so
    // concurrent callers (other devices, other host combines) never serialise
    // behind each other.
    void run(size_t nparts, void (*fn)(void *, size_t), void *ctx) {
        std::unique_lock<std::mutex> job(job_mu_, std::defer_lock);
        // a forked child has none of the workers: run alone there
        if (n_ <= 1 || nparts <= 1 || getpid() != pid_ || !job.try_lock()) {
            for (size_t k = 0; k < nparts; ++k) fn(ctx, k);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = fn;
            ctx_ = ctx;
            nparts_ = nparts;
            next_ = 1;                                  // part 0 is the caller's
            pending_ = nparts - 1;
            ++gen_;
        }
        // wake only as many workers as there are parts for (a copy of 4
        // parts on a 16-thread pool: +9 us at 1 MiB with notify_all)
        for (size_t k = 1; k < nparts && k < (size_t)n_; ++k) cv_.notify_one();
        fn(ctx, 0);
        std::unique_lock<std::mutex> lk(mu_);
        while (next_ < nparts_) {
            const size_t k = next_++;
            lk.unlock();
            fn(ctx, k);
            lk.lock();
            --pending_;
        }
        done_.wait(lk, [this] { return pending_ == 0; });
    }
    // copies split into at most copy_n_ parts: PCIe, not the host's memory,
    // bounds them, and more parts only add wake-ups (host->device 1 MiB 52 ->
    // 74 us with 16 parts, profiles/archive/r02/host_threads_ab.log)
    void copy(char *dst, const char *src, size_t bytes, size_t min_split = (size_t)1 << 20) {
        if (copy_n_ <= 1 || bytes < min_split || getpid() != pid_) {
            memcpy(dst, src, bytes);
            return;
        }
        struct C {
            char *d;
            const char *s;
            size_t bytes, part;
        } c{dst, src, bytes, ((bytes + copy_n_ - 1) / copy_n_ + 63) & ~(size_t)63};
        run((bytes + c.part - 1) / c.part, [](void *p, size_t k) {
            const C *c = static_cast<const C *>(p);
            const size_t o = k * c->part;
            memcpy(c->d + o, c->s + o, std::min(c->part, c->bytes - o));
        }, &c);
    }

  private:
    void work() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            while (next_ < nparts_) {
                const size_t k = next_++;
                lk.unlock();
                fn_(ctx_, k);
                lk.lock();
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_, copy_n_;
    pid_t pid_;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_;
    void (*fn_)(void *, size_t) = nullptr;
    void *ctx_ = nullptr;
    size_t nparts_ = 0, next_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
};

// Ranks of this job on this node (>= 1).  Every rank of a host-buffer
// MPI_Allreduce reaches its combine at the same moment, so the node's CPUs are
// shared by all of them.  Sources, in order: MPIR_Hip_set_local_ranks() (inside
// libmpi the glue passes MPICH's node communicator size, mpich_glue.c), then
// the launcher's environment -- MPI_LOCALNRANKS (Hydra, pmip_cb.c:658-662),
// MPIR_PIP_SIZE (this repo's mpiexec: one node), LOCAL_WORLD_SIZE (torchrun),
// OMPI_COMM_WORLD_LOCAL_SIZE (Open MPI's launcher); none: 1.
std::atomic<int> g_local_ranks{0};
int local_ranks() {
    const int set = g_local_ranks.load(std::memory_order_relaxed);
    if (set > 0) return set;
    static const int env = [] {
        for (const char *k : {"MPI_LOCALNRANKS", "MPIR_PIP_SIZE", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"})
            if (const char *e = getenv(k)) {
                const int n = atoi(e);
                if (n >= 1 && n <= (1 << 20)) return n;
            }
        return 1;
    }();
    return env;
}

// Host-combine threads for one rank, from the CPUs the node's L local ranks
// share (the reference's combine is one thread per rank,
// opsum.c:21-76):
//   * affinity: a mask of m of the c CPUs the job may use (the cgroup's cpuset,
//     else the online CPUs).  Ranks bound to disjoint sets (L * m <= c) each
//     own their mask; unbound ranks (m = c) share it L ways; in between (e.g.
//     --bind-to socket) ceil(L * m / c) ranks share each mask;
//   * cgroup quota q (cpu.max): the job's or container's, shared by all L.
// The share is at most 16 (the host combine's measured scaling: 256 MiB fp32
// SUM, 16-CPU quota, 131-136 GiB/s on 4 threads, 259-299 on 16;
// profiles/archive/r02/host_threads_ab.log).  No floor: with at most one CPU
// per rank the caller combines alone and the library starts no thread, as
// MPICH's loop starts none (8 unbound ranks on this job's 16-CPU quota: one
// worker each beside the caller).  Copies (bounce path, mixed-residency slots)
// keep to at most 4 parts, which already outrun a PCIe upload.
// MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS sets both (1 = the caller alone).
// (pool_threads() sizes a pool without creating one: the floating pool's
// threads start only when a copy or a combine off the operands' node needs
// them, never beside a NUMA node's pool that does the work; the size is fixed
// at the first call, so MPIR_Hip_set_local_ranks() acts before the first host
// combine)
int parse_cpulist(const char *path, std::vector<int> &out);
// This process's own cgroup, as /proc/self/cgroup names it: the v2 path ("0::")
// or the v1 path of `controller`; "" if the file or the entry is missing.  The
// cgroup files are read there and up its ancestors (without a
// cgroup namespace -- Slurm on bare metal -- the mount's root files describe
// the whole node, not this job).
std::string own_cgroup(const char *controller) {
    FILE *f = fopen("/proc/self/cgroup", "r");
    if (!f) return "";
    char line[1024];
    std::string v2, v1;
    while (fgets(line, sizeof line, f)) {
        line[strcspn(line, "\n")] = 0;
        char *c1 = strchr(line, ':');
        char *c2 = c1 ? strchr(c1 + 1, ':') : nullptr;
        if (!c2) continue;
        *c2 = 0;
        const char *ctrls = c1 + 1, *path = c2 + 1;
        if (!strncmp(line, "0", 2) && !*ctrls) v2 = path;
        for (const char *t = ctrls; *t;) {                  // "cpu,cpuacct"
            const size_t n = strcspn(t, ",");
            if (n == strlen(controller) && !strncmp(t, controller, n)) v1 = path;
            t += n + (t[n] == ',');
        }
    }
    fclose(f);
    return !v1.empty() ? "/sys/fs/cgroup/" + std::string(controller) + v1 : (!v2.empty() ? "/sys/fs/cgroup" + v2 : "");
}
// dir and its ancestors up to the mount point (inclusive), innermost first
std::vector<std::string> cgroup_chain(const std::string &dir, const char *mount) {
    std::vector<std::string> out;
    std::string d = dir;
    while (d.size() > strlen(mount) && d.compare(0, strlen(mount), mount) == 0) {
        while (d.size() > 1 && d.back() == '/') d.pop_back();
        out.push_back(d);
        d = d.substr(0, d.rfind('/'));
    }
    out.push_back(mount);
    return out;
}
// The CPUs the job's ranks can share: this process's cgroup cpuset (a
// container pinned to 16 of the host's 256 CPUs gives every unbound rank that
// same 16-CPU mask), read at its own cgroup or the nearest ancestor that has
// one.  If no cpuset can be found, `mask` (this process's affinity): the L
// local ranks are then taken to share it, the conservative reading.
int online_cpus(int mask) {
    const std::string v1 = own_cgroup("cpuset");
    const bool is_v1 = v1.compare(0, 22, "/sys/fs/cgroup/cpuset/") == 0 || v1 == "/sys/fs/cgroup/cpuset";
    const char *mount = is_v1 ? "/sys/fs/cgroup/cpuset" : "/sys/fs/cgroup";
    const char *file = is_v1 ? "/cpuset.effective_cpus" : "/cpuset.cpus.effective";
    if (!v1.empty())
        for (const std::string &d : cgroup_chain(v1, mount)) {
            std::vector<int> cpus;
            if (parse_cpulist((d + file).c_str(), cpus) == 0 && !cpus.empty()) return (int)cpus.size();
        }
    return mask >= 1 ? mask : 1;
}
// the cgroup's CPU quota in CPUs (v2 cpu.max "quota period", v1 cfs_quota_us /
// cfs_period_us) -- the smallest along this process's cgroup and its
// ancestors -- 0 if none
int cgroup_quota_cpus() {
    const std::string own = own_cgroup("cpu");
    if (own.empty()) return 0;
    const bool is_v1 = own.compare(0, 19, "/sys/fs/cgroup/cpu/") == 0 || own == "/sys/fs/cgroup/cpu";
    long best = 0;
    for (const std::string &d : cgroup_chain(own, is_v1 ? "/sys/fs/cgroup/cpu" : "/sys/fs/cgroup")) {
        long quota = -1, period = 0;
        if (!is_v1) {
            if (FILE *f = fopen((d + "/cpu.max").c_str(), "r")) {
                char q[32];
                if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0) quota = atol(q);
                fclose(f);
            }
        } else if (FILE *fq = fopen((d + "/cpu.cfs_quota_us").c_str(), "r")) {
            if (fscanf(fq, "%ld", &quota) != 1) quota = -1;
            fclose(fq);
            if (FILE *fp = fopen((d + "/cpu.cfs_period_us").c_str(), "r")) {
                if (fscanf(fp, "%ld", &period) != 1) period = 0;
                fclose(fp);
            }
        }
        if (quota <= 0 || period <= 0) continue;
        const long v = (quota + period - 1) / period;
        if (v >= 1 && v < (1L << 20) && (best == 0 || v < best)) best = v;
    }
    return (int)best;
}
int share_threads(int mask, int online, int quota, int L) {
    if (L < 1) L = 1;
    if (mask < 1) mask = 1;
    if (online < mask) online = mask;
    int sharers = (int)(((long)L * mask + online - 1) / online);
    sharers = std::max(1, std::min(L, sharers));
    int n = mask / sharers;
    if (quota > 0) n = std::min(n, quota / L);
    return std::max(1, std::min(16, n));
}
const char *stage_threads_env() {
    static const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS");
    return e;
}
int pool_threads() {
    static const int n = [] {
        const char *e = stage_threads_env();
        if (e) {
            const int v = atoi(e);
            return v < 1 || v > 64 ? 4 : v;
        }
        cpu_set_t set;
        const int mask = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : 1;
        return share_threads(mask, online_cpus(mask), cgroup_quota_cpus(), local_ranks());
    }();
    return n;
}
CopyPool &copy_pool() {
    static CopyPool *pool = new CopyPool(pool_threads(), stage_threads_env() ? pool_threads() : 4);
    return *pool;
}

// ---- NUMA placement of the host combine ---------------------------------
// A both-host combine is bound by the host's memory bandwidth, and a thread
// reading the other socket's memory runs at about half the rate: torch /
// hipHostMalloc place pinned buffers on the GPU's node while a rank's pageable
// buffers sit wherever it first touched them, and the floating pool then
// reads most of one kind remotely (tools/pinned_read_probe.py,
// profiles/archive/r03/pinned_read_probe.log: the same 256 MiB fp32 SUM at 70-76 GiB/s
// for pinned operands on node 0 against 100-136 for pageable ones on node 1).
// When both operands' sampled pages sit on one node, the split runs on a pool
// confined to that node's CPUs (within the process's affinity mask);
// MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA=0 keeps the floating pool.
bool host_numa_enabled() {
    static const bool on = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

int parse_cpulist(const char *path, std::vector<int> &out) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    char buf[4096];
    const bool ok = fgets(buf, sizeof buf, f) != nullptr;
    fclose(f);
    if (!ok) return -1;
    for (char *p = buf; *p && *p != '\n';) {
        char *end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p) break;
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            p = end;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back((int)c);
        if (*p == ',') ++p;
    }
    return 0;
}

// per NUMA node: the CPUs of this process's affinity mask on it, the first
// hardware thread of every core before the second ones
const std::vector<std::vector<int>> &node_cpus() {
    static const std::vector<std::vector<int>> nodes = [] {
        std::vector<std::vector<int>> v;
        cpu_set_t mask;
        if (sched_getaffinity(0, sizeof mask, &mask) != 0) return v;
        for (int node = 0; node < 64; ++node) {
            char path[96];
            snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
            std::vector<int> all;
            v.emplace_back();
            if (parse_cpulist(path, all) != 0) continue;     // node ids need not be contiguous
            std::vector<int> first, second;
            for (int c : all) {
                if (!CPU_ISSET(c, &mask)) continue;
                snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", c);
                std::vector<int> sib;
                (parse_cpulist(path, sib) == 0 && !sib.empty() && sib[0] != c ? second : first).push_back(c);
            }
            first.insert(first.end(), second.begin(), second.end());
            v.back() = first;
        }
        return v;
    }();
    return nodes;
}

// NUMA nodes with CPUs this process may use
int usable_nodes() {
    static const int n = [] {
        int c = 0;
        for (const auto &cpus : node_cpus()) c += !cpus.empty();
        return c;
    }();
    return n;
}

// the NUMA node holding the sampled pages of both operands (start, middle and
// end of each), or -1 (mixed, not yet touched, or unknown)
int host_node(const void *a, const void *b, size_t bytes) {
    if (bytes == 0 || usable_nodes() < 2) return -1;
    void *pages[6];
    int status[6];
    const uintptr_t base[2] = {reinterpret_cast<uintptr_t>(a), reinterpret_cast<uintptr_t>(b)};
    for (int i = 0; i < 2; ++i) {
        pages[3 * i] = reinterpret_cast<void *>(base[i] & ~(uintptr_t)4095);
        pages[3 * i + 1] = reinterpret_cast<void *>((base[i] + bytes / 2) & ~(uintptr_t)4095);
        pages[3 * i + 2] = reinterpret_cast<void *>((base[i] + bytes - 1) & ~(uintptr_t)4095);
    }
    if (syscall(SYS_move_pages, 0, 6, pages, nullptr, status, 0) != 0) return -1;
    for (int i = 1; i < 6; ++i)
        if (status[i] != status[0]) return -1;
    return status[0] >= 0 && status[0] < (int)node_cpus().size() ? status[0] : -1;
}

// the pool for a both-host combine of `bytes` per operand: pinned to the
// operands' node when they share one (and it has CPUs of ours), else the
// floating pool
CopyPool &combine_pool(const void *a, const void *b, size_t bytes) {
    static std::mutex mu;
    static CopyPool *per_node[64] = {};
    const int node = host_numa_enabled() ? host_node(a, b, bytes) : -1;
    if (node < 0 || node >= 64 || node_cpus()[(size_t)node].size() < 2) return copy_pool();
    std::lock_guard<std::mutex> lk(mu);
    if (!per_node[node]) {
        const std::vector<int> &cpus = node_cpus()[(size_t)node];
        const int n = std::min<int>(pool_threads(), (int)cpus.size());
        // n - 1 workers confined to the node's CPUs and the caller: no more
        // threads than the floating pool (the CPUs the process may use)
        per_node[node] = new CopyPool(n, 4, cpus);
    }
    return *per_node[node];
}

// LOC_HOST: pageable (or unknown to HIP); LOC_PINNED: page-locked host memory
// (hipHostMalloc / hipHostRegister), which DMA copies and kernels may still be
// writing when the caller hands it over
enum Loc { LOC_HOST = 0, LOC_DEVICE = 1, LOC_PINNED = 2 };

// Both operands in host memory and at most this many bytes each: the combine
// runs on the host (host_loop, the same functors as the kernels; split over
// the copy pool's threads from host_split_bytes()) instead of a staged GPU
// round trip -- SURVEY.md §8b's dispatch rule ("both host -> CPU").  Measured
// on the MI355X host, fp32 SUM (tools/host_latency.py, tools/host_crossover.py,
// profiles/archive/r02/host_latency*.log, host_crossover.log): the host combine wins at
// every size -- 0.4 us against 48 us staged at 4 B, 35 against 125-194 us at
// 1 MiB, 108 against 299-466 us at 4 MiB, 5.6-5.7 against 10.7-13.9 ms at 256 MiB
// (staging is PCIe-bound, ~50 GB/s up).  MPIR_CVAR_REDUCE_LOCAL_HOST_MAX_KB:
// unset or negative = no limit (default), 0 = always stage through the GPU;
// MPIR_Hip_set_host_max_bytes() changes it at run time (as an MPI_T cvar write).
std::atomic<uint64_t> g_host_max{[] {
    const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_HOST_MAX_KB");
    if (!e) return ~(uint64_t)0;
    const long long kb = atoll(e);
    return kb < 0 ? ~(uint64_t)0 : ((uint64_t)kb << 10);
}()};
uint64_t host_max_bytes() { return g_host_max.load(std::memory_order_relaxed); }

// One operand in host memory, the other on a device, at most this many bytes:
// the host operand is copied into a pinned, device-mapped slot and the kernel
// reads (and for a host inoutbuf writes) it there over PCIe -- one dispatch, no
// DMA copies, no staging pipeline.  Measured fp32 SUM host -> device at count 1:
// 33 us through the staged pipeline (profiles/archive/r02/host_latency.log).
// MPIR_CVAR_REDUCE_LOCAL_MIXED_MAX_KB (default 1024; 0 = always stage).
uint64_t mixed_max_bytes() {
    static const uint64_t v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_MIXED_MAX_KB");
        const long kb = e ? atol(e) : 1024;
        return (uint64_t)(kb >= 0 && kb <= (1L << 20) ? kb : 1024) << 10;
    }();
    return v;
}

// copies into / out of the mixed path's slot of at least this many bytes go
// through the copy pool (MPIR_CVAR_REDUCE_LOCAL_MIXED_SPLIT_KB, default 512: the
// pool's wake-up costs ~10 us, more than it saves at 256 KiB, less at 1 MiB --
// device -> host 135 -> 72-85 us; profiles/archive/r02/mixed_split_ab.log)
size_t zc_split_bytes() {
    static const size_t v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_MIXED_SPLIT_KB");
        const long kb = e ? atol(e) : 512;
        return (size_t)(kb > 0 && kb <= (1L << 20) ? kb : 512) << 10;
    }();
    return v;
}

// the calling thread's small pinned slot (fine-grained: kernel stores land in
// host memory without a cache flush)
int get_zc(int dev, size_t bytes, char **out) {
    DevCtx &d = ctx().dev[dev];
    if (d.zc_bytes < bytes) {
        // a synchronous call's kernel is done with the old slot when it returned
        if (d.zc) HIPCHK(hipHostFree(d.zc));
        d.zc = nullptr;
        d.zc_bytes = 0;
        const size_t want = bytes < ((size_t)64 << 10) ? ((size_t)64 << 10) : bytes;
        HIPCHK(hipHostMalloc(&d.zc, want, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
        d.zc_bytes = want;
    }
    *out = d.zc;
    return MPIR_HIP_OK;
}

// host combines of at least this many bytes per operand are split over the
// copy pool's threads (MPIR_CVAR_REDUCE_LOCAL_HOST_SPLIT_KB, default 512)
uint64_t host_split_bytes() {
    static const uint64_t v = [] {
        const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_HOST_SPLIT_KB");
        const long kb = e ? atol(e) : 512;
        return (uint64_t)(kb > 0 && kb <= (1L << 22) ? kb : 512) << 10;
    }();
    return v;
}

// Whether this process has started the GPU runtime.  HIP runs on the HSA
// runtime, and device or pinned memory exists only once it is open, so until
// then every pointer is pageable host memory and the call needs no HIP query:
// a CPU-only program linked against libmpi with this drop-in never opens
// /dev/kfd for its host-buffer reductions, as MPICH's loop (opsum.c:21-76)
// never does.  hsa_system_get_info answers HSA_STATUS_ERROR_NOT_INITIALIZED
// without starting anything (ROCr's API table is bound when the library loads;
// measured: tools/kfd_probe.py), ~2 ns a call; once open, the answer is cached.
bool gpu_runtime_started() {
    static std::atomic<bool> up{false};
    if (up.load(std::memory_order_relaxed)) return true;
    uint16_t major = 0;
    if (hsa_system_get_info(HSA_SYSTEM_INFO_VERSION_MAJOR, &major) != HSA_STATUS_SUCCESS) return false;
    up.store(true, std::memory_order_relaxed);
    return true;
}

// HIP's view of a pointer (100-165 ns a query once HIP is up:
// profiles/r05/classify_cost.log)
Loc classify_hip(const void *p, int *dev) {
    hipPointerAttribute_t at;
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return LOC_HOST;
    }
    if (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged || at.type == hipMemoryTypeUnified) {
        *dev = at.device;
        return LOC_DEVICE;
    }
    if (at.type != hipMemoryTypeHost) return LOC_HOST;
    *dev = at.device;       // the device whose context allocated (registered) it
    return LOC_PINNED;
}

// HIP device ordinal of each HSA GPU agent, matched by PCI domain, bus and
// device (HIP_VISIBLE_DEVICES may hide and renumber agents HSA still lists).
// Empty when any visible device matches no agent or more than one (e.g. a
// partition mode sharing one BDF): the HSA query then answers nothing.
struct AgentMap {
    int n = 0;
    uint64_t handle[kMaxDev];
    int dev[kMaxDev];
    int ncpu = 0;
    uint64_t cpu[kMaxDev];      // CPU agents (owners of host pools)
};
const AgentMap &agent_map() {
    static const AgentMap m = [] {
        AgentMap am;
        struct Gpu { uint64_t handle; uint32_t bdf, domain; };
        std::vector<Gpu> gpus;
        (void)hsa_iterate_agents([](hsa_agent_t a, void *v) {
            hsa_device_type_t t;
            if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
            if (t == HSA_DEVICE_TYPE_CPU) {
                // a CPU agent: bdf 0xffffffff marks it (domain unused)
                static_cast<std::vector<Gpu> *>(v)->push_back(Gpu{a.handle, ~0u, ~0u});
                return HSA_STATUS_SUCCESS;
            }
            if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
            Gpu g{a.handle, 0, 0};
            if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &g.bdf) != HSA_STATUS_SUCCESS ||
                hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &g.domain) != HSA_STATUS_SUCCESS)
                return HSA_STATUS_SUCCESS;
            static_cast<std::vector<Gpu> *>(v)->push_back(g);
            return HSA_STATUS_SUCCESS;
        }, &gpus);
        for (const Gpu &g : gpus)
            if (g.bdf == ~0u && g.domain == ~0u && am.ncpu < kMaxDev) am.cpu[am.ncpu++] = g.handle;
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || ndev > kMaxDev) {
            (void)hipGetLastError();
            am.n = 0;
            return am;
        }
        for (int d = 0; d < ndev; ++d) {
            int dom = 0, bus = 0, slot = 0;
            if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, d) != hipSuccess ||
                hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, d) != hipSuccess ||
                hipDeviceGetAttribute(&slot, hipDeviceAttributePciDeviceId, d) != hipSuccess) {
                (void)hipGetLastError();
                am.n = 0;
                return am;
            }
            int hits = 0;
            for (const Gpu &g : gpus)
                if (g.bdf != ~0u && g.domain == (uint32_t)dom && ((g.bdf >> 8) & 0xff) == (uint32_t)bus &&
                    ((g.bdf >> 3) & 0x1f) == (uint32_t)slot) {
                    am.handle[am.n] = g.handle;
                    am.dev[am.n] = d;
                    ++hits;
                }
            if (hits != 1) {
                am.n = 0;
                return am;
            }
            ++am.n;
        }
        return am;
    }();
    return m;
}

int agent_device(hsa_agent_t a) {
    const AgentMap &m = agent_map();
    for (int i = 0; i < m.n; ++i)
        if (m.handle[i] == a.handle) return m.dev[i];
    return -1;
}

bool cpu_agent(hsa_agent_t a) {
    const AgentMap &m = agent_map();
    for (int i = 0; i < m.ncpu; ++i)
        if (m.cpu[i] == a.handle) return true;
    return false;
}

// Device memory (hipMalloc, stream-ordered pools, VMM mappings, IPC imports,
// managed) is combined in place; host memory (pageable or pinned) takes the
// host combine, the pinned slot or staging.  One HSA pointer query (24-66 ns
// against HIP's 100-165, profiles/r05/classify_cost.log) answers for memory HSA
// knows as a GPU's: allocations of its pools (HSA), its virtual-memory mappings
// (HSA_VMEM: stream-ordered pools, hipMemCreate + hipMemMap) and IPC imports
// (hsa_ext_amd.h:2344-2372).  Every other answer asks HIP: host pools
// (hipHostMalloc: pinned, whose owning device orders the caller's null-stream
// work before the read), RESERVED_ADDR, graphics interop -- and UNKNOWN, which
// is pageable memory, memory registered with hipHostRegister (HIP registers it
// without HSA's lock), but also managed memory (hipMallocManaged answers
// RESERVED_ADDR in a plain C process, UNKNOWN in a Python process that also
// loaded torch's bundled ROCm runtime: profiles/r05/classify_cost.log,
// classify_diag.log).  For host
// pages -- UNKNOWN, LOCKED, or an allocation owned by a CPU agent -- HIP's host
// verdicts (pageable, pinned) are kept per thread, keyed by the 4 KiB page: the
// next call on the same host buffers costs the HSA query and a lookup.  Only
// host verdicts are kept, and only looked up behind one of those answers, so a
// stale one never sends host memory to a kernel: a page that later becomes a GPU
// allocation answers HSA as the GPU's, and one that becomes managed memory is
// host-accessible (the host path reads it correctly); a device verdict is never
// reused.  What a stale host verdict can change is the host path's choice, since
// HSA reports pages pinned by hipHostRegister as UNKNOWN before and after: a
// page registered after its verdict was kept would be bounced like pageable
// memory instead of DMA'd.  So only calls that cannot reach the staged pipeline
// (`reuse`, verdict_reusable below: within both the mixed slot's and the host
// combine's limits, where pinned and pageable differ only in the null-stream
// ordering) take a kept verdict; a larger call asks HIP again and refreshes it.
// And because the page, not the buffer, keys the table (a registered buffer
// may share its first page with a pageable one classified earlier, or be
// registered after its verdict was kept: ADVICE r5), a call that took a kept
// host verdict (`*kept`) orders its host reads after the null stream whatever
// the verdict says -- the one thing pinned and pageable differ in there.
Loc classify(const void *p, int *dev, bool reuse = true, bool *kept = nullptr) {
    if (kept) *kept = false;
    if (!gpu_runtime_started()) return LOC_HOST;
    hsa_amd_pointer_info_t info;
    info.size = sizeof info;
    const bool known = hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS;
    if (known && (info.type == HSA_EXT_POINTER_TYPE_HSA || info.type == HSA_EXT_POINTER_TYPE_HSA_VMEM ||
                  info.type == HSA_EXT_POINTER_TYPE_IPC)) {
        const int d = agent_device(info.agentOwner);
        if (d >= 0) {
            *dev = d;
            return LOC_DEVICE;
        }
    }
    const bool host_page = known && (info.type == HSA_EXT_POINTER_TYPE_UNKNOWN ||
                                     info.type == HSA_EXT_POINTER_TYPE_LOCKED ||
                                     (info.type == HSA_EXT_POINTER_TYPE_HSA && cpu_agent(info.agentOwner)));
    if (!host_page) return classify_hip(p, dev);
    const uintptr_t page = reinterpret_cast<uintptr_t>(p) >> 12;
    HostVerdict &v = ctx().verdict[(page ^ (page >> 7)) & (kVerdicts - 1)];
    if (reuse && v.page == page) {
        *dev = v.dev;
        if (kept) *kept = true;
        return (Loc)v.loc;
    }
    const Loc l = classify_hip(p, dev);
    if (l != LOC_DEVICE) {
        v.page = page;
        v.loc = l;
        v.dev = l == LOC_PINNED ? *dev : 0;
    } else if (v.page == page) {
        v.page = ~(uintptr_t)0;
    }
    return l;
}

bool verdict_reusable(uint64_t bytes) { return bytes <= mixed_max_bytes() && bytes <= host_max_bytes(); }

// devices visible to this process (0 on a CPU-only rank: host operands are
// still combined there, as the reference's loop runs anywhere)
int device_count() {
    static const int n = [] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) { (void)hipGetLastError(); c = 0; }
        return c;
    }();
    return n;
}

// A pinned host operand may be the target of work the caller queued on the
// legacy null stream (a hipMemcpyAsync D2H, a kernel writing mapped memory):
// the host reads it only after that work, the ordering the device path keeps
// for device operands (direct_reduce) and the blocking library streams keep for
// staged ones.  hipStreamQuery(NULL) keeps answering "not ready" for finished
// work until the host synchronises (profiles/archive/r02/direct_probe.log), so "not
// ready" is followed by hipStreamSynchronize(NULL).  Pageable operands need
// nothing: HIP's copies into pageable memory complete before they return.
int order_after_null_stream() {
    if (hipStreamQuery(nullptr) == hipSuccess) return MPIR_HIP_OK;
    (void)hipGetLastError();
    HIPCHK(hipStreamSynchronize(nullptr));
    return MPIR_HIP_OK;
}

// the same for a pinned operand of device `dev`'s context, which the caller may
// have filled through that device's null stream while another was current
// (ADVICE r3): that device's null stream, then the caller's device back
int order_after_null_stream_of(int dev) {
    if (dev < 0) return order_after_null_stream();      // the caller's current device
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (dev == cur) return order_after_null_stream();
    HIPCHK(hipSetDevice(dev));
    const int rc = order_after_null_stream();
    (void)hipSetDevice(cur);
    return rc;
}

// Both operands in host memory: g_table's host loop (the kernels' functors
// compiled for x86) over n units of `unit` bytes, on the calling thread, or
// from host_split_bytes() split over a pool's threads (combine_pool: the
// operands' NUMA node) in parts on 64-byte boundaries.
int host_combine(int op, int elem, const void *inbuf, void *inoutbuf, uint64_t n, uint64_t unit) {
    const host_fn fn = g_table[op][elem].host;
    if (!fn) return MPIR_HIP_ENOKERNEL;
    if (n * unit < host_split_bytes() || pool_threads() <= 1) {
        fn(inbuf, inoutbuf, n);
        return MPIR_HIP_OK;
    }
    CopyPool &pool = combine_pool(inbuf, inoutbuf, (size_t)(n * unit));
    struct H {
        host_fn fn;
        const char *in;
        char *io;
        uint64_t n, part, unit;
    } h{fn, static_cast<const char *>(inbuf), static_cast<char *>(inoutbuf), n, 0, unit};
    // four parts per thread, handed out one at a time (a slower thread takes
    // fewer), of at least 256 KiB: a worker's wake-up costs a few us
    const uint64_t per = std::max<uint64_t>((n + 4 * (uint64_t)pool.threads() - 1) / (4 * (uint64_t)pool.threads()),
                                            ((uint64_t)256 << 10) / unit);
    const uint64_t grain = unit >= 64 ? 1 : 64 / unit;
    h.part = (per + grain - 1) / grain * grain;
    pool.run((size_t)((n + h.part - 1) / h.part), [](void *p, size_t k) {
        const H *h = static_cast<const H *>(p);
        const uint64_t b = k * h->part, e = std::min(h->n, b + h->part);
        h->fn(h->in + b * h->unit, h->io + b * h->unit, e - b);
    }, &h);
    return MPIR_HIP_OK;
}

// How the synchronous entry points wait for their launch.
//   MPIR_CVAR_REDUCE_LOCAL_WAIT=flag  (default): after the kernel, the stream
//       writes a per-thread sequence number into pinned host memory
//       (hipStreamWriteValue32, executed by the command processor in stream
//       order) and the caller spins on that word.  Measured on MI355X: an empty
//       launch + wait costs 7.2 us this way vs 11.5 us with
//       hipStreamSynchronize, 17.3 us polling hipStreamQuery (tools/latency.hip).
//   MPIR_CVAR_REDUCE_LOCAL_WAIT=block : hipStreamSynchronize.
// The spin re-checks hipStreamQuery every 64Ki polls so a faulted stream
// returns an error instead of spinning forever.
int wait_mode() {
    static const int mode = [] {
        const char *v = getenv("MPIR_CVAR_REDUCE_LOCAL_WAIT");
        return (v && !strcmp(v, "block")) ? 0 : 1;
    }();
    return mode;
}

int wait_stream_block(hipStream_t s) {
    HIPCHK(hipStreamSynchronize(s));
    return MPIR_HIP_OK;
}

int wait_stream(int dev, hipStream_t s) {
    if (wait_mode() == 0) return wait_stream_block(s);
    DevCtx &d = ctx().dev[dev];
    if (!d.flag) {
        void *p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            return wait_stream_block(s);
        }
        d.flag = static_cast<volatile uint32_t *>(p);
        *d.flag = 0;
    }
    const uint32_t seq = ++d.seq ? d.seq : ++d.seq;
    if (hipStreamWriteValue32(s, (void *)d.flag, seq, 0) != hipSuccess) {
        (void)hipGetLastError();
        return wait_stream_block(s);
    }
    for (uint64_t it = 1; *d.flag != seq; ++it) {
        if ((it & 0xFFFF) == 0) {
            hipError_t e = hipStreamQuery(s);
            if (e != hipSuccess && e != hipErrorNotReady) return set_err(e, "stream fault while waiting");
        }
        __builtin_ia32_pause();
    }
    return MPIR_HIP_OK;
}

// Both operands reachable by device `dev`'s kernels (device memory, or the
// pinned slot of the mixed path): direct AQL dispatch of plan_reduce's kernel
// for a synchronous call on the library stream (any count, any alignment) when
// nothing queued on the library stream is still pending; otherwise -- REPLACE,
// the 32-byte classes, the stream variant -- the HIP launch (then the wait,
// for a synchronous call).
int device_call(int dev, const void *inbuf, void *inoutbuf, uint64_t count, int op, int elem, hipStream_t user_s,
                int sync) {
    launch_fn fn = g_table[op][elem].fn;
    const size_t esz = g_elem_size[elem];
    // REPLACE is registered as a byte copy: its launcher counts bytes
    const uint64_t unit = (op == MPIR_HIP_OP_REPLACE) ? 1 : esz;
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != dev) HIPCHK(hipSetDevice(dev));
    hipStream_t s = user_s;
    int rc = MPIR_HIP_OK;
    DevCtx &d = ctx().dev[dev];
    if (sync && !s && g_table[op][elem].plan) {
        ReducePlan plan;
        g_table[op][elem].plan(inbuf, inoutbuf, count, &plan);
        bool idle = !d.main_pending;
        if (!idle && d.stream[S_MAIN] && hipStreamQuery(d.stream[S_MAIN]) == hipSuccess) {
            d.main_pending = false;
            idle = true;
        }
        (void)hipGetLastError();
        if (idle && direct_reduce(dev, op, elem, plan, &rc)) {
            if (rc != MPIR_HIP_OK) snprintf(ctx().err, sizeof(ctx().err), "direct dispatch: queue error");
            if (cur != dev) (void)hipSetDevice(cur);
            return rc;
        }
    }
    if (!s) rc = get_stream(dev, S_MAIN, &s);
    if (rc == MPIR_HIP_OK) {
        hipError_t e = fn(inbuf, inoutbuf, count * esz / unit, s);
        if (e != hipSuccess) rc = set_err(e, "kernel launch");
        else if (sync) rc = wait_stream(dev, s);
        else if (!user_s) d.main_pending = true;
    }
    if (cur != dev) (void)hipSetDevice(cur);
    return rc;
}

}  // namespace

extern "C" {

size_t MPIR_Hip_elem_size(int elem) {
    return (elem > 0 && elem < MPIR_HIP_NELEMS) ? g_elem_size[elem] : 0;
}

int MPIR_Hip_has_kernel(int op, int elem) {
    if (op <= 0 || op >= MPIR_HIP_NOPS || elem <= 0 || elem >= MPIR_HIP_NELEMS) return 0;
    return g_table[op][elem].fn != nullptr;
}

const char *MPIR_Hip_error_string(void) { return ctx().err; }

uint64_t MPIR_Hip_host_max_bytes(void) { return host_max_bytes(); }

uint64_t MPIR_Hip_set_host_max_bytes(uint64_t bytes) { return g_host_max.exchange(bytes); }

uint64_t MPIR_Hip_set_keep_bytes(uint64_t bytes) { return mpir_hip::g_keep.exchange(bytes); }

uint64_t MPIR_Hip_set_keep_min_bytes(uint64_t bytes) { return mpir_hip::g_keep_min.exchange(bytes); }

uint64_t MPIR_Hip_mixed_max_bytes(void) { return mixed_max_bytes(); }

uint64_t MPIR_Hip_direct_dispatches(void) { return direct_calls(); }

void MPIR_Hip_direct_profile(int on) { direct_profile(on); }

uint64_t MPIR_Hip_direct_last_kernel_ns(void) { return direct_last_kernel_ns(); }

int MPIR_Hip_direct_state(int dev) { return direct_state(dev); }

int MPIR_Hip_direct_prepare(int dev) { return direct_prepare(dev); }

void MPIR_Hip_direct_last_split(uint64_t out[4]) { direct_last_split(out); }

uint64_t MPIR_Hip_direct_busy_skips(void) { return direct_busy_skips(); }

uint64_t MPIR_Hip_direct_kernarg_writes(void) { return direct_kernarg_writes(); }
uint32_t MPIR_Hip_direct_test_write_delay_us(uint32_t us) { return direct_test_write_delay_us(us); }
void MPIR_Hip_direct_test_fail_probe(void) { direct_test_fail_probe(); }
void MPIR_Hip_direct_placement(int dev, int out[5]) { direct_placement(dev, out); }

int MPIR_Hip_set_local_ranks(int n) {
    return g_local_ranks.exchange(n > 0 ? n : 0);
}

int MPIR_Hip_host_threads(void) { return pool_threads(); }

int MPIR_Hip_combine_set_flags(int flags) {
    const int prev = mpir_hip::t_combine_flags;
    mpir_hip::t_combine_flags = flags & MPIR_HIP_COMBINE_UNCAPPED;
    return prev;
}

int MPIR_Hip_thread_contexts(void) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    return g_ctx_created;
}

int MPIR_Hip_device_count(void) { return device_count(); }

int MPIR_Hip_pointer_kind(const void *p, uint64_t bytes) {
    int dev = 0;
    return classify(p, &dev, verdict_reusable(bytes));
}

int MPIR_Hip_is_device_ptr(const void *p) {
    int dev = 0;
    return classify(p, &dev) == LOC_DEVICE;
}

int MPIR_Hip_memcpy(void *dst, const void *src, size_t bytes) {
    if (!bytes) return MPIR_HIP_OK;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    return MPIR_HIP_OK;
}

int MPIR_Hip_combine(const void *const *inbufs, int n, void *outbuf, uint64_t count, int op, int elem,
                     int order, void *hip_stream, int sync) {
    ctx().err[0] = 0;
    if (n < 1 || n > 64 || (order != MPIR_HIP_ORDER_TREE && order != MPIR_HIP_ORDER_CHAIN)) return MPIR_HIP_ENOKERNEL;
    if (op <= 0 || op >= MPIR_HIP_NOPS || elem <= 0 || elem >= MPIR_HIP_NELEMS) return MPIR_HIP_ENOKERNEL;
    if (order == MPIR_HIP_ORDER_TREE && (n & (n - 1))) return MPIR_HIP_ENOKERNEL;
    const size_t esz = g_elem_size[elem];
    int dev = -1;
    if (classify(outbuf, &dev) != LOC_DEVICE) return MPIR_HIP_EBUFFER;
    for (int j = 0; j < n; ++j) {
        int d = -1;
        if (classify(inbufs[j], &d) != LOC_DEVICE || d != dev) return MPIR_HIP_EBUFFER;
    }
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != dev) HIPCHK(hipSetDevice(dev));
    hipStream_t s = (hipStream_t)hip_stream;
    int rc = MPIR_HIP_OK;
    if (!s) rc = get_stream(dev, S_MAIN, &s);
    hipError_t e = hipSuccess;
    if (rc == MPIR_HIP_OK && count > 0) {
        const bool fused = g_multi[op][elem][0][0] != nullptr;
        if (n == 1) {
            if (outbuf != inbufs[0]) e = hipMemcpyAsync(outbuf, inbufs[0], count * esz, hipMemcpyDeviceToDevice, s);
        } else if (op == MPIR_HIP_OP_REPLACE) {
            // a fold of REPLACE in either order is the last operand
            if (outbuf != inbufs[n - 1])
                e = hipMemcpyAsync(outbuf, inbufs[n - 1], count * esz, hipMemcpyDeviceToDevice, s);
        } else if (order == MPIR_HIP_ORDER_TREE && fused && n <= 8) {
            e = g_multi[op][elem][0][n - 2](inbufs, outbuf, count, s);
        } else if (order == MPIR_HIP_ORDER_CHAIN && fused) {
            // CHAIN: acc = y0; fold y1..y_{n-1} in order, one pass for n <= 8;
            // beyond, chunks of up to 8 operands, each chunk's first operand the
            // running acc
            const void *acc = inbufs[0];
            int i = 1;
            while (e == hipSuccess && i < n) {
                const int P = std::min(kMultiMaxP, n - i + 1);
                const void *ops[kMultiMaxP];
                ops[0] = acc;
                for (int j = 1; j < P; ++j) ops[j] = inbufs[i + j - 1];
                e = g_multi[op][elem][1][P - 2](ops, outbuf, count, s);
                i += P - 1;
                acc = outbuf;
            }
        } else if (g_table[op][elem].any) {
            // one pass, no temporaries (k_combine_any)
            e = g_table[op][elem].any(inbufs, n, order == MPIR_HIP_ORDER_TREE, outbuf, count, s);
        } else {
            rc = MPIR_HIP_ENOKERNEL;
        }
        if (e != hipSuccess) rc = set_err(e, "combine launch");
        if (rc == MPIR_HIP_OK && sync) rc = wait_stream(dev, s);
    }
    if (cur != dev) (void)hipSetDevice(cur);
    return rc;
}

int MPIR_Hip_reduce(const void *inbuf, void *inoutbuf, uint64_t count, int op, int elem, void *hip_stream,
                    int sync) {
    if (!MPIR_Hip_has_kernel(op, elem)) return MPIR_HIP_ENOKERNEL;
    if (count == 0) return MPIR_HIP_OK;
    const size_t esz = g_elem_size[elem];
    // REPLACE is registered as a byte copy: its launcher counts bytes
    const uint64_t unit = (op == MPIR_HIP_OP_REPLACE) ? 1 : esz;

    // ---- no GPU runtime in this process: both operands are pageable host
    // ---- memory, combined here with no HIP call (the reference's loop,
    // ---- opsum.c:21-76, touches no device either)
    if (!gpu_runtime_started() && count * esz <= host_max_bytes()) {
        if (!sync) return MPIR_HIP_EBUFFER;
        return host_combine(op, elem, inbuf, inoutbuf, count * esz / unit, unit);
    }

    ctx().err[0] = 0;
    launch_fn fn = g_table[op][elem].fn;
    int din = -1, dio = -1;
    bool kin = false, kio = false;
    const bool reuse = verdict_reusable(count * esz);
    const Loc lin = classify(inbuf, &din, reuse, &kin);
    const Loc lio = classify(inoutbuf, &dio, reuse, &kio);
    // a host operand the host reads below waits for the null stream if it is
    // pinned, or if its verdict was a kept one (classify: it may be stale)
    const bool order_in = lin == LOC_PINNED || (lin == LOC_HOST && kin);
    const bool order_io = lio == LOC_PINNED || (lio == LOC_HOST && kio);
    // the device whose null stream that is: the pinned buffer's, else the caller's
    const int odin = lin == LOC_PINNED ? din : -1, odio = lio == LOC_PINNED ? dio : -1;

    // ---- fast path: both operands device-resident on one device ----------
    if (lin == LOC_DEVICE && lio == LOC_DEVICE && din == dio)
        return device_call(dio, inbuf, inoutbuf, count, op, elem, (hipStream_t)hip_stream, sync);
    if (!sync) return MPIR_HIP_EBUFFER;  // the stream variant needs device buffers

    // ---- both host-resident: combine on the host (no device needed) ------
    if (lin != LOC_DEVICE && lio != LOC_DEVICE && (count * esz <= host_max_bytes() || device_count() == 0) &&
        g_table[op][elem].host) {
        int rc = MPIR_HIP_OK;
        if (order_in) rc = order_after_null_stream_of(odin);
        if (rc == MPIR_HIP_OK && order_io && !(order_in && odin == odio)) rc = order_after_null_stream_of(odio);
        if (rc != MPIR_HIP_OK) return rc;
        return host_combine(op, elem, inbuf, inoutbuf, count * esz / unit, unit);
    }

    // ---- small, one operand host memory and the other on a device: the host
    // ---- operand goes through the thread's pinned slot, which the kernel
    // ---- reads (writes) directly; the slot copy keeps the device operand's
    // ---- offset mod 256 so the aligned tile kernels still apply
    if ((lin == LOC_DEVICE) != (lio == LOC_DEVICE) && count * esz <= mixed_max_bytes()) {
        const uint64_t bytes = count * esz;
        const int dev = lin == LOC_DEVICE ? din : dio;
        const uintptr_t adev = reinterpret_cast<uintptr_t>(lin == LOC_DEVICE ? inbuf : (const void *)inoutbuf);
        char *slot = nullptr;
        int rc = MPIR_HIP_OK;
        if (lin == LOC_DEVICE ? order_io : order_in) {
            // the host operand is read (copied into the slot) before device_call's
            // own null-stream check: order it first, after the null stream of the
            // device that owns the pinned buffer (the caller's for a
            // kept pageable verdict) and of the device the kernel runs on
            const int pdev = lin == LOC_DEVICE ? odio : odin;
            rc = order_after_null_stream_of(pdev);
            if (rc == MPIR_HIP_OK && pdev >= 0 && pdev != dev) rc = order_after_null_stream_of(dev);
            if (rc != MPIR_HIP_OK) return rc;
        }
        rc = get_zc(dev, (size_t)bytes + 256, &slot);
        if (rc != MPIR_HIP_OK) return rc;
        slot += adev & 255;
        // host <-> slot copies: split over the copy pool from zc_split_bytes() up
        auto hcopy = [&](void *dst, const void *src) {
            if (bytes >= zc_split_bytes())
                copy_pool().copy(static_cast<char *>(dst), static_cast<const char *>(src), bytes, zc_split_bytes());
            else
                memcpy(dst, src, bytes);
        };
        if (lio == LOC_DEVICE) {
            hcopy(slot, inbuf);
            return device_call(dev, slot, inoutbuf, count, op, elem, nullptr, 1);
        }
        hcopy(slot, inoutbuf);
        rc = device_call(dev, inbuf, slot, count, op, elem, nullptr, 1);
        if (rc == MPIR_HIP_OK) hcopy(inoutbuf, slot);
        return rc;
    }

    // ---- staged path: at least one operand is host memory (or the two ----
    // ---- operands live on different devices): the up / comp / down      ----
    // ---- pipeline described at stage_chunk().                            ----
    int dev = 0;
    if (lio == LOC_DEVICE) dev = dio;
    else if (lin == LOC_DEVICE) dev = din;
    else {
        if (device_count() == 0) return MPIR_HIP_ENODEV;
        HIPCHK(hipGetDevice(&dev));
    }
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != dev) HIPCHK(hipSetDevice(dev));

    int rc = MPIR_HIP_OK;
    DevCtx &d = ctx().dev[dev];
    const bool stage_in = !(lin == LOC_DEVICE && din == dev);
    const bool stage_io = !(lio == LOC_DEVICE && dio == dev);
    const uint64_t total = count * esz;
    uint64_t chunk_elems = stage_chunk() / esz;
    if (chunk_elems > count) chunk_elems = count;
    const uint64_t chunk_bytes = chunk_elems * esz;
    const uint64_t slot_bytes = (chunk_bytes + 255) & ~(uint64_t)255;
    const int nslots = stage_slots();
    char *scratch = nullptr;
    hipStream_t up = nullptr, comp = nullptr, down = nullptr;
    rc = get_scratch(dev, (size_t)(2 * nslots) * slot_bytes, &scratch);
    if (rc == MPIR_HIP_OK) rc = get_stream(dev, S_UP, &up);
    if (rc == MPIR_HIP_OK) rc = get_stream(dev, S_COMP, &comp);
    if (rc == MPIR_HIP_OK) rc = get_stream(dev, S_DOWN, &down);
    if (rc == MPIR_HIP_OK) rc = get_stage_events(dev, nslots);
    const char *cin = static_cast<const char *>(inbuf);
    char *cio = static_cast<char *>(inoutbuf);
    // Pageable host operands go through pinned bounce slots that the copy pool
    // fills and drains while the GPU works on earlier chunks (HIP's own
    // pageable path uploads ~36 GB/s; pinned memory is DMA'd directly).
    const bool bounce_in = stage_in && lin == LOC_HOST;
    const bool bounce_io = stage_io && lio == LOC_HOST;
    char *bounce = nullptr;
    if (rc == MPIR_HIP_OK && (bounce_in || bounce_io))
        rc = get_bounce(dev, (size_t)(2 * nslots) * slot_bytes, &bounce);
    CopyPool *pool = (bounce_in || bounce_io) ? &copy_pool() : nullptr;   // threads only when needed
    const uint64_t nchunks = (total + chunk_bytes - 1) / chunk_bytes;
    // chunk j's result: from its bounce slot to the caller's inoutbuf, once its
    // copy-back (recorded as ev_free of its slot) has landed
    auto drain = [&](uint64_t j) -> int {
        const int sl = (int)(j % (uint64_t)nslots);
        const uint64_t o = j * chunk_bytes, n = (total - o < chunk_bytes) ? total - o : chunk_bytes;
        hipError_t e = hipEventSynchronize(d.ev_free[sl]);
        if (e != hipSuccess) return set_err(e, "staged reduce");
        pool->copy(cio + o, bounce + (2 * sl + 1) * slot_bytes, n);
        return MPIR_HIP_OK;
    };
    for (uint64_t off = 0, k = 0; rc == MPIR_HIP_OK && off < total; off += chunk_bytes, ++k) {
        const uint64_t nb = (total - off < chunk_bytes) ? total - off : chunk_bytes;
        const int slot = (int)(k % (uint64_t)nslots);
        char *sin = scratch + (2 * slot) * slot_bytes;
        char *sio = scratch + (2 * slot + 1) * slot_bytes;
        char *bin = bounce ? bounce + (2 * slot) * slot_bytes : nullptr;
        char *bio = bounce ? bounce + (2 * slot + 1) * slot_bytes : nullptr;
        const void *kin = stage_in ? (const void *)sin : (const void *)(cin + off);
        void *kio = stage_io ? (void *)sio : (void *)(cio + off);
        hipError_t e = hipSuccess;
        // the slot's previous chunk must be fully consumed (kernel read, copy-back done)
        if (k >= (uint64_t)nslots) {
            if (bounce_io) {
                if ((rc = drain(k - nslots)) != MPIR_HIP_OK) break;
            } else if (bounce_in) {
                e = hipEventSynchronize(d.ev_free[slot]);   // the host rewrites bin
            }
            if (e == hipSuccess) e = hipStreamWaitEvent(up, d.ev_free[slot], 0);
        }
        if (e == hipSuccess && bounce_in) pool->copy(bin, cin + off, nb);
        if (e == hipSuccess && bounce_io) pool->copy(bio, cio + off, nb);
        if (e == hipSuccess && stage_in)
            e = hipMemcpyAsync(sin, bounce_in ? (const void *)bin : (const void *)(cin + off), nb, hipMemcpyDefault, up);
        if (e == hipSuccess && stage_io)
            e = hipMemcpyAsync(sio, bounce_io ? (const void *)bio : (const void *)(cio + off), nb, hipMemcpyDefault, up);
        if (e == hipSuccess) e = hipEventRecord(d.ev_up[slot], up);
        if (e == hipSuccess) e = hipStreamWaitEvent(comp, d.ev_up[slot], 0);
        if (e == hipSuccess) e = fn(kin, kio, nb / unit, comp);
        if (e == hipSuccess) e = hipEventRecord(d.ev_comp[slot], comp);
        if (stage_io) {
            if (e == hipSuccess) e = hipStreamWaitEvent(down, d.ev_comp[slot], 0);
            if (e == hipSuccess) e = hipMemcpyAsync(bounce_io ? (void *)bio : (void *)(cio + off), sio, nb, hipMemcpyDefault, down);
            if (e == hipSuccess) e = hipEventRecord(d.ev_free[slot], down);
        } else if (e == hipSuccess) {
            e = hipEventRecord(d.ev_free[slot], comp);
        }
        if (e != hipSuccess) rc = set_err(e, "staged reduce");
    }
    if (rc == MPIR_HIP_OK && bounce_io)
        for (uint64_t j = nchunks > (uint64_t)nslots ? nchunks - nslots : 0; rc == MPIR_HIP_OK && j < nchunks; ++j)
            rc = drain(j);
    if (rc == MPIR_HIP_OK) rc = wait_stream_block(comp);
    if (rc == MPIR_HIP_OK) rc = wait_stream_block(down);
    if (cur != dev) (void)hipSetDevice(cur);
    return rc;
}

}  // extern "C"
