// aql_ab.cpp -- A/B of the synchronous-call overhead: HIP launch + completion
// word (the product's MPI_Reduce_local wait) against a direct AQL dispatch on
// a queue of our own with a completion signal polled by the host.
//   see tools/aql/build.sh; run: tools/aql/aql_ab tools/aql/aql_kernels.co
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mpi_reduce_local.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char *m_; hsa_status_string(s_, &m_); printf("HSA %s line %d: %s\n", #x, __LINE__, m_); exit(3);} } while (0)

__global__ void hip_empty() {}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct TileArgsF {       // mirrors mpir_hip::TileArgs<float> (72 bytes)
    const char *in; char *io; uint64_t vbytes;
    const float *head_in; float *head_io; uint32_t nhead;
    const float *tail_in; float *tail_io; uint32_t ntail;
};
static_assert(sizeof(TileArgsF) == 72, "kernarg layout");

static hsa_agent_t g_gpu;
static uint32_t g_bdf;
static hsa_region_t g_kernarg;

static hsa_status_t find_gpu(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
    uint32_t bdf = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    if (bdf == g_bdf) { g_gpu = a; return HSA_STATUS_INFO_BREAK; }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg(hsa_region_t r, void *) {
    hsa_region_segment_t seg;
    hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg);
    if (seg != HSA_REGION_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    hsa_region_global_flag_t f;
    hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &f);
    if (f & HSA_REGION_GLOBAL_FLAG_KERNARG) { g_kernarg = r; return HSA_STATUS_INFO_BREAK; }
    return HSA_STATUS_SUCCESS;
}

struct Aql {
    hsa_queue_t *q;
    hsa_signal_t sig;
    void *karg;
    uint64_t ko_empty, ko_tile;
    uint16_t acq, rel;
    void dispatch(uint64_t ko, uint32_t groups, const void *args, size_t nargs) {
        if (nargs) memcpy(karg, args, nargs);
        hsa_signal_store_relaxed(sig, 1);
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {}
        hsa_kernel_dispatch_packet_t *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
        memset((char *)p + 4, 0, sizeof(*p) - 4);
        p->workgroup_size_x = 256; p->workgroup_size_y = 1; p->workgroup_size_z = 1;
        p->grid_size_x = groups * 256; p->grid_size_y = 1; p->grid_size_z = 1;
        p->kernel_object = ko;
        p->kernarg_address = karg;
        p->private_segment_size = 0;
        p->group_segment_size = 0;
        p->completion_signal = sig;
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (1 << HSA_PACKET_HEADER_BARRIER) |
                                (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, idx);
    }
    void wait() {
        while (hsa_signal_load_scacquire(sig) != 0) __builtin_ia32_pause();
    }
};

int main(int argc, char **argv) {
    if (argc < 2) { printf("usage: aql_ab code_object\n"); return 1; }
    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);
    CK(hipSetDevice(0));
    int bus = 0, devn = 0, dom = 0;
    CK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
    CK(hipDeviceGetAttribute(&devn, hipDeviceAttributePciDeviceId, 0));
    CK(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, 0));
    g_bdf = ((uint32_t)bus << 8) | ((uint32_t)devn << 3);
    HK(hsa_init());
    hsa_status_t st = hsa_iterate_agents(find_gpu, nullptr);
    if (st != HSA_STATUS_INFO_BREAK) { printf("no HSA agent with bdf %x\n", g_bdf); return 4; }
    st = hsa_agent_iterate_regions(g_gpu, find_kernarg, nullptr);
    if (st != HSA_STATUS_INFO_BREAK) { printf("no kernarg region\n"); return 4; }

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
    Aql aq{};
    hsa_executable_symbol_t sym;
    uint32_t kas = 0;
    HK(hsa_executable_get_symbol_by_name(exe, "aql_empty.kd", &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &aq.ko_empty));
    HK(hsa_executable_get_symbol_by_name(exe, "aql_tile_sum_f32.kd", &g_gpu, &sym));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &aq.ko_tile));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kas));
    printf("tile kernarg segment %u bytes\n", kas);
    if (kas != sizeof(TileArgsF)) { printf("kernarg size mismatch\n"); return 5; }
    HK(hsa_memory_allocate(g_kernarg, 256, &aq.karg));
    HK(hsa_queue_create(g_gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &aq.q));
    HK(hsa_signal_create(1, 0, nullptr, &aq.sig));
    aq.acq = HSA_FENCE_SCOPE_SYSTEM; aq.rel = HSA_FENCE_SCOPE_SYSTEM;

    // ---- correctness on a ragged count: AQL tile == product MPI_Reduce_local
    {
        const size_t n = (1 << 20) + 4;  // multiple of 4 floats: no head/tail
        float *a, *b, *c;
        CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&c, n * 4));
        std::vector<float> ha(n), hb(n);
        for (size_t i = 0; i < n; ++i) { ha[i] = (float)((i * 2654435761u) % 1000) * 0.001f - 0.5f; hb[i] = (float)((i * 40503u) % 777) * 0.01f; }
        CK(hipMemcpy(a, ha.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(c, ha.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(b, hb.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        if (MPI_Reduce_local(b, a, (int)n, MPI_FLOAT, MPI_SUM)) { printf("product call failed\n"); return 6; }
        TileArgsF ta{(const char *)b, (char *)c, n * 4, b, c, 0, b + n, c + n, 0};
        aq.dispatch(aq.ko_tile, (uint32_t)((n * 4 + 16383) / 16384), &ta, sizeof ta);
        aq.wait();
        std::vector<float> ra(n), rc(n);
        CK(hipMemcpy(ra.data(), a, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(rc.data(), c, n * 4, hipMemcpyDeviceToHost));
        printf("AQL tile vs MPI_Reduce_local: %s\n", memcmp(ra.data(), rc.data(), n * 4) ? "MISMATCH" : "bit-identical");
        CK(hipFree(a)); CK(hipFree(b)); CK(hipFree(c));
    }

    // ---- empty-kernel round trips
    hipStream_t sb, snb;
    CK(hipStreamCreate(&sb));
    CK(hipStreamCreateWithFlags(&snb, hipStreamNonBlocking));
    volatile unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    unsigned seq = 0;
    const int K = 2000, R = 5;
    auto hip_flag = [&](hipStream_t s) {
        hipLaunchKernelGGL(hip_empty, 1, 256, 0, s);
        CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
        while (*flag != seq) __builtin_ia32_pause();
    };
    for (int i = 0; i < 100; ++i) { hip_flag(sb); hip_flag(snb); aq.dispatch(aq.ko_empty, 1, nullptr, 0); aq.wait(); }
    for (int r = 0; r < R; ++r) {
        double t0 = now();
        for (int i = 0; i < K; ++i) hip_flag(sb);
        double t1 = now();
        for (int i = 0; i < K; ++i) hip_flag(snb);
        double t2 = now();
        aq.acq = HSA_FENCE_SCOPE_SYSTEM; aq.rel = HSA_FENCE_SCOPE_SYSTEM;
        for (int i = 0; i < K; ++i) { aq.dispatch(aq.ko_empty, 1, nullptr, 0); aq.wait(); }
        double t3 = now();
        aq.acq = HSA_FENCE_SCOPE_AGENT; aq.rel = HSA_FENCE_SCOPE_SYSTEM;
        for (int i = 0; i < K; ++i) { aq.dispatch(aq.ko_empty, 1, nullptr, 0); aq.wait(); }
        double t4 = now();
        aq.acq = HSA_FENCE_SCOPE_AGENT; aq.rel = HSA_FENCE_SCOPE_AGENT;
        for (int i = 0; i < K; ++i) { aq.dispatch(aq.ko_empty, 1, nullptr, 0); aq.wait(); }
        double t5 = now();
        printf("empty round trip us: hip+flag blocking %.2f | hip+flag nonblocking %.2f | aql sys/sys %.2f | aql agent/sys %.2f | aql agent/agent %.2f\n",
               (t1 - t0) / K * 1e6, (t2 - t1) / K * 1e6, (t3 - t2) / K * 1e6, (t4 - t3) / K * 1e6, (t5 - t4) / K * 1e6);
    }
    aq.acq = HSA_FENCE_SCOPE_SYSTEM; aq.rel = HSA_FENCE_SCOPE_SYSTEM;

    // ---- 256 MiB fp32 SUM, 4 rotating pairs: product sync call vs AQL + signal
    const size_t n = 64ull << 20;
    const int NP = 4;
    float *pa[NP], *pb[NP];
    for (int j = 0; j < NP; ++j) {
        CK(hipMalloc(&pa[j], n * 4)); CK(hipMalloc(&pb[j], n * 4));
        CK(hipMemset(pa[j], 0, n * 4)); CK(hipMemset(pb[j], 0x3c, n * 4));
    }
    CK(hipDeviceSynchronize());
    const int KS = 50;
    for (int r = 0; r < R; ++r) {
        for (int i = 0; i < 5; ++i) MPI_Reduce_local(pb[i % NP], pa[i % NP], (int)n, MPI_FLOAT, MPI_SUM);
        double t0 = now();
        for (int i = 0; i < KS; ++i) MPI_Reduce_local(pb[i % NP], pa[i % NP], (int)n, MPI_FLOAT, MPI_SUM);
        double t1 = now();
        for (int i = 0; i < 5; ++i) {
            TileArgsF ta{(const char *)pb[i % NP], (char *)pa[i % NP], n * 4, pb[0], pa[0], 0, pb[0], pa[0], 0};
            aq.dispatch(aq.ko_tile, (uint32_t)(n * 4 / 16384), &ta, sizeof ta);
            aq.wait();
        }
        double t2 = now();
        for (int i = 0; i < KS; ++i) {
            TileArgsF ta{(const char *)pb[i % NP], (char *)pa[i % NP], n * 4, pb[0], pa[0], 0, pb[0], pa[0], 0};
            aq.dispatch(aq.ko_tile, (uint32_t)(n * 4 / 16384), &ta, sizeof ta);
            aq.wait();
        }
        double t3 = now();
        const double us0 = (t1 - t0) / KS * 1e6, us1 = (t3 - t2) / KS * 1e6;
        printf("256 MiB sync call us: MPI_Reduce_local %.2f (%.4f of 8 TB/s) | aql+signal %.2f (%.4f)\n",
               us0, 805306368.0 / (us0 * 1e-6) / 8e12, us1, 805306368.0 / (us1 * 1e-6) / 8e12);
    }
    hsa_queue_destroy(aq.q);
    hsa_signal_destroy(aq.sig);
    hsa_executable_destroy(exe);
    hsa_code_object_reader_destroy(rd);
    return 0;
}
