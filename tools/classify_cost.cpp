// classify_cost.cpp -- what the HSA runtime's hsa_amd_pointer_info reports for
// every kind of buffer a caller can hand MPI_Reduce_local, next to HIP's
// hipPointerGetAttributes (type, device), and what one query of each costs
// once HIP is up.
//
//   hipcc -O2 -std=c++17 tools/classify_cost.cpp -o tools/classify_cost -lhsa-runtime64
//   tools/classify_cost
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e9 + ts.tv_nsec;
}

static const char *agent_kind(hsa_agent_t a) {
    if (!a.handle) return "none";
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return "?";
    return t == HSA_DEVICE_TYPE_GPU ? "gpu" : (t == HSA_DEVICE_TYPE_CPU ? "cpu" : "other");
}

int main() {
    const size_t MB = 1 << 20;
    void *dev = nullptr, *pin = nullptr, *man = nullptr, *pool = nullptr, *coh = nullptr;
    if (hipMalloc(&dev, MB) != hipSuccess || hipHostMalloc(&pin, MB, 0) != hipSuccess) return 1;
    if (hipMallocManaged(&man, MB) != hipSuccess) man = nullptr;
    if (hipHostMalloc(&coh, MB, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) coh = nullptr;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    if (hipMallocAsync(&pool, MB, s) != hipSuccess) pool = nullptr;
    (void)hipStreamSynchronize(s);
    void *page = malloc(MB);
    memset(page, 0, MB);
    void *reg = aligned_alloc(4096, MB);
    memset(reg, 0, MB);
    if (hipHostRegister(reg, MB, hipHostRegisterDefault) != hipSuccess) reg = nullptr;
    // VMM: physical allocation on device 0 mapped into a reserved range
    void *vmm = nullptr;
    {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        size_t gran = 0;
        hipMemGenericAllocationHandle_t h;
        if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) == hipSuccess) {
            const size_t sz = ((MB + gran - 1) / gran) * gran;
            if (hipMemCreate(&h, sz, &prop, 0) == hipSuccess && hipMemAddressReserve(&vmm, sz, 0, nullptr, 0) == hipSuccess &&
                hipMemMap(vmm, sz, 0, h, 0) == hipSuccess) {
                hipMemAccessDesc acc = {};
                acc.location = prop.location;
                acc.flags = hipMemAccessFlagsProtReadWrite;
                if (hipMemSetAccess(vmm, sz, &acc, 1) != hipSuccess) vmm = nullptr;
            } else {
                vmm = nullptr;
            }
        }
    }
    (void)hipGetLastError();
    struct K { const char *name; void *p; } ks[] = {{"hipMalloc", dev},        {"hipHostMalloc", pin},
                                                     {"hipHostMalloc coh+map", coh}, {"hipMallocManaged", man},
                                                     {"hipMallocAsync", pool},  {"hipHostRegister", reg},
                                                     {"VMM hipMemMap", vmm},    {"malloc (pageable)", page}};
    const int N = 200000;
    for (const K &k : ks) {
        if (!k.p) {
            printf("%-22s (allocation failed)\n", k.name);
            continue;
        }
        hipPointerAttribute_t at;
        memset(&at, 0, sizeof at);
        const hipError_t he = hipPointerGetAttributes(&at, (char *)k.p + 64);
        (void)hipGetLastError();
        hsa_amd_pointer_info_t info;
        memset(&info, 0, sizeof info);
        info.size = sizeof info;
        const hsa_status_t hs = hsa_amd_pointer_info((char *)k.p + 64, &info, nullptr, nullptr, nullptr);
        for (int i = 0; i < 1000; ++i) {
            (void)hipPointerGetAttributes(&at, k.p);
            (void)hipGetLastError();
        }
        double t0 = now_ns();
        for (int i = 0; i < N; ++i) {
            (void)hipPointerGetAttributes(&at, (char *)k.p + (i & 1023));
            (void)hipGetLastError();
        }
        double t1 = now_ns();
        hsa_amd_pointer_info_t inf2;
        for (int i = 0; i < N; ++i) {
            inf2.size = sizeof inf2;
            (void)hsa_amd_pointer_info((char *)k.p + (i & 1023), &inf2, nullptr, nullptr, nullptr);
        }
        double t2 = now_ns();
        printf("%-22s hip: err %d type %d device %2d | hsa: status %d type %d owner %-4s flags 0x%x registered %d "
               "base_ok %d | hip %6.1f ns  hsa %6.1f ns\n",
               k.name, (int)he, (int)at.type, at.device, (int)hs, (int)info.type, agent_kind(info.agentOwner),
               info.global_flags, (int)info.registered,
               (char *)info.agentBaseAddress <= (char *)k.p && (char *)k.p < (char *)info.agentBaseAddress + info.sizeInBytes,
               (t1 - t0) / N, (t2 - t1) / N);
    }
    // hipMallocManaged at several sizes: HSA's answer at the base and inside
    const size_t msz[4] = {MB, MB + 12, 64 * MB, 4096};
    for (size_t sz : msz) {
        void *m = nullptr;
        if (hipMallocManaged(&m, sz) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        int types[2];
        for (int i = 0; i < 2; ++i) {
            hsa_amd_pointer_info_t info;
            memset(&info, 0, sizeof info);
            info.size = sizeof info;
            (void)hsa_amd_pointer_info((char *)m + (i ? sz / 2 : 0), &info, nullptr, nullptr, nullptr);
            types[i] = (int)info.type;
        }
        printf("hipMallocManaged %9zu B: hsa type at base %d, mid %d\n", sz, types[0], types[1]);
        (void)hipFree(m);
    }
    return 0;
}
