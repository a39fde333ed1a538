// ptrinfo_probe.hip -- what classifying a pointer costs, and what each query answers, for the memory
// kinds an MPI program hands ompi_op_reduce: hipPointerGetAttributes (what mi355x_ptr_is_device
// asks today) vs ROCr's hsa_amd_pointer_info, on heap, private / shared anonymous mappings,
// hipMalloc, hipHostMalloc, hipMallocManaged and VMM-mapped device memory (hipMemCreate +
// hipMemMap, PyTorch's expandable segments).  One JSON line per (kind, query): ns per call and the
// answer (HIP memory type / HSA pointer type).  (measurement tool, not part of the product)
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double ns_per(void (*f)(void *), void *p, int reps)
{
    std::vector<double> t;
    for (int k = 0; k < 7; ++k) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r) f(p);
        t.push_back(std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / reps);
    }
    std::sort(t.begin(), t.end());
    return t[3];
}

static volatile int sink;
static void q_hip(void *p)
{
    hipPointerAttribute_t a;
    std::memset(&a, 0, sizeof(a));
    if (hipPointerGetAttributes(&a, p) != hipSuccess) (void)hipGetLastError();
    sink = a.type;
}
static void q_hsa(void *p)
{
    hsa_amd_pointer_info_t i;
    std::memset(&i, 0, sizeof(i));
    i.size = sizeof(i);
    (void)hsa_amd_pointer_info(p, &i, nullptr, nullptr, nullptr);
    sink = i.type;
}

int main()
{
    if (hipSetDevice(0) != hipSuccess) return 1;
    (void)hipFree(nullptr);
    struct Kind {
        const char *name;
        void *p;
    };
    std::vector<Kind> kinds;
    kinds.push_back({"heap", std::malloc(4096)});
    kinds.push_back({"mmap_private", mmap(nullptr, 1 << 20, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0)});
    kinds.push_back({"mmap_shared", mmap(nullptr, 1 << 20, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0)});
    void *d = nullptr, *h = nullptr, *m = nullptr;
    if (hipMalloc(&d, 1 << 20) == hipSuccess) kinds.push_back({"hipMalloc", (char *)d + 4096});
    if (hipHostMalloc(&h, 1 << 20, 0) == hipSuccess) kinds.push_back({"hipHostMalloc", (char *)h + 4096});
    if (hipMallocManaged(&m, 1 << 20) == hipSuccess) kinds.push_back({"hipMallocManaged", (char *)m + 4096});
    // VMM: a physical allocation mapped into a reserved range
    hipMemAllocationProp prop;
    std::memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    void *va = nullptr;
    hipMemGenericAllocationHandle_t hd;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) == hipSuccess &&
        hipMemCreate(&hd, gran, &prop, 0) == hipSuccess && hipMemAddressReserve(&va, gran, 0, nullptr, 0) == hipSuccess &&
        hipMemMap(va, gran, 0, hd, 0) == hipSuccess) {
        hipMemAccessDesc acc;
        std::memset(&acc, 0, sizeof(acc));
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        if (hipMemSetAccess(va, gran, &acc, 1) == hipSuccess) kinds.push_back({"vmm_device", (char *)va + 256});
    } else {
        (void)hipGetLastError();
    }
    for (const Kind &k : kinds) {
        hipPointerAttribute_t a;
        std::memset(&a, 0, sizeof(a));
        const hipError_t e = hipPointerGetAttributes(&a, k.p);
        (void)hipGetLastError();
        hsa_amd_pointer_info_t i;
        std::memset(&i, 0, sizeof(i));
        i.size = sizeof(i);
        const hsa_status_t s = hsa_amd_pointer_info(k.p, &i, nullptr, nullptr, nullptr);
        printf("{\"kind\": \"%s\", \"hip_rc\": %d, \"hip_type\": %d, \"hip_ns\": %.1f, \"hsa_rc\": %d, \"hsa_type\": %d, "
               "\"hsa_ns\": %.1f}\n",
               k.name, (int)e, e == hipSuccess ? (int)a.type : -1, ns_per(q_hip, k.p, 20000), (int)s, (int)i.type,
               ns_per(q_hsa, k.p, 20000));
    }
    fflush(stdout);
    return 0;
}
