// svc_queue.cpp -- a private HSA queue for the resident LL service kernel (coll_svc.hip).
//
// The service kernel stays resident between calls, so it must not sit in a hardware queue that
// anything else uses: HIP deals its streams over a few pooled queues per priority (GPU_MAX_HW_
// QUEUES), and work on a stream that shares the resident kernel's queue would wait behind it
// (profiles/r03_svc_probe.jsonl: 1 of 8 fresh plain streams stalled), and hipDeviceSynchronize
// would wait for the kernel to leave.  So the service is dispatched as an AQL packet on a queue
// of its own, created with hsa_queue_create on the HIP device's agent -- HIP never sees it.
// The kernel is the one compiled into this library: a probe launch through HIP makes the runtime
// load the code object on the device, and the loader extension finds its kernel descriptor
// (`mi355x_k_svc`) among the loaded executables.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <sched.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "coll_internal.hpp"
#include "svc_queue.hpp"

namespace mi355x {

namespace {

struct AgentFind {
    uint32_t bdfid, domain;
    hsa_agent_t agent;
    bool found;
};

hsa_status_t find_agent(hsa_agent_t ag, void *data)
{
    AgentFind *f = static_cast<AgentFind *>(data);
    hsa_device_type_t type;
    if (hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS || type != HSA_DEVICE_TYPE_GPU)
        return HSA_STATUS_SUCCESS;
    uint32_t bdfid = 0, domain = 0;
    if (hsa_agent_get_info(ag, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdfid) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    (void)hsa_agent_get_info(ag, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain);
    if (bdfid == f->bdfid && domain == f->domain) {
        f->agent = ag;
        f->found = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

struct PoolFind {
    hsa_amd_memory_pool_t pool;
    bool found;
};

hsa_status_t find_fine_pool(hsa_amd_memory_pool_t pool, void *data)
{
    PoolFind *f = static_cast<PoolFind *>(data);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    bool alloc = false;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    (void)hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    (void)hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED)) {
        f->pool = pool;
        f->found = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t find_cpu(hsa_agent_t ag, void *data)
{
    hsa_device_type_t type;
    if (hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &type) == HSA_STATUS_SUCCESS && type == HSA_DEVICE_TYPE_CPU) {
        *static_cast<hsa_agent_t *>(data) = ag;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

struct SymFind {
    hsa_agent_t agent;
    hsa_executable_symbol_t sym;
    bool found;
};

hsa_status_t find_sym(hsa_executable_t exe, hsa_agent_t ag, hsa_executable_symbol_t sym, void *data)
{
    (void)exe;
    (void)ag;
    SymFind *f = static_cast<SymFind *>(data);
    hsa_symbol_kind_t kind;
    if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
        kind != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    std::string name(len, '\0');
    if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    if (name == "mi355x_k_svc" || name == "mi355x_k_svc.kd") {
        f->sym = sym;
        f->found = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t find_exe(hsa_executable_t exe, void *data)
{
    SymFind *f = static_cast<SymFind *>(data);
    (void)hsa_executable_iterate_agent_symbols(exe, f->agent, find_sym, data);
    return f->found ? HSA_STATUS_INFO_BREAK : HSA_STATUS_SUCCESS;
}

int fail(std::string *why, const char *what)
{
    if (why) *why = what;
    return -1;
}

} // namespace

// (experiment, MI355X_SVC_PREP) parts of the service's creation on their own, kept for the process
int svc_prep(int device, int mask)
{
    if (mask & 1) (void)hsa_init();
    if (mask & 2) (void)svc_probe_launch(device);
    if (mask & (8 | 16)) {
        (void)hsa_init();
        int bus = 0, dev = 0, dom = 0;
        (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device);
        (void)hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device);
        (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device);
        AgentFind af{(uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom, {0}, false};
        (void)hsa_iterate_agents(find_agent, &af);
        if (!af.found) return -1;
        if (mask & 8) {
            hsa_queue_t *hq = nullptr;
            (void)hsa_queue_create(af.agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &hq);
        }
        if (mask & 16) {
            hsa_signal_t sig;
            (void)hsa_signal_create(0, 0, nullptr, &sig);
        }
    }
    return 0;
}

int svc_queue_create(int device, SvcQueue *q, std::string *why)
{
    std::memset(static_cast<void *>(q), 0, sizeof(*q));
    if (hsa_init() != HSA_STATUS_SUCCESS) return fail(why, "hsa_init");  // reference-counted
    q->hsa_inited = true;
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
        return fail(why, "PCI location of the HIP device");
    AgentFind af{(uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom, {0}, false};
    (void)hsa_iterate_agents(find_agent, &af);
    if (!af.found) return fail(why, "no HSA agent at the HIP device's PCI location");
    q->agent = af.agent.handle;
    // make HIP load this library's code object on the device, then find the kernel in it
    if (svc_probe_launch(device) != 0) return fail(why, "probe launch of the service kernel");
    hsa_ven_amd_loader_1_03_pfn_t ldr;
    std::memset(&ldr, 0, sizeof(ldr));
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ldr), &ldr) != HSA_STATUS_SUCCESS ||
        !ldr.hsa_ven_amd_loader_iterate_executables)
        return fail(why, "HSA loader extension");
    SymFind sf{af.agent, {0}, false};
    (void)ldr.hsa_ven_amd_loader_iterate_executables(find_exe, &sf);
    if (!sf.found) return fail(why, "mi355x_k_svc not among the loaded executables");
    uint32_t kargs = 0, group = 0, priv = 0;
    if (hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &q->kernel_object) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargs) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &group) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sf.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &priv) !=
            HSA_STATUS_SUCCESS)
        return fail(why, "kernel symbol info");
    q->kernarg_bytes = kargs > sizeof(SvcArgs) ? kargs : (uint32_t)sizeof(SvcArgs);
    q->group_bytes = group;
    q->private_bytes = priv;
    // kernel arguments in pinned host memory the GPU reads (one launch in flight at a time)
    if (hipHostMalloc(&q->kernarg, (q->kernarg_bytes + 4095) / 4096 * 4096, hipHostMallocCoherent) != hipSuccess)
        return fail(why, "kernarg buffer");
    hsa_queue_t *hq = nullptr;
    if (hsa_queue_create(af.agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &hq) !=
        HSA_STATUS_SUCCESS)
        return fail(why, "hsa_queue_create");
    q->queue = hq;
    hsa_signal_t sig;
    if (hsa_signal_create(0, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return fail(why, "hsa_signal_create");
    q->signal = sig.handle;
    return 0;
}

int svc_dispatch(SvcQueue *q, const SvcArgs &args, int nwg)
{
    hsa_queue_t *hq = static_cast<hsa_queue_t *>(q->queue);
    hsa_signal_t sig{q->signal};
    if (hsa_signal_load_scacquire(sig) != 0) return -1;  // the previous launch is still resident
    std::memset(q->kernarg, 0, q->kernarg_bytes);
    std::memcpy(q->kernarg, &args, sizeof(args));
    hsa_signal_store_screlease(sig, 1);
    const uint64_t idx = hsa_queue_add_write_index_scacq_screl(hq, 1);
    while (idx - hsa_queue_load_read_index_scacquire(hq) >= hq->size) sched_yield();
    hsa_kernel_dispatch_packet_t *p =
        static_cast<hsa_kernel_dispatch_packet_t *>(hq->base_address) + (idx & (hq->size - 1));
    p->workgroup_size_x = (uint16_t)kSvcThreads;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = (uint32_t)nwg * (uint32_t)kSvcThreads;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = q->private_bytes;
    p->group_segment_size = q->group_bytes;
    p->kernel_object = q->kernel_object;
    p->kernarg_address = q->kernarg;
    p->reserved2 = 0;
    p->completion_signal = sig;
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1u << HSA_PACKET_HEADER_BARRIER) |
                                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = (uint16_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
    __atomic_store_n(reinterpret_cast<uint32_t *>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(hq->doorbell_signal, (hsa_signal_value_t)idx);
    return 0;
}

bool svc_resident(const SvcQueue *q)
{
    return q->queue && hsa_signal_load_scacquire(hsa_signal_t{q->signal}) != 0;
}

bool svc_wait_exit(const SvcQueue *q, double seconds)
{
    if (!q->queue) return true;
    const uint64_t ns = (uint64_t)(seconds * 1e9);
    return hsa_signal_wait_scacquire(hsa_signal_t{q->signal}, HSA_SIGNAL_CONDITION_EQ, 0, ns,
                                     HSA_WAIT_STATE_BLOCKED) == 0;
}

int svc_page_alloc(SvcQueue *q, size_t bytes, void **p, bool *device)
{
    *p = nullptr;
    *device = false;
    // fine-grained memory of the GPU, opened to the CPU: the host's stores reach it through the
    // BAR (write-combined: the caller fences them), the kernel polls it without crossing PCIe
    PoolFind pf{{0}, false};
    hsa_agent_t cpu{0};
    const char *host_only = getenv("MI355X_SVC_HOST_PAGE");
    if (!(host_only && atoi(host_only))) {
        (void)hsa_amd_agent_iterate_memory_pools(hsa_agent_t{q->agent}, find_fine_pool, &pf);
        (void)hsa_iterate_agents(find_cpu, &cpu);
    }
    if (pf.found && cpu.handle) {
        void *m = nullptr;
        if (hsa_amd_memory_pool_allocate(pf.pool, bytes, 0, &m) == HSA_STATUS_SUCCESS) {
            if (hsa_amd_agents_allow_access(1, &cpu, nullptr, m) == HSA_STATUS_SUCCESS) {
                std::memset(m, 0, bytes);
                *p = m;
                *device = true;
                return 0;
            }
            (void)hsa_amd_memory_pool_free(m);
        }
    }
    // else pinned host memory (the kernel's polls cross PCIe: ~0.8 us more per call)
    if (hipHostMalloc(p, bytes, hipHostMallocCoherent) != hipSuccess) return -1;
    std::memset(*p, 0, bytes);
    return 0;
}

void svc_page_free(void *p, bool device)
{
    if (!p) return;
    if (device)
        (void)hsa_amd_memory_pool_free(p);
    else
        (void)hipHostFree(p);
}

void svc_queue_destroy(SvcQueue *q)
{
    if (q->queue) (void)hsa_queue_destroy(static_cast<hsa_queue_t *>(q->queue));
    if (q->signal) (void)hsa_signal_destroy(hsa_signal_t{q->signal});
    if (q->kernarg) (void)hipHostFree(q->kernarg);
    if (q->hsa_inited) (void)hsa_shut_down();
    std::memset(static_cast<void *>(q), 0, sizeof(*q));
}

} // namespace mi355x
