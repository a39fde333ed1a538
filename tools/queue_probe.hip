// queue_probe.hip -- what an extra hardware queue costs the rest of the process (round 3).
// The resident LL service (coll_svc.hip) first ran on a private HSA queue; with that queue merely
// existing, the host-synchronised small allreduce went from 17 to 55 us on the same box.  This
// probe times HIP's launch-to-completion (1-workgroup kernel + hipStreamSynchronize, a plain
// stream) in the states such a queue goes through:
//   base                 nothing extra
//   hsa_queue_idle       a private HSA queue exists, nothing dispatched
//   hsa_queue_resident   a kernel resident on it (polling a host word)
//   hsa_queue_done       that kernel has left; the queue still exists
//   hsa_queue_destroyed  the queue is gone
//   hip_hi_resident      the resident kernel on a high-priority HIP stream instead
//   hip_hi_done          that kernel has left; the stream still exists
// One JSON line per state: median / mean microseconds over N calls.  Every resident kernel leaves
// on a host word or after 5 s.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/build/queue_probe tools/queue_probe.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)
#define HK(x)                                                                                   \
    do {                                                                                        \
        if ((x) != HSA_STATUS_SUCCESS) {                                                        \
            fprintf(stderr, "%s:%d HSA call failed\n", __FILE__, __LINE__);                     \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

struct RArgs {
    const uint64_t *stop;
    uint64_t *alive;
    uint64_t limit_ticks;
    int probe;
};

extern "C" __global__ void qprobe_resident(RArgs a)
{
    if (a.probe || threadIdx.x != 0) return;
    __hip_atomic_store(a.alive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
           __builtin_amdgcn_s_memrealtime() - t0 < a.limit_ticks)
        __builtin_amdgcn_s_sleep(2);
}

__global__ void k_tiny(float *x) { if (threadIdx.x == 0 && blockIdx.x == 0) x[0] += 1.f; }

using clk = std::chrono::steady_clock;
static double el(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

static void measure(const char *state, hipStream_t s, float *x, int n)
{
    std::vector<double> us(n);
    for (int i = 0; i < 20; ++i) {
        k_tiny<<<1, 64, 0, s>>>(x);
        CK(hipStreamSynchronize(s));
    }
    for (int i = 0; i < n; ++i) {
        const auto a = clk::now();
        k_tiny<<<1, 64, 0, s>>>(x);
        CK(hipStreamSynchronize(s));
        us[i] = el(a, clk::now());
    }
    std::sort(us.begin(), us.end());
    double sum = 0;
    for (double u : us) sum += u;
    printf("{\"probe\": \"launch_sync\", \"state\": \"%s\", \"median_us\": %.2f, \"mean_us\": %.2f, \"p90_us\": %.2f}\n",
           state, us[n / 2], sum / n, us[n * 9 / 10]);
    fflush(stdout);
}

struct Find {
    hsa_agent_t agent;
    hsa_executable_symbol_t sym;
    bool found;
};
static hsa_status_t gpu_cb(hsa_agent_t ag, void *d)
{
    hsa_device_type_t t;
    hsa_agent_get_info(ag, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        *(hsa_agent_t *)d = ag;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t sym_cb(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void *d)
{
    Find *f = (Find *)d;
    uint32_t len = 0;
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
    std::string name(len, '\0');
    hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]);
    if (name == "qprobe_resident" || name == "qprobe_resident.kd") {
        f->sym = sym;
        f->found = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t exe_cb(hsa_executable_t exe, void *d)
{
    Find *f = (Find *)d;
    hsa_executable_iterate_agent_symbols(exe, f->agent, sym_cb, d);
    return f->found ? HSA_STATUS_INFO_BREAK : HSA_STATUS_SUCCESS;
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    // Q_EARLY=1: a private HSA queue created before HIP has made any queue for its streams
    hsa_queue_t *early = nullptr;
    if (getenv("Q_EARLY") && atoi(getenv("Q_EARLY"))) {
        CK(hipSetDevice(0));
        CK(hipFree(nullptr));
        HK(hsa_init());
        hsa_agent_t ag{0};
        hsa_iterate_agents(gpu_cb, &ag);
        HK(hsa_queue_create(ag, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &early));
        printf("{\"probe\": \"early_hsa_queue\", \"created\": true}\n");
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x;
    CK(hipMalloc(&x, 4096));
    uint64_t *host;
    CK(hipHostMalloc((void **)&host, 4096, hipHostMallocCoherent));
    memset(host, 0, 4096);
    auto *stop = reinterpret_cast<std::atomic<uint64_t> *>(host);
    auto *alive = reinterpret_cast<std::atomic<uint64_t> *>(host + 8);
    // Q_STREAMS=k: k more HIP streams, each used once (HIP deals them over up to GPU_MAX_HW_QUEUES
    // hardware queues), before anything is measured
    const int extra = getenv("Q_STREAMS") ? atoi(getenv("Q_STREAMS")) : 0;
    std::vector<hipStream_t> xs(extra);
    for (auto &e : xs) {
        CK(hipStreamCreateWithFlags(&e, hipStreamNonBlocking));
        k_tiny<<<1, 64, 0, e>>>(x);
        CK(hipStreamSynchronize(e));
    }
    printf("{\"probe\": \"extra_hip_streams\", \"n\": %d}\n", extra);
    measure("base", s, x, n);

    RArgs pr{host, host + 8, 0, 1};
    hipLaunchKernelGGL(qprobe_resident, dim3(1), dim3(64), 0, s, pr);
    CK(hipStreamSynchronize(s));
    HK(hsa_init());
    Find f{{0}, {0}, false};
    hsa_iterate_agents(gpu_cb, &f.agent);
    hsa_ven_amd_loader_1_03_pfn_t ldr;
    memset(&ldr, 0, sizeof(ldr));
    HK(hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ldr), &ldr));
    ldr.hsa_ven_amd_loader_iterate_executables(exe_cb, &f);
    if (!f.found) {
        fprintf(stderr, "kernel not found\n");
        return 1;
    }
    uint64_t kobj = 0;
    uint32_t kargs = 0, grp = 0, prv = 0;
    hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj);
    hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargs);
    hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &grp);
    hsa_executable_symbol_get_info(f.sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &prv);
    void *karg;
    CK(hipHostMalloc(&karg, 4096, hipHostMallocCoherent));
    memset(karg, 0, 4096);
    RArgs ra{host, host + 8, (uint64_t)5e8, 0};
    memcpy(karg, &ra, sizeof(ra));
    hsa_queue_t *q = nullptr;
    HK(hsa_queue_create(f.agent, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    hsa_signal_t sig;
    HK(hsa_signal_create(0, 0, nullptr, &sig));
    measure("hsa_queue_idle", s, x, n);
    // dispatch the resident kernel
    hsa_signal_store_screlease(sig, 1);
    const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q, 1);
    auto *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
    memset((char *)p + 4, 0, sizeof(*p) - 4);
    p->workgroup_size_x = 64;
    p->workgroup_size_y = p->workgroup_size_z = 1;
    p->grid_size_x = 64;
    p->grid_size_y = p->grid_size_z = 1;
    p->private_segment_size = prv;
    p->group_segment_size = grp;
    p->kernel_object = kobj;
    p->kernarg_address = karg;
    p->completion_signal = sig;
    const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                         (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                         (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    __atomic_store_n((uint32_t *)p, hdr | ((1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, idx);
    const auto t0 = clk::now();
    while (alive->load() == 0 && el(t0, clk::now()) < 2e6) {
    }
    printf("{\"probe\": \"resident_started\", \"alive\": %llu}\n", (unsigned long long)alive->load());
    measure("hsa_queue_resident", s, x, n);
    stop->store(1);
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, 6000000000ull, HSA_WAIT_STATE_BLOCKED);
    measure("hsa_queue_done", s, x, n);
    HK(hsa_queue_destroy(q));
    measure("hsa_queue_destroyed", s, x, n);
    // the same on a high-priority HIP stream
    stop->store(0);
    alive->store(0);
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t hs;
    CK(hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, hi));
    measure("hip_hi_stream_idle", s, x, n);
    hipLaunchKernelGGL(qprobe_resident, dim3(1), dim3(64), 0, hs, ra);
    const auto t1 = clk::now();
    while (alive->load() == 0 && el(t1, clk::now()) < 2e6) {
    }
    measure("hip_hi_resident", s, x, n);
    stop->store(1);
    CK(hipStreamSynchronize(hs));
    measure("hip_hi_done", s, x, n);
    hsa_signal_destroy(sig);
    return 0;
}
