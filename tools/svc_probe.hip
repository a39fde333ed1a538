// svc_probe.hip -- can a resident (persistent) service kernel replace the launch of a small
// collective?  Measures, on one MI355X:
//   * the doorbell round trip: the host stores a call number into host memory, a resident
//     one-workgroup kernel polling that word picks it up, copies a small payload on the device,
//     publishes it (system-scope release) and stores the number into a host completion word the
//     host spins on -- per stream kind (plain, CU-masked, high priority);
//   * whether the resident kernel's hardware queue is its own: while it runs, a trivial kernel is
//     launched on the null stream and on 8 fresh plain streams and each is waited for (50 ms);
//     a stream that does not complete shares the resident kernel's queue.
// The resident kernel always exits: on a QUIT number, or after 2 s without a doorbell.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/build/svc_probe tools/svc_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <csetjmp>
#include <csignal>
#include <sys/mman.h>
#include <vector>
#include <immintrin.h>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr uint64_t kQuit = ~0ull;

struct Desc {  // written by the host before the doorbell
    const uint64_t *src;
    uint64_t *dst;
    uint64_t nwords;
};

__global__ __launch_bounds__(64) void k_svc(const uint64_t *door, uint64_t *done, const Desc *desc, uint64_t idle_ticks,
                                            uint64_t *exit_word, int fence)
{
    __shared__ uint64_t cur;
    uint64_t last = 0;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            uint64_t v;
            for (;;) {
                v = __hip_atomic_load(door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v != last) break;
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
                    v = kQuit;
                    break;
                }
            }
            cur = v;
        }
        __syncthreads();
        const uint64_t v = cur;
        __syncthreads();
        if (v == kQuit) break;
        last = v;
        // the call: copy the payload (system-scope loads: the descriptor lives in host memory)
        const uint64_t *src = (const uint64_t *)__hip_atomic_load((const uint64_t *)&desc->src, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_SYSTEM);
        uint64_t *dst = (uint64_t *)__hip_atomic_load((const uint64_t *)&desc->dst, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t nw = __hip_atomic_load(&desc->nwords, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (uint64_t i = threadIdx.x; i < nw; i += blockDim.x)
            __hip_atomic_store(dst + i, src[i] + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (fence) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    if (threadIdx.x == 0) __hip_atomic_store(exit_word, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_tiny(float *x) { if (threadIdx.x == 0 && blockIdx.x == 0) x[0] += 1.f; }

static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }
// can the host store into this device allocation directly (large-BAR mapping)?
static bool host_writable(volatile uint64_t *p)
{
    struct sigaction sa, old_segv, old_bus;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_jmp, 1) == 0) {
        p[0] = 0x1234;
        ok = p[0] == 0x1234;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

using clk = std::chrono::steady_clock;
static double el(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

static void report(const char *name, const char *extra, std::vector<double> &us)
{
    std::sort(us.begin(), us.end());
    double s = 0;
    for (double u : us) s += u;
    printf("{\"probe\": \"%s\", %s\"median_us\": %.2f, \"mean_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, "
           "\"p99_us\": %.2f, \"n\": %zu}\n",
           name, extra, us[us.size() / 2], s / us.size(), us[us.size() / 10], us[us.size() * 9 / 10],
           us[us.size() * 99 / 100], us.size());
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 5000;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint64_t *dsrc, *ddst;
    float *x;
    CK(hipMalloc(&dsrc, 1 << 16));
    CK(hipMalloc(&ddst, 1 << 16));
    CK(hipMalloc(&x, 4096));
    CK(hipMemset(dsrc, 1, 1 << 16));
    CK(hipMemset(x, 0, 4096));
    // host words: a shared mapping registered with HIP (like the engine's control segment)
    void *seg = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    CK(hipHostRegister(seg, 4096, hipHostRegisterMapped));
    char *dseg = nullptr;
    CK(hipHostGetDevicePointer((void **)&dseg, seg, 0));
    auto *done = reinterpret_cast<std::atomic<uint64_t> *>((char *)seg + 256);
    auto *exitw = reinterpret_cast<std::atomic<uint64_t> *>((char *)seg + 512);
    Desc *desc = reinterpret_cast<Desc *>((char *)seg + 768);
    // a doorbell in fine-grained device memory the host stores into directly (if it can)
    uint64_t *fdoor = nullptr;
    CK(hipExtMallocWithFlags((void **)&fdoor, 4096, getenv("SVC_UNCACHED") ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    CK(hipMemset(fdoor, 0, 4096));
    CK(hipDeviceSynchronize());
    const bool fine_ok = host_writable(fdoor);
    printf("{\"probe\": \"host_store_into_finegrained_device_memory\", \"ok\": %s}\n", fine_ok ? "true" : "false");
    fflush(stdout);

    for (int where = 0; where < 2; ++where) {
        if (where == 1 && !fine_ok) break;
        const char *wname = where == 0 ? "host" : "device_finegrained";
        auto *door = where == 0 ? reinterpret_cast<std::atomic<uint64_t> *>((char *)seg)
                                : reinterpret_cast<std::atomic<uint64_t> *>(fdoor);
        const uint64_t *ddoor = where == 0 ? (const uint64_t *)dseg : fdoor;
        for (int kind = 0; kind < 4; ++kind) {
            if (where == 0 && getenv("SVC_DEVICE_ONLY")) continue;
            if (kind == 1) continue;  // CU-masked streams are blocking streams: the null stream waits on them
            if (where == 1 && kind < 2) continue;
            const int fence = kind != 3;
            const char *kname = kind == 0 ? "plain" : kind == 1 ? "cumask_all" : kind == 2 ? "high_priority" : "high_priority_nofence";
            hipStream_t s;
            if (kind == 0) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            if (kind == 1) {
                std::vector<uint32_t> mask((ncu + 31) / 32, 0xffffffffu);
                CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
            }
            if (kind >= 2) {
                int lo, hi;
                CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
                CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
            }
            for (int nw : {1, 512}) {
                door->store(0);
                done->store(0);
                exitw->store(0);
                desc->src = dsrc;
                desc->dst = ddst;
                desc->nwords = (uint64_t)nw;
                hipLaunchKernelGGL(k_svc, dim3(1), dim3(64), 0, s, ddoor, (uint64_t *)(dseg + 256),
                                   (const Desc *)(dseg + 768), (uint64_t)2e8, (uint64_t *)(dseg + 512), fence);
                CK(hipGetLastError());
                // warm up: the kernel must be running before timing
                uint64_t v = 0;
                bool alive = true;
                for (int i = 0; i < 200 && alive; ++i) {
                    door->store(++v, std::memory_order_release);
                    _mm_sfence();
                    const auto t0 = clk::now();
                    while (done->load(std::memory_order_acquire) != v) {
                        if (el(t0, clk::now()) > 1e6) {
                            alive = false;
                            break;
                        }
                    }
                }
                char extra[160];
                snprintf(extra, sizeof(extra), "\"door\": \"%s\", \"stream\": \"%s\", \"payload_bytes\": %d, ", wname,
                         kname, nw * 8);
                if (!alive) {
                    printf("{\"probe\": \"svc_roundtrip\", %s\"error\": \"no answer in 1 s\"}\n", extra);
                    door->store(kQuit, std::memory_order_release);
                    CK(hipStreamSynchronize(s));
                    continue;
                }
                std::vector<double> us(n);
                for (int i = 0; i < n; ++i) {
                    const auto a = clk::now();
                    door->store(++v, std::memory_order_release);
                    _mm_sfence();
                    while (done->load(std::memory_order_acquire) != v) {
                    }
                    us[i] = el(a, clk::now());
                }
                report("svc_roundtrip", extra, us);
                // isolation: trivial kernels on other streams while the resident kernel runs
                if (nw == 1) {
                    std::vector<hipStream_t> o(8);
                    int stalled = 0, null_stalled = 0;
                    for (auto &q : o) CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
                    for (int j = 0; j < 9; ++j) {
                        hipStream_t q = j < 8 ? o[j] : nullptr;
                        const auto t0 = clk::now();
                        k_tiny<<<1, 64, 0, q>>>(x);
                        bool ok = false;
                        while (el(t0, clk::now()) < 5e4)
                            if (hipStreamQuery(q) == hipSuccess) {
                                ok = true;
                                break;
                            }
                        if (!ok) (j < 8 ? stalled : null_stalled)++;
                        // the resident kernel still answers (bounded: it exits after 2 s idle)
                        door->store(++v, std::memory_order_release);
                        _mm_sfence();
                        const auto t1 = clk::now();
                        while (done->load(std::memory_order_acquire) != v && el(t1, clk::now()) < 3e6) {
                        }
                    }
                    printf("{\"probe\": \"svc_isolation\", %s\"plain_streams_stalled\": %d, \"of\": 8, "
                           "\"null_stream_stalled\": %d}\n",
                           extra, stalled, null_stalled);
                    fflush(stdout);
                    door->store(kQuit, std::memory_order_release);
                    CK(hipStreamSynchronize(s));
                    for (auto &q : o) {
                        CK(hipStreamSynchronize(q));
                        CK(hipStreamDestroy(q));
                    }
                    CK(hipStreamSynchronize(nullptr));
                } else {
                    door->store(kQuit, std::memory_order_release);
                    CK(hipStreamSynchronize(s));
                }
                // the copy happened
                std::vector<uint64_t> h(nw);
                CK(hipMemcpy(h.data(), ddst, nw * 8, hipMemcpyDeviceToHost));
                if (h[0] != 0x0101010101010101ull + v)
                    printf("{\"probe\": \"svc_check\", %s\"error\": \"payload %llx\"}\n", extra, (unsigned long long)h[0]);
            }
            CK(hipStreamDestroy(s));
        }
    }
    CK(hipFree(fdoor));
    CK(hipHostUnregister(seg));
    munmap(seg, 4096);
    return 0;
}
