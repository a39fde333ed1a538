// latency_probe.hip -- where a host-synchronised small collective spends its time on one MI355X
// (round 3): the per-call pieces of the engine's one-phase flow, timed alone.
//   sync_idle      hipStreamSynchronize on an idle stream (the "input complete" step)
//   query_idle     hipStreamQuery on an idle stream
//   launch_sync    launch a 1-workgroup kernel + hipStreamSynchronize (launch-to-completion)
//   launch_spin    the same, completion observed by spinning on hipStreamQuery
//   launch_wv      launch + hipStreamWriteValue64 into host-registered memory, host polls the word
//   launch_flag    the kernel's last workgroup stores the word itself (system scope), host polls
//   launch_flag_64 the same with a 64-workgroup grid (last-workgroup counter)
// One JSON line per variant: median and mean microseconds over N calls.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/latency_probe tools/latency_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void k_tiny(float *x) { if (threadIdx.x == 0 && blockIdx.x == 0) x[0] += 1.f; }

// last workgroup out writes `v` into the host-visible word (vector store, system scope)
__global__ void k_flag(float *x, unsigned *ctr, uint64_t *word, uint64_t v)
{
    if (threadIdx.x == 0) x[blockIdx.x] += 1.f;
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);
        const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            *ctr = 0;
            __hip_atomic_store(word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// kernel arguments of the engine's sizes: 64 peer pointers + fields (~0.6 KiB) and ~4 KiB
struct Args600 { const void *src[64]; void *dst; uint64_t a, b, c, d, e, f, g, h; };
struct Args4K { const void *src[64]; void *dst[64]; uint64_t len[64]; uint64_t rest[320]; };
__global__ void k_args600(Args600 a) { if (threadIdx.x == 0 && blockIdx.x == 0) ((float *)a.dst)[0] += (float)a.a; }
__global__ void k_args4k(Args4K a) { if (threadIdx.x == 0 && blockIdx.x == 0) ((float *)a.dst[0])[0] += (float)a.len[0]; }

using clk = std::chrono::steady_clock;

static void report(const char *name, std::vector<double> &us)
{
    std::sort(us.begin(), us.end());
    double s = 0;
    for (double u : us) s += u;
    printf("{\"probe\": \"%s\", \"median_us\": %.2f, \"mean_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"n\": %zu}\n",
           name, us[us.size() / 2], s / us.size(), us[us.size() / 10], us[us.size() * 9 / 10], us.size());
    fflush(stdout);
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *x;
    unsigned *ctr;
    CK(hipMalloc(&x, 4096));
    CK(hipMalloc(&ctr, 4));
    CK(hipMemset(x, 0, 4096));
    CK(hipMemset(ctr, 0, 4));
    // a shared mapping registered with HIP, like the engine's control segment
    void *seg = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    CK(hipHostRegister(seg, 4096, hipHostRegisterMapped));
    uint64_t *hword = (uint64_t *)seg;
    uint64_t *dword = nullptr;
    CK(hipHostGetDevicePointer((void **)&dword, seg, 0));
    auto *aw = reinterpret_cast<std::atomic<uint64_t> *>(hword);
    aw->store(0);
    for (int i = 0; i < 50; ++i) k_tiny<<<1, 64, 0, s>>>(x);
    CK(hipStreamSynchronize(s));
    std::vector<double> us(n);
    auto t = [&]() { return clk::now(); };
    auto el = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    for (int i = 0; i < n; ++i) {
        auto a = t();
        CK(hipStreamSynchronize(s));
        us[i] = el(a, t());
    }
    report("sync_idle", us);
    for (int i = 0; i < n; ++i) {
        auto a = t();
        (void)hipStreamQuery(s);
        us[i] = el(a, t());
    }
    report("query_idle", us);
    for (int i = 0; i < n; ++i) {
        auto a = t();
        k_tiny<<<1, 64, 0, s>>>(x);
        CK(hipStreamSynchronize(s));
        us[i] = el(a, t());
    }
    report("launch_sync", us);
    {
        Args600 a600;
        memset(&a600, 0, sizeof(a600));
        a600.dst = x;
        Args4K a4;
        memset(&a4, 0, sizeof(a4));
        a4.dst[0] = x;
        for (int i = 0; i < n; ++i) {
            auto a = t();
            k_tiny<<<1, 64, 0, s>>>(x);
            us[i] = el(a, t());
            CK(hipStreamSynchronize(s));
        }
        report("launch_only_8B_args", us);
        for (int i = 0; i < n; ++i) {
            auto a = t();
            k_args600<<<1, 64, 0, s>>>(a600);
            us[i] = el(a, t());
            CK(hipStreamSynchronize(s));
        }
        report("launch_only_600B_args", us);
        for (int i = 0; i < n; ++i) {
            auto a = t();
            k_args4k<<<1, 64, 0, s>>>(a4);
            us[i] = el(a, t());
            CK(hipStreamSynchronize(s));
        }
        report("launch_only_4KiB_args", us);
        for (int i = 0; i < n; ++i) {
            auto a = t();
            k_args4k<<<1, 64, 0, s>>>(a4);
            CK(hipStreamSynchronize(s));
            us[i] = el(a, t());
        }
        report("launch_sync_4KiB_args", us);
        for (int i = 0; i < n; ++i) {   // the legacy null stream (an engine call with stream NULL)
            auto a = t();
            k_args600<<<1, 64, 0, nullptr>>>(a600);
            CK(hipStreamSynchronize(nullptr));
            us[i] = el(a, t());
        }
        report("launch_sync_600B_null_stream", us);
        for (int i = 0; i < n; ++i) {
            auto a = t();
            k_args600<<<1, 64, 0, s>>>(a600);
            CK(hipStreamSynchronize(s));
            us[i] = el(a, t());
        }
        report("launch_sync_600B_nonblocking_stream", us);
    }
    for (int i = 0; i < n; ++i) {
        auto a = t();
        k_tiny<<<1, 64, 0, s>>>(x);
        while (hipStreamQuery(s) == hipErrorNotReady) {
        }
        us[i] = el(a, t());
    }
    report("launch_spin", us);
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) {
        auto a = t();
        k_tiny<<<1, 64, 0, s>>>(x);
        CK(hipStreamWriteValue64(s, dword, ++v, 0));
        while (aw->load(std::memory_order_acquire) < v) {
        }
        us[i] = el(a, t());
    }
    report("launch_wv", us);
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i) {
        auto a = t();
        k_flag<<<1, 64, 0, s>>>(x, ctr, dword, ++v);
        while (aw->load(std::memory_order_acquire) < v) {
        }
        us[i] = el(a, t());
    }
    report("launch_flag", us);
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i) {
        auto a = t();
        k_flag<<<64, 64, 0, s>>>(x, ctr, dword, ++v);
        while (aw->load(std::memory_order_acquire) < v) {
        }
        us[i] = el(a, t());
    }
    report("launch_flag_64", us);
    CK(hipStreamSynchronize(s));
    // the flag form followed by a stream sync (what a caller that syncs its stream after us pays)
    for (int i = 0; i < n; ++i) {
        auto a = t();
        k_flag<<<1, 64, 0, s>>>(x, ctr, dword, ++v);
        while (aw->load(std::memory_order_acquire) < v) {
        }
        CK(hipStreamSynchronize(s));
        us[i] = el(a, t());
    }
    report("launch_flag_then_sync", us);
    CK(hipHostUnregister(seg));
    munmap(seg, 4096);
    return 0;
}
