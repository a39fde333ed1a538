// rt_core.cpp -- runtime plumbing of libmi355x_rt: errors, devices, streams, memory, events,
// pointer classification.  Replaces the CUDA driver shim of the reference
// (ompi/mca/common/cuda/common_cuda.c: fn table :68-106, is_gpu_buffer :1687-1783,
// cu_memcpy :1796-1846, memmove :1848-1889) with direct HIP runtime calls: HIP is linked, not
// dlopen'ed, because this library only exists on a ROCm node.
#include "rt_internal.hpp"

#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace mi355x {

static thread_local char g_err[512] = "no error";

int set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int device_cu_count()
{
    static int cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        cache[dev] = cus;
    }
    return cache[dev];
}

hipStream_t resolve_stream(void *stream)
{
    // NULL is HIP's default (null) stream, as in every HIP/CUDA API: it orders with the other
    // blocking streams of the device (torch's default stream is this stream).
    return (hipStream_t)stream;
}

StreamTune &stream_tune()
{
    static StreamTune t;
    return t;
}

} // namespace mi355x

using namespace mi355x;

extern "C" {

const char *mi355x_last_error(void) { return g_err; }
int mi355x_version(void) { return 100; }

int mi355x_device_count(int *count)
{
    if (!count) return set_error(MI355X_ERR_ARG, "count is NULL");
    MI_HIP(hipGetDeviceCount(count));
    return MI355X_SUCCESS;
}
int mi355x_set_device(int dev)
{
    MI_HIP(hipSetDevice(dev));
    return MI355X_SUCCESS;
}
int mi355x_get_device(int *dev)
{
    if (!dev) return set_error(MI355X_ERR_ARG, "dev is NULL");
    MI_HIP(hipGetDevice(dev));
    return MI355X_SUCCESS;
}
int mi355x_stream_create(void **stream)
{
    if (!stream) return set_error(MI355X_ERR_ARG, "stream is NULL");
    hipStream_t s;
    MI_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void *)s;
    return MI355X_SUCCESS;
}
int mi355x_stream_destroy(void *stream)
{
    if (stream) MI_HIP(hipStreamDestroy((hipStream_t)stream));
    return MI355X_SUCCESS;
}
int mi355x_stream_sync(void *stream)
{
    MI_HIP(hipStreamSynchronize(resolve_stream(stream)));
    return MI355X_SUCCESS;
}
int mi355x_device_sync(void)
{
    MI_HIP(hipDeviceSynchronize());
    return MI355X_SUCCESS;
}
int mi355x_malloc(void **p, size_t bytes)
{
    if (!p) return set_error(MI355X_ERR_ARG, "p is NULL");
    MI_HIP(hipMalloc(p, bytes ? bytes : 1));
    return MI355X_SUCCESS;
}
int mi355x_free(void *p)
{
    if (p) MI_HIP(hipFree(p));
    return MI355X_SUCCESS;
}
int mi355x_host_alloc(void **p, size_t bytes)
{
    if (!p) return set_error(MI355X_ERR_ARG, "p is NULL");
    MI_HIP(hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault));
    return MI355X_SUCCESS;
}
int mi355x_host_free(void *p)
{
    if (p) MI_HIP(hipHostFree(p));
    return MI355X_SUCCESS;
}
int mi355x_memcpy(void *dst, const void *src, size_t bytes)
{
    if (bytes == 0) return MI355X_SUCCESS;
    MI_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    return MI355X_SUCCESS;
}
int mi355x_memcpy_async(void *dst, const void *src, size_t bytes, void *stream)
{
    if (bytes == 0) return MI355X_SUCCESS;
    MI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, resolve_stream(stream)));
    return MI355X_SUCCESS;
}
int mi355x_memset_async(void *dst, int value, size_t bytes, void *stream)
{
    if (bytes == 0) return MI355X_SUCCESS;
    MI_HIP(hipMemsetAsync(dst, value, bytes, resolve_stream(stream)));
    return MI355X_SUCCESS;
}

// Host memory the query need not be asked about, decided without a runtime call: the brk heap
// [start_brk, current break) -- where glibc serves the main thread's allocations below the mmap
// threshold, MPI_Reduce_local's and coll/tuned's small temporaries among them -- and the calling
// thread's stack.  Both are ordinary anonymous mappings the process owns; the HIP runtime places
// device allocations in mappings of its own, never inside them, so the answer is exact.  Every
// other pointer (mmap'd host buffers, device memory) asks the runtime (rocr_unknown below).
namespace mi355x {
static uintptr_t heap_start()
{
    static const uintptr_t lo = [] {
        uintptr_t v = 0;
        FILE *f = fopen("/proc/self/stat", "r");
        if (!f) return v;
        char buf[2048];
        const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
        fclose(f);
        buf[n] = 0;
        const char *q = strrchr(buf, ')');  // the command name may hold spaces
        if (!q) return v;
        int field = 2;
        for (++q; *q && field < 47; ++q)
            if (*q == ' ') ++field;
        v = (uintptr_t)strtoull(q, nullptr, 10);  // field 47: start_brk
        return v;
    }();
    return lo;
}

static bool known_host(const void *p)
{
    const uintptr_t a = (uintptr_t)p, lo = heap_start();
    if (lo && a >= lo && a < (uintptr_t)sbrk(0)) return true;
    thread_local uintptr_t s_lo = 0, s_hi = 0;
    if (!s_hi) {
        pthread_attr_t at;
        void *base = nullptr;
        size_t sz = 0;
        if (pthread_getattr_np(pthread_self(), &at) == 0) {
            if (pthread_attr_getstack(&at, &base, &sz) == 0) {
                s_lo = (uintptr_t)base;
                s_hi = (uintptr_t)base + sz;
            }
            pthread_attr_destroy(&at);
        }
        if (!s_hi) s_hi = 1;  // (unknown: never matches)
    }
    return a >= s_lo && a < s_hi;
}
} // namespace mi355x

// Memory ROCr has no record of is ordinary host memory: every device allocation of the process --
// hipMalloc, pools, uncached / fine-grained, IPC and dmabuf imports, VMM mappings (PyTorch's
// expandable segments) -- is a ROCr allocation it can name.  hsa_amd_pointer_info answers that in
// ~42 ns where hipPointerGetAttributes takes ~100 (profiles/r05_ptrinfo.jsonl: VMM-mapped device
// memory reports type 6, managed 5, hipMalloc / hipHostMalloc 1, unregistered host 0); pointers ROCr
// does know still go to HIP for its exact memory type.  Before the runtime is initialised the call
// fails and HIP (which initialises it) answers.
static bool rocr_unknown(const void *p)
{
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    return hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
           info.type == HSA_EXT_POINTER_TYPE_UNKNOWN;
}

int mi355x_ptr_is_device(const void *p, int *is_device)
{
    if (!is_device) return set_error(MI355X_ERR_ARG, "is_device is NULL");
    *is_device = 0;
    if (!p || known_host(p) || rocr_unknown(p)) return MI355X_SUCCESS;
    hipPointerAttribute_t attr;
    std::memset(&attr, 0, sizeof(attr));
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError(); // unregistered host memory: not an error for the caller
        return MI355X_SUCCESS;
    }
    *is_device = (attr.type == hipMemoryTypeDevice) ? 1 : 0;
    return MI355X_SUCCESS;
}

int mi355x_event_create(void **ev)
{
    if (!ev) return set_error(MI355X_ERR_ARG, "ev is NULL");
    hipEvent_t e;
    MI_HIP(hipEventCreate(&e));
    *ev = (void *)e;
    return MI355X_SUCCESS;
}
int mi355x_event_destroy(void *ev)
{
    if (ev) MI_HIP(hipEventDestroy((hipEvent_t)ev));
    return MI355X_SUCCESS;
}
int mi355x_event_record(void *ev, void *stream)
{
    MI_HIP(hipEventRecord((hipEvent_t)ev, resolve_stream(stream)));
    return MI355X_SUCCESS;
}
int mi355x_event_elapsed_ms(void *start, void *stop, float *ms)
{
    if (!ms) return set_error(MI355X_ERR_ARG, "ms is NULL");
    MI_HIP(hipEventSynchronize((hipEvent_t)stop));
    MI_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return MI355X_SUCCESS;
}

int mi355x_op_tune(int unroll, int blocks_per_cu, int nontemporal)
{
    StreamTune &t = stream_tune();
    if (unroll) {
        if (unroll != 1 && unroll != 2 && unroll != 4 && unroll != 8)
            return set_error(MI355X_ERR_ARG, "unroll must be 1, 2, 4 or 8");
        t.unroll = unroll;
    }
    if (blocks_per_cu) {
        if (blocks_per_cu < 1 || blocks_per_cu > 64)
            return set_error(MI355X_ERR_ARG, "blocks_per_cu out of range");
        t.blocks_per_cu = blocks_per_cu;
    }
    if (nontemporal >= -1 && nontemporal <= 3) t.nontemporal = nontemporal;
    else if (nontemporal != -2) return set_error(MI355X_ERR_ARG, "nontemporal must be -2 (keep), -1 (auto) or 0..3");
    return MI355X_SUCCESS;
}
int mi355x_op_set_mode(int mode)
{
    if (mode != 0 && mode != 1) return set_error(MI355X_ERR_ARG, "mode must be 0 or 1");
    stream_tune().mode = mode;
    return MI355X_SUCCESS;
}
int mi355x_op_get_mode(void) { return stream_tune().mode; }
int mi355x_op_set_threads(int threads)
{
    if (threads != 64 && threads != 128 && threads != 256 && threads != 512 && threads != 1024)
        return set_error(MI355X_ERR_ARG, "threads must be 64..1024, power of two");
    stream_tune().threads = threads;
    return MI355X_SUCCESS;
}

int mi355x_op_get_tune(int *unroll, int *blocks_per_cu, int *nontemporal)
{
    StreamTune &t = stream_tune();
    if (unroll) *unroll = t.unroll;
    if (blocks_per_cu) *blocks_per_cu = t.blocks_per_cu;
    if (nontemporal) *nontemporal = t.nontemporal;
    return MI355X_SUCCESS;
}

} // extern "C"
