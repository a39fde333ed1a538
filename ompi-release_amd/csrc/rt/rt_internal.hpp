// rt_internal.hpp -- shared helpers of libmi355x_rt (not part of the public C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>

#include "../../../include/mi355x_rt.h"

namespace mi355x {

// record a formatted error message for mi355x_last_error() and return `code`
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// HIP call wrapper: on failure records "<what>: <hipGetErrorString>" and returns MI355X_ERR_HIP
#define MI_HIP(call)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess)                                                            \
            return ::mi355x::set_error(MI355X_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, \
                                       #call, hipGetErrorString(e_));                    \
    } while (0)

// number of compute units of the current device (cached per device)
int device_cu_count();

// Makes `dev` current for the scope and restores the caller's device afterwards: the engine
// never leaves the application's current device changed (an MPI call must not move later
// application allocations to another GPU).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) {
            (void)hipGetLastError();
            cur = -1;
        }
        if (cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// caller stream as a hipStream_t (NULL = the HIP null stream)
hipStream_t resolve_stream(void *stream);

// launch-shape knobs for the streaming kernels (see mi355x_op_tune)
struct StreamTune {
    int unroll = 1;         // measured best on MI355X for 1 GiB operands (profiles/r01_op_tune.json)
    int blocks_per_cu = 2;  // grid-stride mode: 512 resident blocks
    int nontemporal = -1;   // -1 auto (streams > 256 MiB), else mask: 1 loads, 2 stores
    int mode = 1;           // 0 = grid-stride, 1 = one-shot chunked grid
    int threads = 1024;     // block size of the one-shot grid (measured best, profiles/r01_op_tune.json)
};
StreamTune &stream_tune();

} // namespace mi355x
