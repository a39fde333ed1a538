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

// resolve a caller stream (NULL -> per-thread default stream of the library)
hipStream_t resolve_stream(void *stream);

// launch-shape knobs for the streaming kernels (see mi355x_op_tune)
struct StreamTune {
    int unroll = 4;
    int blocks_per_cu = 8;
    int nontemporal = 0;
};
StreamTune &stream_tune();

} // namespace mi355x
