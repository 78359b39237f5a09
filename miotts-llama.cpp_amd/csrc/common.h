// Shared host-side plumbing for the MI355X (gfx950) MioTTS path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "mio_hip.h"

namespace mio {

// Thread-local last-error text behind mio_hip_last_error().
void set_error(const char *fmt, ...);
const char *last_error();

}  // namespace mio

#define MIO_HIP_CHECK(expr)                                                              \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) {                                                          \
            mio::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,                  \
                           hipGetErrorString(_e));                                       \
            return MIO_ERR_HIP;                                                          \
        }                                                                                \
    } while (0)

#define MIO_REQUIRE(cond, code, ...)                                                     \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            mio::set_error(__VA_ARGS__);                                                 \
            return (code);                                                               \
        }                                                                                \
    } while (0)

struct mio_hip_device {
    int dev = 0;
    hipStream_t stream = nullptr;
    int n_cu = 0;
};

namespace mio {
// Make `d` current on the calling thread.
inline int bind(const mio_hip_device *d) {
    MIO_HIP_CHECK(hipSetDevice(d->dev));
    return MIO_OK;
}
inline hipStream_t pick_stream(const mio_hip_device *d, void *stream) {
    return stream ? (hipStream_t)stream : d->stream;
}
}  // namespace mio
