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

// One WAV sample of wav_write (wav-writer.cpp:24-44):
// static_cast<int16_t>(std::clamp(s * 32767.0f, -32768.0f, 32767.0f)), truncated toward zero.
// std::clamp compares (v < lo) then (hi < v), so a NaN passes through; the reference's x86
// build converts it with cvttss2si (integer indefinite 0x80000000), whose low 16 bits are 0.
// Host writer and device epilogue share this, so both emit the reference's bytes.
__host__ __device__ inline int16_t pcm16_sample(float s) {
    const float t = s * 32767.0f;
    const float c = t < -32768.0f ? -32768.0f : (32767.0f < t ? 32767.0f : t);
    return c != c ? (int16_t)0 : (int16_t)(int)c;
}
}  // namespace mio
