// C-ABI: device, memory and event-timer entry points (include/mio_hip.h).
#include "common.h"

#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <string>

namespace mio {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const char *last_error() { return g_err; }

}  // namespace mio

namespace {
constexpr int kTimerSlots = 16;
struct TimerBank {
    int dev = -1;
    hipEvent_t ev[kTimerSlots] = {};
};
thread_local TimerBank g_timers[8];
}  // namespace

extern "C" const char *mio_hip_last_error(void) { return mio::last_error(); }

extern "C" int mio_hip_device_count(int *n) {
    MIO_REQUIRE(n, MIO_ERR_INVALID, "device_count: null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *n = c;
    return MIO_OK;
}

extern "C" int mio_hip_device_open(int dev, mio_hip_device **out) {
    MIO_REQUIRE(out, MIO_ERR_INVALID, "device_open: null out");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) {
        mio::set_error("device_open: no HIP device visible");
        return MIO_ERR_HIP;
    }
    MIO_REQUIRE(dev >= 0 && dev < c, MIO_ERR_INVALID, "device_open: device %d of %d", dev, c);
    MIO_HIP_CHECK(hipSetDevice(dev));
    auto *d = new mio_hip_device();
    d->dev = dev;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) d->n_cu = prop.multiProcessorCount;
    // MIO_STREAM_PRIO=high|low: priority of the device stream (LLM steps, one-shot codec)
    int prio = 0, least = 0, greatest = 0;
    if (const char *e = getenv("MIO_STREAM_PRIO")) {
        hipDeviceGetStreamPriorityRange(&least, &greatest);
        prio = std::string(e) == "high" ? greatest : std::string(e) == "low" ? least : 0;
    }
    if (hipStreamCreateWithPriority(&d->stream, hipStreamNonBlocking, prio) != hipSuccess) {
        delete d;
        mio::set_error("device_open: stream create failed");
        return MIO_ERR_HIP;
    }
    *out = d;
    return MIO_OK;
}

extern "C" void mio_hip_device_close(mio_hip_device *d) {
    if (!d) return;
    hipSetDevice(d->dev);
    if (d->stream) {
        hipStreamSynchronize(d->stream);
        hipStreamDestroy(d->stream);
    }
    delete d;
}

extern "C" int mio_hip_device_sync(mio_hip_device *d) {
    MIO_REQUIRE(d, MIO_ERR_INVALID, "device_sync: null");
    int rc = mio::bind(d);
    if (rc) return rc;
    MIO_HIP_CHECK(hipStreamSynchronize(d->stream));
    MIO_HIP_CHECK(hipDeviceSynchronize());
    return MIO_OK;
}

extern "C" int mio_hip_device_cu_count(const mio_hip_device *d, int *n_cu) {
    MIO_REQUIRE(d && n_cu, MIO_ERR_INVALID, "cu_count: null");
    *n_cu = d->n_cu;
    return MIO_OK;
}

extern "C" int mio_hip_malloc(mio_hip_device *d, size_t bytes, void **dptr) {
    MIO_REQUIRE(d && dptr, MIO_ERR_INVALID, "malloc: null");
    int rc = mio::bind(d);
    if (rc) return rc;
    if (hipMalloc(dptr, bytes ? bytes : 16) != hipSuccess) {
        mio::set_error("malloc: %zu bytes failed", bytes);
        return MIO_ERR_OOM;
    }
    return MIO_OK;
}

extern "C" int mio_hip_free(mio_hip_device *d, void *dptr) {
    MIO_REQUIRE(d, MIO_ERR_INVALID, "free: null");
    int rc = mio::bind(d);
    if (rc) return rc;
    if (dptr) MIO_HIP_CHECK(hipFree(dptr));
    return MIO_OK;
}

extern "C" int mio_hip_memcpy_h2d(mio_hip_device *d, void *dst, const void *src, size_t bytes) {
    MIO_REQUIRE(d && dst && src, MIO_ERR_INVALID, "memcpy_h2d: null");
    int rc = mio::bind(d);
    if (rc) return rc;
    MIO_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->stream));
    MIO_HIP_CHECK(hipStreamSynchronize(d->stream));
    return MIO_OK;
}

extern "C" int mio_hip_memcpy_d2h(mio_hip_device *d, void *dst, const void *src, size_t bytes) {
    MIO_REQUIRE(d && dst && src, MIO_ERR_INVALID, "memcpy_d2h: null");
    int rc = mio::bind(d);
    if (rc) return rc;
    MIO_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->stream));
    MIO_HIP_CHECK(hipStreamSynchronize(d->stream));
    return MIO_OK;
}

extern "C" int mio_hip_memset(mio_hip_device *d, void *dst, int value, size_t bytes) {
    MIO_REQUIRE(d && dst, MIO_ERR_INVALID, "memset: null");
    int rc = mio::bind(d);
    if (rc) return rc;
    MIO_HIP_CHECK(hipMemsetAsync(dst, value, bytes, d->stream));
    MIO_HIP_CHECK(hipStreamSynchronize(d->stream));
    return MIO_OK;
}

extern "C" int mio_hip_timer_mark(mio_hip_device *d, void *stream, int slot) {
    MIO_REQUIRE(d && slot >= 0 && slot < kTimerSlots && d->dev < 8, MIO_ERR_INVALID,
                "timer_mark: bad argument");
    int rc = mio::bind(d);
    if (rc) return rc;
    TimerBank &tb = g_timers[d->dev];
    if (!tb.ev[slot]) MIO_HIP_CHECK(hipEventCreate(&tb.ev[slot]));
    MIO_HIP_CHECK(hipEventRecord(tb.ev[slot], mio::pick_stream(d, stream)));
    return MIO_OK;
}

extern "C" int mio_hip_timer_elapsed(mio_hip_device *d, int a, int b, float *ms) {
    MIO_REQUIRE(d && ms && a >= 0 && b >= 0 && a < kTimerSlots && b < kTimerSlots && d->dev < 8,
                MIO_ERR_INVALID, "timer_elapsed: bad argument");
    int rc = mio::bind(d);
    if (rc) return rc;
    TimerBank &tb = g_timers[d->dev];
    MIO_REQUIRE(tb.ev[a] && tb.ev[b], MIO_ERR_INVALID, "timer_elapsed: slot not marked");
    MIO_HIP_CHECK(hipEventSynchronize(tb.ev[b]));
    MIO_HIP_CHECK(hipEventElapsedTime(ms, tb.ev[a], tb.ev[b]));
    return MIO_OK;
}
