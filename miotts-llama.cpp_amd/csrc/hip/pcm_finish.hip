// PCM epilogue on the device: the optional peak normalisation of
// test-to-speech.cpp:232-243 (gain 0.95 / max|s| when max|s| > 1e-8) and the PCM16 sample
// conversion of wav-writer.cpp:24-44 (int16(clamp(s * 32767)), truncated toward zero), so a
// synthesized utterance leaves HBM as the WAV payload (2 B per sample instead of 4).
// Bit-exact with the host path (csrc/host/tts.cpp peak_normalize, text.cpp wav_bytes): the
// same float operations in the same order, no contraction.
//
// HBM-bound: 4 B read twice (peak pass, convert pass) + 2 B written per sample.
#include "common.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace {

constexpr int PT = 256;        // threads per workgroup
constexpr int MAX_PARTS = 1024;

// per-workgroup max|s| partials of the peak pass (one call at a time per device, like every
// handle of this ABI)
__device__ float g_peak_part[MAX_PARTS];

// NaN-ignoring max, as std::max(peak, fabs(s)) in peak_normalize (a NaN never replaces peak)
__device__ __forceinline__ float max_keep(float peak, float a) { return peak < a ? a : peak; }

__global__ __launch_bounds__(PT) void k_peak(const float *s, long long n) {
    __shared__ float red[PT / 64];
    float m = 0.0f;
    const long long n4 = n / 4;
    const float4 *s4 = reinterpret_cast<const float4 *>(s);
    for (long long i = blockIdx.x * (long long)PT + threadIdx.x; i < n4; i += (long long)gridDim.x * PT) {
        const float4 v = s4[i];
        m = max_keep(m, fabsf(v.x));
        m = max_keep(m, fabsf(v.y));
        m = max_keep(m, fabsf(v.z));
        m = max_keep(m, fabsf(v.w));
    }
    if (blockIdx.x == 0)
        for (long long i = n4 * 4 + threadIdx.x; i < n; i += PT) m = max_keep(m, fabsf(s[i]));
    for (int o = 32; o > 0; o >>= 1) m = max_keep(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int w = 1; w < PT / 64; ++w) r = max_keep(r, red[w]);
        g_peak_part[blockIdx.x] = r;
    }
}

// every workgroup reduces the partials itself (no third launch, no atomics), then converts
__global__ __launch_bounds__(PT) void k_pcm16(const float *s, long long n, int n_parts, int normalize,
                                              short *out, float *peak_out) {
    __shared__ float red[PT / 64];
    __shared__ float gain_s;
    __shared__ int scale_s;
    float gain = 1.0f;
    bool scale = false;
    if (normalize) {
        float m = 0.0f;
        for (int i = threadIdx.x; i < n_parts; i += PT) m = max_keep(m, g_peak_part[i]);
        for (int o = 32; o > 0; o >>= 1) m = max_keep(m, __shfl_xor(m, o));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            float r = red[0];
            for (int w = 1; w < PT / 64; ++w) r = max_keep(r, red[w]);
            if (peak_out && blockIdx.x == 0) *peak_out = r;
            scale_s = r > 1e-8f;
            gain_s = 0.95f / r;
        }
        __syncthreads();
        scale = scale_s != 0;
        gain = gain_s;
    }
    for (long long i = blockIdx.x * (long long)PT + threadIdx.x; i < n; i += (long long)gridDim.x * PT) {
        float v = s[i];
        if (scale) v = v * gain;
        const float t = v * 32767.0f;
        // std::min(32767, std::max(-32768, t)) with std::max/min's comparison order
        const float a = (-32768.0f < t) ? t : -32768.0f;
        const float c = (a < 32767.0f) ? a : 32767.0f;
        out[i] = (short)(int)c;
    }
}

}  // namespace

extern "C" int mio_hip_pcm_finish(mio_hip_device *d, const float *samples, int64_t n, int normalize,
                                  int16_t *pcm16, float *peak, void *stream) {
    MIO_REQUIRE(d && n >= 0, MIO_ERR_INVALID, "pcm_finish: bad argument");
    if (n == 0) {
        if (peak) *peak = 0.0f;
        return MIO_OK;
    }
    MIO_REQUIRE(samples && pcm16, MIO_ERR_INVALID, "pcm_finish: null buffer");
    MIO_REQUIRE(((uintptr_t)samples & 15) == 0, MIO_ERR_INVALID, "pcm_finish: samples must be 16-byte aligned");
    int rc = mio::bind(d);
    if (rc) return rc;
    hipStream_t s = mio::pick_stream(d, stream);
    const long long n4 = n / 4;
    int parts = (int)std::min<long long>(MAX_PARTS, std::max<long long>(1, (n4 + PT * 4 - 1) / (PT * 4)));
    float *d_peak = nullptr;
    if (normalize) {
        hipLaunchKernelGGL(k_peak, dim3(parts), dim3(PT), 0, s, samples, (long long)n);
        MIO_HIP_CHECK(hipGetLastError());
        if (peak) {
            MIO_HIP_CHECK(hipMallocAsync((void **)&d_peak, sizeof(float), s));
        }
    }
    const int grid = (int)std::min<long long>(4 * (long long)d->n_cu, std::max<long long>(1, (n + PT * 8 - 1) / (PT * 8)));
    hipLaunchKernelGGL(k_pcm16, dim3(grid), dim3(PT), 0, s, samples, (long long)n, parts, normalize,
                       reinterpret_cast<short *>(pcm16), d_peak);
    MIO_HIP_CHECK(hipGetLastError());
    if (peak) {
        if (d_peak) {
            MIO_HIP_CHECK(hipMemcpyAsync(peak, d_peak, sizeof(float), hipMemcpyDeviceToHost, s));
            MIO_HIP_CHECK(hipFreeAsync(d_peak, s));
            MIO_HIP_CHECK(hipStreamSynchronize(s));
        } else {
            *peak = 0.0f;  // not normalizing: no peak pass was run
        }
    }
    return MIO_OK;
}
