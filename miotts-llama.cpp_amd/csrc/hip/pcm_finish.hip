// PCM epilogue on the device: the optional peak normalisation of
// test-to-speech.cpp:232-243 (gain 0.95 / max|s| when max|s| > 1e-8) and the PCM16 sample
// conversion of wav-writer.cpp:24-44 (int16(clamp(s * 32767)), truncated toward zero), so a
// synthesized utterance leaves HBM as the WAV payload (2 B per sample instead of 4).
// Bit-exact with the host path (csrc/host/tts.cpp peak_normalize, text.cpp wav_bytes): the
// same float operations in the same order, no contraction.
//
// HBM-bound: 4 B read twice (peak pass, convert pass) + 2 B written per sample. Scratch (peak
// partials) is allocated per call, stream-ordered, so concurrent calls never share it.
#include "common.h"

#include <algorithm>
#include <type_traits>

#pragma clang fp contract(off)

namespace {

constexpr int PT = 256;        // threads per workgroup
constexpr int MAX_PARTS = 1024;

// NaN-ignoring max, as std::max(peak, fabs(s)) in peak_normalize (a NaN never replaces peak)
__device__ __forceinline__ float max_keep(float peak, float a) { return peak < a ? a : peak; }

// part[blockIdx.x] = this workgroup's max|s| (part: per-call stream-ordered scratch)
__global__ __launch_bounds__(PT) void k_peak(const float *s, long long n, float *part) {
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
        part[blockIdx.x] = r;
    }
}

// every workgroup reduces the partials itself (no third launch, no atomics), then converts:
// OutT short = the WAV sample (pcm16_sample), float = the normalised float sample (in place
// allowed: each element is read once, by the thread that writes it)
template <class OutT>
__global__ __launch_bounds__(PT) void k_finish(const float *s, long long n, const float *part, int n_parts,
                                               int normalize, OutT *out, float *peak_out) {
    __shared__ float red[PT / 64];
    __shared__ float gain_s;
    __shared__ int scale_s;
    float gain = 1.0f;
    bool scale = false;
    if (normalize) {
        float m = 0.0f;
        for (int i = threadIdx.x; i < n_parts; i += PT) m = max_keep(m, part[i]);
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
        if constexpr (std::is_same_v<OutT, short>)
            out[i] = mio::pcm16_sample(v);
        else
            out[i] = v;
    }
}

}  // namespace

namespace {
template <class OutT>
int finish(mio_hip_device *d, const float *samples, int64_t n, int normalize, OutT *out, float *peak,
           void *stream) {
    MIO_REQUIRE(d && n >= 0, MIO_ERR_INVALID, "pcm_finish: bad argument");
    if (n == 0) {
        if (peak) *peak = 0.0f;
        return MIO_OK;
    }
    MIO_REQUIRE(samples && out, MIO_ERR_INVALID, "pcm_finish: null buffer");
    MIO_REQUIRE(((uintptr_t)samples & 15) == 0, MIO_ERR_INVALID, "pcm_finish: samples must be 16-byte aligned");
    int rc = mio::bind(d);
    if (rc) return rc;
    hipStream_t s = mio::pick_stream(d, stream);
    const long long n4 = n / 4;
    int parts = (int)std::min<long long>(MAX_PARTS, std::max<long long>(1, (n4 + PT * 4 - 1) / (PT * 4)));
    // peak partials + the peak itself in stream-ordered scratch owned by this call: calls on
    // different streams (or handles) of one GPU never share it
    float *scratch = nullptr;
    if (normalize) {
        MIO_HIP_CHECK(hipMallocAsync((void **)&scratch, sizeof(float) * (parts + 1), s));
        hipLaunchKernelGGL(k_peak, dim3(parts), dim3(PT), 0, s, samples, (long long)n, scratch);
        MIO_HIP_CHECK(hipGetLastError());
    }
    float *d_peak = scratch && peak ? scratch + parts : nullptr;
    const int grid = (int)std::min<long long>(4 * (long long)d->n_cu, std::max<long long>(1, (n + PT * 8 - 1) / (PT * 8)));
    hipLaunchKernelGGL(k_finish<OutT>, dim3(grid), dim3(PT), 0, s, samples, (long long)n, scratch, parts, normalize,
                       out, d_peak);
    MIO_HIP_CHECK(hipGetLastError());
    if (d_peak) MIO_HIP_CHECK(hipMemcpyAsync(peak, d_peak, sizeof(float), hipMemcpyDeviceToHost, s));
    if (scratch) MIO_HIP_CHECK(hipFreeAsync(scratch, s));
    if (peak) {
        if (d_peak)
            MIO_HIP_CHECK(hipStreamSynchronize(s));
        else
            *peak = 0.0f;  // not normalizing: no peak pass was run
    }
    return MIO_OK;
}
}  // namespace

extern "C" int mio_hip_pcm_finish(mio_hip_device *d, const float *samples, int64_t n, int normalize,
                                  int16_t *pcm16, float *peak, void *stream) {
    return finish<short>(d, samples, n, normalize, reinterpret_cast<short *>(pcm16), peak, stream);
}

extern "C" int mio_hip_pcm_normalize(mio_hip_device *d, const float *samples, int64_t n, float *out,
                                     float *peak, void *stream) {
    return finish<float>(d, samples, n, 1, out, peak, stream);
}
