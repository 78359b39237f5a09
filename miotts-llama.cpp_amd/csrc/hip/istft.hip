// iSTFT for gfx950: fused IRFFT (as an f32-MFMA GEMM against the reference's own
// float twiddles) + Hann window + gather-form overlap-add + /sum(w^2) + "same" trim,
// one launch, spectrogram in -> PCM out (no intermediate frames in HBM).
//
// Reference semantics (all cited from /root/reference/src/istft.cpp):
//   tables   :7-32   cos/sin of (2pi/N)*k*n computed in float, periodic Hann
//   irfft    :43-66  x[n] = (X0 + X_{N/2}(-1)^n + sum_k 2(Re cos - Im sin)) / N,
//                    Im(DC) and Im(Nyquist) ignored
//   OLA      :84-93  audio[t*hop+j] += y_t[j]*w[j]; wsum += w[j]^2  (ascending t)
//   normalise:95-99  divide where wsum > 1e-8
//   trim     :101-107 drop (win-hop)/2 samples at each end
// The OLA/normalise/trim arithmetic is performed in exactly the reference order
// (ascending frame index, same products); only the DFT inner sum is reordered
// (MFMA fma chain over k), which is the only source of difference vs istft.cpp.
//
// Tiling: a workgroup owns IST_M = 64 consecutive frames [t0, t0+64) and finalises
// the (64 - R) * hop output samples whose every contributing frame lies inside the
// tile (R = ceil(win/hop) - 1 halo frames are recomputed by the neighbour tile,
// 3/64 = 4.7% extra DFT work at hop = N/4). The DFT of the tile is
//   Y[64][N] = A[64][K] * B[K][N],  A = spec row with element 1 := Re(X_{N/2}),
//   B[0][n] = 1, B[1][n] = (-1)^n, B[2j][n] = 2cos, B[2j+1][n] = -2sin
// with K = 2*n_freq - 2 (= N for even N), on v_mfma_f32_32x32x2_f32 (exact f32
// fma chain, so the f32 parity budget is spent only on summation order). K is walked
// in IST_KC chunks through two LDS stages: chunk c+1 is loaded into registers before
// chunk c's MFMAs issue and stored to the other stage after them, one barrier per chunk.
#include "common.h"

#include <cmath>
#include <cstring>
#include <utility>
#include <vector>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int IST_M = 64;    // frames per tile
constexpr int IST_KC = 32;   // K chunk staged per iteration
constexpr int IST_ALD = IST_KC + 1;  // padded A row (conflict-free column reads)
constexpr int IST_THREADS = 256;
constexpr int IST_MAX_NT = 16;  // n-tiles of 32 -> n_fft <= 512
constexpr int IST_A_PER = IST_M * IST_KC / IST_THREADS;  // A floats per thread per chunk
// B float4s per thread per chunk and (frame half, n-tile) pairs per wave for NT n-tiles
template <int NT> constexpr int ist_b_per() { return (IST_KC * NT * 8 + IST_THREADS - 1) / IST_THREADS; }
template <int NT> constexpr int ist_pairs() { return (2 * NT + 3) / 4; }

struct IstftParams {
    const float *spec;   // [F][n_freq][2]
    float *out;          // [out_len]
    const float *basis;  // [Kp][NP]
    const float *hann;   // [win]
    int n_frames, n_fft, win, hop, n_freq, K, Kp, NP, R, S, n_out, n_pad;
    int hann_off;        // LDS float offset of the window copy (past stages and frames)
    float inv_n;
};

// One K chunk of the tile's operands held in registers while the previous chunk feeds
// the MFMAs (two LDS stages, one barrier per chunk).
template <int NT> struct IstftStage {
    float a[IST_A_PER];
    float4 b[ist_b_per<NT>()];
};

template <int NT>
__device__ __forceinline__ void istft_load(const IstftParams &p, int t0, int kc, int tid, IstftStage<NT> &st) {
    const int row_stride = p.n_freq * 2;
#pragma unroll
    for (int i = 0; i < IST_A_PER; ++i) {
        // k' -> spec element: k' (k' != 1), 2*(n_freq-1) for k' == 1.
        const int e = tid + i * IST_THREADS;
        const int f = t0 + e / IST_KC, k = kc + (e % IST_KC);
        float v = 0.0f;
        if (f >= 0 && f < p.n_frames && k < p.K) {
            const int src = (k == 1) ? 2 * (p.n_freq - 1) : k;
            v = p.spec[(size_t)f * row_stride + src];
        }
        st.a[i] = v;
    }
    const float4 *bsrc = reinterpret_cast<const float4 *>(p.basis + (size_t)kc * (NT * 32));
    constexpr int nb4 = IST_KC * NT * 8;
#pragma unroll
    for (int i = 0; i < ist_b_per<NT>(); ++i) {
        const int e = tid + i * IST_THREADS;
        st.b[i] = e < nb4 ? bsrc[e] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

template <int NT>
__device__ __forceinline__ void istft_store(float *stage, int tid, const IstftStage<NT> &st) {
    float *A_lds = stage;
    float4 *B_lds = reinterpret_cast<float4 *>(stage + IST_M * IST_ALD);
#pragma unroll
    for (int i = 0; i < IST_A_PER; ++i) {
        const int e = tid + i * IST_THREADS;
        A_lds[(e / IST_KC) * IST_ALD + (e % IST_KC)] = st.a[i];
    }
    constexpr int nb4 = IST_KC * NT * 8;
#pragma unroll
    for (int i = 0; i < ist_b_per<NT>(); ++i) {
        const int e = tid + i * IST_THREADS;
        if (nb4 % IST_THREADS == 0 || e < nb4) B_lds[e] = st.b[i];
    }
}

// NT = NP / 32 n-tiles is a template parameter so the pair loop below is branch-free: the
// LDS fragment reads of a K step are issued together ahead of its MFMAs.
template <int NT>
__global__ __launch_bounds__(IST_THREADS) void istft_fused_kernel(IstftParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int t0 = blockIdx.x * p.S - p.R;  // first frame of this tile (may be < 0)

    // The tile's (32-frame half m, 32-column n-tile) pairs are dealt round-robin to the
    // four waves: 2 * NT pairs, JP per wave (7/7/6/6 at n_fft = 392). A wave whose last
    // slot has no pair runs it on a clamped pair and drops the result: the block time is the
    // longest wave's either way.
    constexpr int NP = NT * 32;
    constexpr int JP = ist_pairs<NT>();
    constexpr int stage_floats = IST_M * IST_ALD + IST_KC * NP;
    int pm[JP], pn[JP];
#pragma unroll
    for (int j = 0; j < JP; ++j) {
        int pr = wave + 4 * j;
        if (pr >= 2 * NT) pr = 2 * NT - 1;
        pm[j] = pr >= NT;
        pn[j] = (pr - pm[j] * NT) * 32 + (lane & 31);
    }

    f32x16 acc[JP];
#pragma unroll
    for (int j = 0; j < JP; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;

    // window -> LDS once (the epilogue reads it ~4x per output sample)
    float *W = lds + p.hann_off;
    for (int i = tid; i < p.win; i += IST_THREADS) W[i] = p.hann[i];

    IstftStage<NT> st;
    istft_load<NT>(p, t0, 0, tid, st);
    istft_store<NT>(lds, tid, st);
    __syncthreads();
    int buf = 0;
    for (int kc = 0; kc < p.Kp; kc += IST_KC) {
        const bool more = kc + IST_KC < p.Kp;
        if (more) istft_load<NT>(p, t0, kc + IST_KC, tid, st);  // in flight under the MFMAs
        const float *A_lds = lds + buf * stage_floats;
        const float *B_lds = A_lds + IST_M * IST_ALD;
#pragma unroll
        for (int kk = 0; kk < IST_KC; kk += 2) {
            const int k = kk + (lane >> 5);
            const float a0 = A_lds[(lane & 31) * IST_ALD + k];
            const float a1 = A_lds[(32 + (lane & 31)) * IST_ALD + k];
#pragma unroll
            for (int j = 0; j < JP; ++j) {
                const float b = B_lds[k * NP + pn[j]];
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(pm[j] ? a1 : a0, b, acc[j], 0, 0, 0);
            }
        }
        if (more) istft_store<NT>(lds + (buf ^ 1) * stage_floats, tid, st);
        __syncthreads();
        buf ^= 1;
    }

    // Windowed frames -> LDS (reuses the staging area): y[f][n] = (sum * inv_n) * w[n]
    // (istft.cpp:65 then :91, same two roundings).
    float *Y = lds;  // [64][win]
#pragma unroll
    for (int j = 0; j < JP; ++j) {
        if (wave + 4 * j < 2 * NT) {
            const int m = pm[j];
            const int n = pn[j];
            if (n < p.win) {
                const float w = W[n];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const float v = acc[j][r] * p.inv_n;
                    Y[row * p.win + n] = v * w;
                }
            }
        }
    }
    __syncthreads();

    // Gather OLA for samples whose contributing frames all lie in this tile.
    const int s_begin = (t0 + p.R) * p.hop;
    int s_end = (t0 + IST_M) * p.hop;
    if (s_end > p.n_out) s_end = p.n_out;
    const int keep_lo = p.n_pad, keep_hi = p.n_out - p.n_pad;
    for (int n = s_begin + tid; n < s_end; n += IST_THREADS) {
        if (n < keep_lo || n >= keep_hi) continue;
        const int lo_num = n - p.win + 1;
        int tmin = lo_num <= 0 ? 0 : (lo_num + p.hop - 1) / p.hop;
        int tmax = n / p.hop;
        if (tmax > p.n_frames - 1) tmax = p.n_frames - 1;
        float a = 0.0f, ws = 0.0f;
        for (int t = tmin; t <= tmax; ++t) {
            const int jj = n - t * p.hop;
            const float w = W[jj];
            a += Y[(t - t0) * p.win + jj];
            ws += w * w;
        }
        if (ws > 1e-8f) a /= ws;
        p.out[n - p.n_pad] = a;
    }
}

template <int... I> const void *istft_kernel_pick(int nt, std::integer_sequence<int, I...>) {
    static const void *const tab[] = {(const void *)istft_fused_kernel<I + 1>...};
    return tab[nt - 1];
}
// n-tile count (1..IST_MAX_NT, checked by mio_hip_istft_create) -> kernel instantiation
const void *istft_kernel_for(int nt) {
    return istft_kernel_pick(nt, std::make_integer_sequence<int, IST_MAX_NT>());
}

}  // namespace

struct mio_hip_istft {
    mio_hip_device *d = nullptr;
    int n_fft = 0, win = 0, n_freq = 0, K = 0, Kp = 0, NP = 0;
    float *d_basis = nullptr, *d_hann = nullptr;
    float *d_in = nullptr, *d_out = nullptr;
    size_t in_cap = 0, out_cap = 0;
};

static int istft_geometry(const mio_hip_istft *h, int n_frames, int hop, int *n_out, int *n_pad,
                          int *out_len) {
    *n_out = (n_frames - 1) * hop + h->win;
    *n_pad = (h->win - hop) / 2;
    const int lo = *n_pad, hi = *n_out - *n_pad;
    *out_len = (n_frames > 0 && hi > lo) ? hi - lo : 0;
    return MIO_OK;
}

extern "C" int mio_hip_istft_create(mio_hip_device *d, int n_fft, int win_length,
                                    mio_hip_istft **out) {
    MIO_REQUIRE(d && out, MIO_ERR_INVALID, "istft_create: null argument");
    MIO_REQUIRE(n_fft >= 2 && n_fft <= 32 * IST_MAX_NT, MIO_ERR_UNSUPPORTED,
                "istft_create: n_fft %d outside [2, %d]", n_fft, 32 * IST_MAX_NT);
    MIO_REQUIRE(win_length >= 1 && win_length <= n_fft, MIO_ERR_UNSUPPORTED,
                "istft_create: win_length %d must be in [1, n_fft]", win_length);
    int rc = mio::bind(d);
    if (rc) return rc;
    auto *h = new mio_hip_istft();
    h->d = d;
    h->n_fft = n_fft;
    h->win = win_length;
    h->n_freq = n_fft / 2 + 1;
    const int n_mid = h->n_freq - 2 > 0 ? h->n_freq - 2 : 0;
    h->K = 2 * h->n_freq - 2;
    h->Kp = (h->K + IST_KC - 1) / IST_KC * IST_KC;
    h->NP = (n_fft + 31) / 32 * 32;

    // Float tables exactly as istft.cpp:17-31 computes them.
    const float two_pi_over_n = 2.0f * (float)M_PI / (float)n_fft;
    std::vector<float> basis((size_t)h->Kp * h->NP, 0.0f), hann(win_length);
    for (int n = 0; n < n_fft; n++) {
        basis[(size_t)0 * h->NP + n] = 1.0f;
        basis[(size_t)1 * h->NP + n] = (n & 1) ? -1.0f : 1.0f;
        for (int k = 1; k <= n_mid; k++) {
            const float w = two_pi_over_n * (float)k * (float)n;
            basis[(size_t)(2 * k) * h->NP + n] = 2.0f * cosf(w);
            basis[(size_t)(2 * k + 1) * h->NP + n] = -2.0f * sinf(w);
        }
    }
    for (int i = 0; i < win_length; i++)
        hann[i] = 0.5f * (1.0f - cosf(2.0f * (float)M_PI * i / win_length));

    if (hipMalloc(&h->d_basis, basis.size() * 4) != hipSuccess ||
        hipMalloc(&h->d_hann, hann.size() * 4) != hipSuccess) {
        mio::set_error("istft_create: hipMalloc failed");
        mio_hip_istft_destroy(h);
        return MIO_ERR_OOM;
    }
    if (hipMemcpy(h->d_basis, basis.data(), basis.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->d_hann, hann.data(), hann.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        mio::set_error("istft_create: upload failed");
        mio_hip_istft_destroy(h);
        return MIO_ERR_HIP;
    }
    // the 160 KB LDS opt-in applies to the current device: set it for every handle (once per
    // create, cheap), so a second device in the same process gets it too
    if (hipFuncSetAttribute(istft_kernel_for(h->NP / 32), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess) {
        mio::set_error("istft_create: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
        mio_hip_istft_destroy(h);
        return MIO_ERR_HIP;
    }
    *out = h;
    return MIO_OK;
}

extern "C" void mio_hip_istft_destroy(mio_hip_istft *h) {
    if (!h) return;
    if (h->d) hipSetDevice(h->d->dev);
    if (h->d_basis) hipFree(h->d_basis);
    if (h->d_hann) hipFree(h->d_hann);
    if (h->d_in) hipFree(h->d_in);
    if (h->d_out) hipFree(h->d_out);
    delete h;
}

extern "C" int mio_hip_istft_out_len(const mio_hip_istft *h, int n_frames, int hop_length,
                                     int *out_len) {
    MIO_REQUIRE(h && out_len && hop_length > 0 && n_frames >= 0, MIO_ERR_INVALID,
                "istft_out_len: bad argument");
    int n_out, n_pad;
    return istft_geometry(h, n_frames, hop_length, &n_out, &n_pad, out_len);
}

// Device-pointer launch used by the codec pipeline as well (no sync, no allocation).
int mio_istft_launch_device(mio_hip_istft *h, const float *d_spec, int n_frames, int hop,
                            float *d_out, hipStream_t s) {
    int n_out, n_pad, out_len;
    istft_geometry(h, n_frames, hop, &n_out, &n_pad, &out_len);
    if (out_len <= 0) return MIO_OK;
    IstftParams p;
    p.spec = d_spec;
    p.out = d_out;
    p.basis = h->d_basis;
    p.hann = h->d_hann;
    p.n_frames = n_frames;
    p.n_fft = h->n_fft;
    p.win = h->win;
    p.hop = hop;
    p.n_freq = h->n_freq;
    p.K = h->K;
    p.Kp = h->Kp;
    p.NP = h->NP;
    p.R = (h->win + hop - 1) / hop - 1;
    p.S = IST_M - p.R;
    p.n_out = n_out;
    p.n_pad = n_pad;
    p.inv_n = 1.0f / (float)h->n_fft;
    MIO_REQUIRE(p.S >= 1, MIO_ERR_UNSUPPORTED, "istft: hop %d too small for win %d", hop, h->win);
    const int span = p.S * hop;
    const int grid = (n_out + span - 1) / span;
    size_t lds_stage = (size_t)2 * (IST_M * IST_ALD + IST_KC * p.NP) * 4;  // two stages
    size_t lds_frames = (size_t)IST_M * p.win * 4;
    size_t lds = lds_stage > lds_frames ? lds_stage : lds_frames;
    p.hann_off = (int)(lds / 4);
    lds += (size_t)p.win * 4;
    void *args[] = {&p};
    MIO_HIP_CHECK(hipLaunchKernel(istft_kernel_for(p.NP / 32), dim3(grid), dim3(IST_THREADS), args, lds, s));
    return MIO_OK;
}

extern "C" int mio_hip_istft_run(mio_hip_istft *h, const float *spec, int n_frames,
                                 int hop_length, float *out, int *out_len, unsigned flags,
                                 void *stream) {
    MIO_REQUIRE(h && hop_length > 0 && n_frames >= 0, MIO_ERR_INVALID, "istft_run: bad argument");
    int rc = mio::bind(h->d);
    if (rc) return rc;
    hipStream_t s = mio::pick_stream(h->d, stream);
    int n_out, n_pad, len;
    istft_geometry(h, n_frames, hop_length, &n_out, &n_pad, &len);
    if (out_len) *out_len = len;
    if (len <= 0) return MIO_OK;
    MIO_REQUIRE(spec && out, MIO_ERR_INVALID, "istft_run: null buffer");

    const float *d_spec = spec;
    float *d_out = out;
    const size_t in_bytes = (size_t)n_frames * h->n_freq * 2 * 4;
    const size_t out_bytes = (size_t)len * 4;
    if (!(flags & MIO_IN_DEVICE)) {
        if (in_bytes > h->in_cap) {
            if (h->d_in) hipFree(h->d_in);
            h->d_in = nullptr;
            MIO_HIP_CHECK(hipMalloc(&h->d_in, in_bytes));
            h->in_cap = in_bytes;
        }
        MIO_HIP_CHECK(hipMemcpyAsync(h->d_in, spec, in_bytes, hipMemcpyHostToDevice, s));
        d_spec = h->d_in;
    }
    if (!(flags & MIO_OUT_DEVICE)) {
        if (out_bytes > h->out_cap) {
            if (h->d_out) hipFree(h->d_out);
            h->d_out = nullptr;
            MIO_HIP_CHECK(hipMalloc(&h->d_out, out_bytes));
            h->out_cap = out_bytes;
        }
        d_out = h->d_out;
    }
    rc = mio_istft_launch_device(h, d_spec, n_frames, hop_length, d_out, s);
    if (rc) return rc;
    if (!(flags & MIO_OUT_DEVICE)) {
        MIO_HIP_CHECK(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s));
        MIO_HIP_CHECK(hipStreamSynchronize(s));
    }
    return MIO_OK;
}
