// Single-token LLM decode step for gfx950 (replaces llama_decode for one token,
// test-to-speech.cpp:178-185 / :589-596, and the sampler chain :127-130, :165-166).
//
// Per layer, five launches, every one of them streaming its weights exactly once:
//   k_attn_in   RMSNorm(x) -> act re-quantized in LDS (Q8_K / Q8_0, ggml vec_dot_type)
//               -> fused q|k|v dequant-matvec
//   k_attention per (kv head, 64-position split): q/k RMSNorm (qwen3) + RoPE, F16 KV-cache
//               append by the split that owns `pos`, online-softmax partials
//   k_attn_out  split combine -> re-quantize -> O matvec -> x += .
//   k_ffn_in    RMSNorm(x) -> re-quantize -> gate & up matvec -> silu(g)*u
//   k_ffn_down  re-quantize h -> down matvec -> x += .
// then k_final_norm, k_lm_head (logits + per-block Gumbel-max), k_sample (token,
// next embedding, position++). All state is device-resident (StepState), so one hipGraph
// of a step replays every token with no host round trip.
//
// Matvec arithmetic = ggml's integer block dots: per superblock the integer sums
// (v_dot4c_i32_i8 on the raw 4/6/8-bit codes x int8 activations) are bit-exact with
// ggml vec_dot_{q4_K,q6_K}_q8_K / vec_dot_q8_0_q8_0; only the float sum over blocks is
// reordered. Weight streams are 16 B per lane, one contiguous run per row (split layout,
// csrc/host/quant.h).
#include "llm_kernels.h"

#include <cfloat>
#include <climits>

#pragma clang fp contract(off)

namespace mio {
namespace {

constexpr int NT = 256;
constexpr int NWAVE = NT / 64;

__device__ __forceinline__ float h2f(uint32_t bits16) {
    const uint16_t b = (uint16_t)bits16;
    return (float)__builtin_bit_cast(_Float16, b);
}
__device__ __forceinline__ float f16r(float f) { return (float)(_Float16)f; }
__device__ __forceinline__ int sdot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }
__device__ __forceinline__ uint4 ld16(const uint8_t *p) { return *reinterpret_cast<const uint4 *>(p); }

// ------------------------------------------------------------------ activation in LDS
struct ActL {
    int8_t *qs;
    float *d;
    int16_t *bs;
};

struct Smem {
    float *xs;   // [K] float staging
    ActL a;
    double *red; // [NWAVE]
};

__host__ __device__ inline size_t smem_bytes(int K) {
    return (size_t)K * 4 + (size_t)K + (size_t)(K / 32 + 8) * 4 + (size_t)(K / 16 + 8) * 2 + 64;
}

__device__ inline Smem carve(char *base, int K) {
    Smem s;
    s.xs = (float *)base;
    s.a.qs = (int8_t *)(base + (size_t)K * 4);
    s.a.d = (float *)(base + (size_t)K * 5);
    s.a.bs = (int16_t *)(base + (size_t)K * 5 + (size_t)(K / 32 + 8) * 4);
    s.red = (double *)(base + smem_bytes(K) - 64);
    return s;
}

__device__ double block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) t += red[w];
    __syncthreads();
    return t;
}

// ggml_rms_norm + mul(weight): xs = (x * 1/sqrtf(mean(x^2) + eps)) * w
__device__ void rmsnorm_to(const float *x, const float *w, int K, float eps, const Smem &s) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < K; i += NT) {
        const float v = x[i];
        s.xs[i] = v;
        acc += (double)(v * v);
    }
    const double tot = block_sum(acc, s.red);
    const float mean = (float)(tot / K);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int i = threadIdx.x; i < K; i += NT) {
        const float v = s.xs[i] * scale;
        s.xs[i] = v * w[i];
    }
    __syncthreads();
}

// quantize_row_q8_K_ref semantics (iscale = -127/max_signed, nearest-even, clamp 127, bsums)
__device__ void quant_q8k(const float *xs, int K, const ActL &a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int b = wave; b < K / 256; b += NWAVE) {
        float v[4];
        float am = -1.0f;
        int ai = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[i] = xs[b * 256 + 4 * lane + i];
            const float t = fabsf(v[i]);
            if (t > am) am = t, ai = 4 * lane + i;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float om = __shfl_xor(am, o);
            const int oi = __shfl_xor(ai, o);
            if (om > am || (om == am && oi < ai)) am = om, ai = oi;
        }
        int q[4] = {0, 0, 0, 0};
        float dd = 0.0f;
        if (am > 0.0f) {
            const float mx = xs[b * 256 + ai];
            const float iscale = -127.f / mx;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int t = (int)rintf(iscale * v[i]);
                q[i] = t < 127 ? t : 127;
            }
            dd = 1.0f / iscale;
        }
        const int packed = (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
        *reinterpret_cast<int *>(a.qs + b * 256 + 4 * lane) = packed;
        int sm = q[0] + q[1] + q[2] + q[3];
        sm += __shfl_xor(sm, 1);
        sm += __shfl_xor(sm, 2);
        if ((lane & 3) == 0) a.bs[b * 16 + (lane >> 2)] = (int16_t)sm;
        if (lane == 0) a.d[b] = dd;
    }
}

// quantize_row_q8_0_ref semantics (d = amax/127 stored as f16, q = roundf(x * 1/d))
__device__ void quant_q80(const float *xs, int K, const ActL &a) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = K / 32;
    for (int b0 = wave * 8; b0 < nb; b0 += NWAVE * 8) {
        const int b = b0 + (lane >> 3);
        const bool ok = b < nb;
        float v[4];
        float am = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[i] = ok ? xs[b * 32 + 4 * (lane & 7) + i] : 0.0f;
            am = fmaxf(am, fabsf(v[i]));
        }
        am = fmaxf(am, __shfl_xor(am, 1));
        am = fmaxf(am, __shfl_xor(am, 2));
        am = fmaxf(am, __shfl_xor(am, 4));
        const float dd = am / 127.0f;
        const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
        int q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = (int)roundf(v[i] * id);
        if (ok) {
            *reinterpret_cast<int *>(a.qs + b * 32 + 4 * (lane & 7)) =
                (q[0] & 0xFF) | ((q[1] & 0xFF) << 8) | ((q[2] & 0xFF) << 16) | ((q[3] & 0xFF) << 24);
            if ((lane & 7) == 0) a.d[b] = f16r(dd);
        }
    }
}

__device__ inline void quantize(const float *xs, int K, bool kquant, const ActL &a) {
    if (kquant)
        quant_q8k(xs, K, a);
    else
        quant_q80(xs, K, a);
    __syncthreads();
}

// ------------------------------------------------------------------ row dots (one wave)
// A row's quant payload for one "pass" (8 superblocks = 2048 weights for K-quants, 64
// blocks = 2048 weights for Q8_0) is one 16-B-per-lane load (+ headers); loads are issued
// into Frags BEFORE the activation prologue so HBM latency overlaps the RMSNorm/quantize.
__device__ inline int sbyte(const uint4 &h, int i) {
    const uint32_t w = i < 4 ? h.y : (i < 8 ? h.z : h.w);
    return (int)((w >> ((i & 3) * 8)) & 0xFF);
}

__device__ inline void scale_min_k4(int j, const uint4 &h, int &sc, int &m) {
    if (j < 4) {
        sc = sbyte(h, j) & 63;
        m = sbyte(h, j + 4) & 63;
    } else {
        sc = (sbyte(h, j + 4) & 0xF) | ((sbyte(h, j - 4) >> 6) << 4);
        m = (sbyte(h, j + 4) >> 4) | ((sbyte(h, j) >> 6) << 4);
    }
}

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

constexpr uint32_t M4 = 0x0F0F0F0Fu, M2 = 0x03030303u;

struct Frag {
    uint4 a, b;
    int c, d;
    uint32_t e;
};

__device__ inline int npass_of(const QMat &W) {
    return W.type == 8 ? ((W.k >> 5) + 63) / 64 : ((W.k >> 8) + 7) / 8;
}

__device__ inline Frag load_frag(const QMat &W, int row, int pass) {
    const int lane = threadIdx.x & 63;
    Frag f;
    f.a = f.b = make_uint4(0, 0, 0, 0);
    f.c = f.d = 0;
    f.e = 0;
    if (row < 0) return f;
    if (W.type == 12) {
        const int nsb = W.k >> 8, sb = pass * 8 + (lane >> 3), pc = lane & 7;
        if (sb < nsb) {
            f.a = ld16(W.p0 + (size_t)row * (W.k / 2) + sb * 128 + pc * 16);
            f.b = ld16(W.p1 + ((size_t)row * nsb + sb) * 16);
        }
    } else if (W.type == 14) {
        const int nsb = W.k >> 8, sb = pass * 8 + (lane >> 3), pc = lane & 7;
        if (sb < nsb) {
            const int n = pc >> 2, qq = pc & 3, gl = qq >> 1, l0 = 16 * (qq & 1);
            f.a = ld16(W.p0 + (size_t)row * (W.k / 2) + sb * 128 + pc * 16);
            f.b = ld16(W.p1 + (size_t)row * (W.k / 4) + sb * 64 + 32 * n + l0);
            const int8_t *sc = (const int8_t *)W.p2 + (size_t)row * (W.k / 16) + sb * 16 + 8 * n + 2 * gl + (l0 >> 4);
            f.c = sc[0];
            f.d = sc[4];
            f.e = ((const uint16_t *)W.p3)[(size_t)row * nsb + sb];
        }
    } else {
        const int nb = W.k >> 5, b = pass * 64 + lane;
        if (b < nb) {
            const uint8_t *p = W.p0 + (size_t)row * W.k + 32 * b;
            f.a = ld16(p);
            f.b = ld16(p + 16);
            f.e = ((const uint16_t *)W.p1)[(size_t)row * nb + b];
        }
    }
    return f;
}

// This lane's share of the row dot for one pass (summed over lanes by the caller).
// Integer parts per superblock / block are exact (ggml vec_dot semantics).
__device__ inline float compute_frag(const QMat &W, const Frag &f, int pass, const ActL &a) {
    const int lane = threadIdx.x & 63;
    if (W.type == 12) {
        const int nsb = W.k >> 8, sb = pass * 8 + (lane >> 3), pc = lane & 7, jj = pc >> 1, hh = pc & 1;
        const bool ok = sb < nsb;
        const int sbc = ok ? sb : 0;
        const int e_lo = sbc * 256 + 64 * jj + 16 * hh;
        const int4 alo = *reinterpret_cast<const int4 *>(a.qs + e_lo);
        const int4 ahi = *reinterpret_cast<const int4 *>(a.qs + e_lo + 32);
        int dlo = 0, dhi = 0;
        dlo = sdot4((int)(f.a.x & M4), alo.x, dlo);
        dlo = sdot4((int)(f.a.y & M4), alo.y, dlo);
        dlo = sdot4((int)(f.a.z & M4), alo.z, dlo);
        dlo = sdot4((int)(f.a.w & M4), alo.w, dlo);
        dhi = sdot4((int)((f.a.x >> 4) & M4), ahi.x, dhi);
        dhi = sdot4((int)((f.a.y >> 4) & M4), ahi.y, dhi);
        dhi = sdot4((int)((f.a.z >> 4) & M4), ahi.z, dhi);
        dhi = sdot4((int)((f.a.w >> 4) & M4), ahi.w, dhi);
        int sc0, m0, sc1, m1;
        scale_min_k4(2 * jj, f.b, sc0, m0);
        scale_min_k4(2 * jj + 1, f.b, sc1, m1);
        int isum = sc0 * dlo + sc1 * dhi;
        int imin = m0 * a.bs[e_lo >> 4] + m1 * a.bs[(e_lo + 32) >> 4];
        isum += __shfl_xor(isum, 1);
        isum += __shfl_xor(isum, 2);
        isum += __shfl_xor(isum, 4);
        imin += __shfl_xor(imin, 1);
        imin += __shfl_xor(imin, 2);
        imin += __shfl_xor(imin, 4);
        if (!(ok && pc == 0)) return 0.0f;
        const float da = a.d[sbc];
        const float d = h2f(f.b.x & 0xFFFF) * da;
        const float dmin = h2f(f.b.x >> 16) * da;
        float v = d * (float)isum;
        v = v - dmin * (float)imin;
        return v;
    } else if (W.type == 14) {
        const int nsb = W.k >> 8, sb = pass * 8 + (lane >> 3), pc = lane & 7;
        const int n = pc >> 2, qq = pc & 3, gl = qq >> 1, l0 = 16 * (qq & 1);
        const bool ok = sb < nsb;
        const int sbc = ok ? sb : 0;
        const int e_lo = sbc * 256 + 128 * n + 32 * gl + l0;
        const int4 alo = *reinterpret_cast<const int4 *>(a.qs + e_lo);
        const int4 ahi = *reinterpret_cast<const int4 *>(a.qs + e_lo + 64);
        const int shl = 2 * gl, shh = 2 * gl + 4;
        auto lo = [&](uint32_t l, uint32_t h) { return (int)((l & M4) | (((h >> shl) & M2) << 4)); };
        auto hi = [&](uint32_t l, uint32_t h) { return (int)(((l >> 4) & M4) | (((h >> shh) & M2) << 4)); };
        int dlo = 0, dhi = 0;
        dlo = sdot4(lo(f.a.x, f.b.x), alo.x, dlo);
        dlo = sdot4(lo(f.a.y, f.b.y), alo.y, dlo);
        dlo = sdot4(lo(f.a.z, f.b.z), alo.z, dlo);
        dlo = sdot4(lo(f.a.w, f.b.w), alo.w, dlo);
        dhi = sdot4(hi(f.a.x, f.b.x), ahi.x, dhi);
        dhi = sdot4(hi(f.a.y, f.b.y), ahi.y, dhi);
        dhi = sdot4(hi(f.a.z, f.b.z), ahi.z, dhi);
        dhi = sdot4(hi(f.a.w, f.b.w), ahi.w, dhi);
        int isum = f.c * (dlo - 32 * a.bs[e_lo >> 4]) + f.d * (dhi - 32 * a.bs[(e_lo + 64) >> 4]);
        isum += __shfl_xor(isum, 1);
        isum += __shfl_xor(isum, 2);
        isum += __shfl_xor(isum, 4);
        if (!(ok && pc == 0)) return 0.0f;
        const float d = h2f(f.e) * a.d[sbc];
        return d * (float)isum;
    } else {
        const int nb = W.k >> 5, b = pass * 64 + lane;
        if (b >= nb) return 0.0f;
        const int4 a0 = *reinterpret_cast<const int4 *>(a.qs + 32 * b);
        const int4 a1 = *reinterpret_cast<const int4 *>(a.qs + 32 * b + 16);
        int s = 0;
        s = sdot4((int)f.a.x, a0.x, s);
        s = sdot4((int)f.a.y, a0.y, s);
        s = sdot4((int)f.a.z, a0.z, s);
        s = sdot4((int)f.a.w, a0.w, s);
        s = sdot4((int)f.b.x, a1.x, s);
        s = sdot4((int)f.b.y, a1.y, s);
        s = sdot4((int)f.b.z, a1.z, s);
        s = sdot4((int)f.b.w, a1.w, s);
        return (float)s * (h2f(f.e) * a.d[b]);
    }
}

// NR rows of W, all passes. PRE = passes whose loads were issued before the prologue
// (pre[r][p], p < PRE); remaining passes are loaded one pass ahead.
template <int NR, int PMAX>
__device__ inline void preload(const QMat &W, const int (&rows)[NR], Frag (&pre)[NR][PMAX]) {
    const int np = npass_of(W);
#pragma unroll
    for (int p = 0; p < PMAX; ++p)
#pragma unroll
        for (int r = 0; r < NR; ++r)
            if (p < np) pre[r][p] = load_frag(W, rows[r], p);
}

template <int NR, int PMAX>
__device__ inline void finish_rows(const QMat &W, const int (&rows)[NR], const Frag (&pre)[NR][PMAX],
                                   const ActL &a, float (&out)[NR]) {
    const int np = npass_of(W);
    float acc[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int p = 0; p < PMAX; ++p)
#pragma unroll
        for (int r = 0; r < NR; ++r)
            if (p < np) acc[r] += compute_frag(W, pre[r][p], p, a);
    if (np > PMAX) {
        Frag cur[NR], nxt[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) cur[r] = load_frag(W, rows[r], PMAX);
        for (int p = PMAX; p < np; ++p) {
#pragma unroll
            for (int r = 0; r < NR; ++r)
                if (p + 1 < np) nxt[r] = load_frag(W, rows[r], p + 1);
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r] += compute_frag(W, cur[r], p, a);
#pragma unroll
            for (int r = 0; r < NR; ++r) cur[r] = nxt[r];
        }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) out[r] = wave_sum(acc[r]);
}

// Registers for the prologue input vector: x loaded as float4 before the weight loads.
template <int XV>
struct XRegs {
    float4 v[XV];
};

template <int XV>
__device__ inline void load_x(const float *x, int K, XRegs<XV> &xr) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (threadIdx.x + i * NT) * 4;
        xr.v[i] = e < K ? *reinterpret_cast<const float4 *>(x + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// RMSNorm (ggml_rms_norm * weight) of the register copy into s.xs, then quantize.
template <int XV>
__device__ void rmsnorm_quant(const XRegs<XV> &xr, const float *w, int K, float eps, bool kquant, const Smem &s) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (threadIdx.x + i * NT) * 4;
        if (e < K) {
            const float4 v = xr.v[i];
            acc += (double)(v.x * v.x);
            acc += (double)(v.y * v.y);
            acc += (double)(v.z * v.z);
            acc += (double)(v.w * v.w);
        }
    }
    const double tot = block_sum(acc, s.red);
    const float mean = (float)(tot / K);
    const float scale = 1.0f / sqrtf(mean + eps);
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (threadIdx.x + i * NT) * 4;
        if (e < K) {
            const float4 v = xr.v[i];
            const float4 ww = *reinterpret_cast<const float4 *>(w + e);
            float t;
            t = v.x * scale, s.xs[e + 0] = t * ww.x;
            t = v.y * scale, s.xs[e + 1] = t * ww.y;
            t = v.z * scale, s.xs[e + 2] = t * ww.z;
            t = v.w * scale, s.xs[e + 3] = t * ww.w;
        }
    }
    __syncthreads();
    quantize(s.xs, K, kquant, s.a);
}

template <int XV>
__device__ inline void plain_quant(const XRegs<XV> &xr, int K, bool kquant, const Smem &s) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (threadIdx.x + i * NT) * 4;
        if (e < K) *reinterpret_cast<float4 *>(s.xs + e) = xr.v[i];
    }
    __syncthreads();
    quantize(s.xs, K, kquant, s.a);
}

// Quantized activation blob in global memory (same carve layout) -> LDS.
__device__ inline void act_from_global(const float *blob, int K, const Smem &s) {
    const Smem gs = carve((char *)blob, K);
    for (int i = threadIdx.x; i < K / 4; i += NT) ((int *)s.a.qs)[i] = ((const int *)gs.a.qs)[i];
    for (int i = threadIdx.x; i < K / 32; i += NT) s.a.d[i] = gs.a.d[i];
    for (int i = threadIdx.x; i < K / 16; i += NT) s.a.bs[i] = gs.a.bs[i];
    __syncthreads();
}

// ------------------------------------------------------------------ kernels
constexpr int QKV_ROWS = 16;   // rows per workgroup (4 waves x NR=4)
constexpr int RES_ROWS = 8;    // O / down: 4 waves x NR=2
constexpr int FFN_PAIRS = 8;   // gate/up pairs per workgroup: 4 waves x NR=2
constexpr int LM_ROWS = 64;    // lm_head: 4 waves x 4 groups x NR=4

template <int P, int XV>
__global__ __launch_bounds__(NT) void k_attn_in(LlmDims d, const float *norm_w, QMat wq, QMat wk, QMat wv,
                                                LlmBuffers b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    XRegs<XV> xr;
    load_x(b.x, K, xr);
    int row0 = blockIdx.x * QKV_ROWS;
    const int seg = row0 >= wq.rows + wk.rows ? 2 : (row0 >= wq.rows ? 1 : 0);
    const QMat W = seg == 2 ? wv : (seg == 1 ? wk : wq);
    const int off = seg == 2 ? wq.rows + wk.rows : (seg == 1 ? wq.rows : 0);
    row0 -= off;
    float *out = b.qkv + off;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int rows[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) rows[r] = row0 + wave * 4 + r < W.rows ? row0 + wave * 4 + r : -1;
    Frag pre[4][P];
    preload<4, P>(W, rows, pre);
    rmsnorm_quant(xr, norm_w, K, d.eps, wq.type != 8, s);
    float o[4];
    finish_rows<4, P>(W, rows, pre, s.a, o);
    if (lane == 0)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (rows[r] >= 0) out[rows[r]] = o[r];
}

// Attention for one (kv head, split of d.split positions). HD = head dim.
template <int HD, int G>
__global__ __launch_bounds__(NT) void k_attention(LlmDims d, const float *q_norm, const float *k_norm,
                                                  _Float16 *kc, _Float16 *vc, LlmBuffers b) {
    constexpr int LP = HD / 8;          // lanes per position (8 dims each)
    constexpr int NS = NT / LP;         // position slots per workgroup
    constexpr int GMAX = G;
    __shared__ float qs[GMAX][HD];
    __shared__ float knew[HD], vnew[HD];
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *slot = (float *)smem;  // [NS][G][HD + 2]

    const int kvh = blockIdx.y, sp = blockIdx.x;
    const int pos = b.st->pos;
    const int t0 = sp * d.split;
    if (t0 > pos) return;
    const int t1 = min(t0 + d.split, pos + 1);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float2 *rope = b.rope + (size_t)pos * (HD / 2);

    // q (and, for the owner of `pos`, k/v): optional per-head RMSNorm, RoPE, f16 rounding
    auto prep = [&](const float *src, const float *nw, float *dst, bool round_f16) {
        // one wave, HD values
        float v[HD / 64 > 0 ? HD / 64 : 1];
        constexpr int PER = HD / 64;
        double ss = 0.0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            v[i] = src[lane + 64 * i];
            ss += (double)(v[i] * v[i]);
        }
        if (d.qk_norm) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
            const float mean = (float)(ss / HD);
            const float scale = 1.0f / sqrtf(mean + d.eps);
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const float t = v[i] * scale;
                v[i] = t * nw[lane + 64 * i];
            }
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) dst[lane + 64 * i] = v[i];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // rope: pair p (HD/2 pairs)
        float o0[PER], o1[PER];
        int i0s[PER], i1s[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int p = lane + 64 * i;
            i0s[i] = -1;
            if (p < HD / 2) {
                const int i0 = d.neox ? p : 2 * p, i1 = d.neox ? p + HD / 2 : 2 * p + 1;
                const float x0 = dst[i0], x1 = dst[i1];
                const float2 cs = rope[p];
                o0[i] = x0 * cs.x - x1 * cs.y;
                o1[i] = x0 * cs.y + x1 * cs.x;
                i0s[i] = i0, i1s[i] = i1;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int i = 0; i < PER; ++i)
            if (i0s[i] >= 0) {
                dst[i0s[i]] = round_f16 ? f16r(o0[i]) : o0[i];
                dst[i1s[i]] = round_f16 ? f16r(o1[i]) : o1[i];
            }
    };
    for (int g = wave; g < G; g += NWAVE)
        prep(b.qkv + (size_t)(kvh * G + g) * HD, q_norm, qs[g], true);
    const bool owner = pos >= t0 && pos < t0 + d.split;
    if (owner && wave == NWAVE - 1) {
        const float *kr = b.qkv + (size_t)d.n_head * HD + (size_t)kvh * HD;
        const float *vr = b.qkv + (size_t)(d.n_head + d.n_kv) * HD + (size_t)kvh * HD;
        prep(kr, k_norm, knew, true);
        __builtin_amdgcn_wave_barrier();
        _Float16 *kd = kc + ((size_t)kvh * d.n_ctx + pos) * HD;
        _Float16 *vd = vc + ((size_t)kvh * d.n_ctx + pos) * HD;
        for (int i = lane; i < HD; i += 64) {
            const float vv = f16r(vr[i]);
            vnew[i] = vv;
            kd[i] = (_Float16)knew[i];
            vd[i] = (_Float16)vv;
        }
    }
    __syncthreads();

    // main loop: LP lanes per position, 8 dims per lane, online softmax per q head
    const int lp = lane % LP;
    const int sl = tid / LP;
    float qv[GMAX][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) qv[g][i] = qs[g][lp * 8 + i];
    float m[GMAX], l[GMAX], acc[GMAX][8];
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
        m[g] = -INFINITY, l[g] = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[g][i] = 0.0f;
    }
    const _Float16 *kbase = kc + (size_t)kvh * d.n_ctx * HD;
    const _Float16 *vbase = vc + (size_t)kvh * d.n_ctx * HD;
    for (int t = t0 + sl; t < t1; t += NS) {
        float kf[8], vf[8];
        if (t == pos) {
#pragma unroll
            for (int i = 0; i < 8; ++i) kf[i] = knew[lp * 8 + i], vf[i] = vnew[lp * 8 + i];
        } else {
            typedef _Float16 h8 __attribute__((ext_vector_type(8)));
            const h8 kk = *reinterpret_cast<const h8 *>(kbase + (size_t)t * HD + lp * 8);
            const h8 vv = *reinterpret_cast<const h8 *>(vbase + (size_t)t * HD + lp * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) kf[i] = (float)kk[i], vf[i] = (float)vv[i];
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float sdot = 0.0f;
#pragma unroll
            for (int i = 0; i < 8; ++i) sdot = fmaf(qv[g][i], kf[i], sdot);
#pragma unroll
            for (int o = 1; o < LP; o <<= 1) sdot += __shfl_xor(sdot, o);
            const float sc = sdot * d.scale;
            const float mn = fmaxf(m[g], sc);
            const float c = expf(m[g] - mn);
            const float p = expf(sc - mn);
            l[g] = l[g] * c + p;
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[g][i] = acc[g][i] * c + p * vf[i];
            m[g] = mn;
        }
    }
    // slot partials -> LDS
    const int rec = HD + 2;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float *sp_ = slot + ((size_t)sl * G + g) * rec;
#pragma unroll
        for (int i = 0; i < 8; ++i) sp_[lp * 8 + i] = acc[g][i];
        if (lp == 0) sp_[HD] = m[g], sp_[HD + 1] = l[g];
    }
    __syncthreads();
    // combine slots: thread per (g, dim)
    for (int e = tid; e < G * HD; e += NT) {
        const int g = e / HD, dd = e - g * HD;
        float M = -INFINITY;
        for (int q = 0; q < NS; ++q) M = fmaxf(M, slot[((size_t)q * G + g) * rec + HD]);
        float L = 0.0f, O = 0.0f;
        for (int q = 0; q < NS; ++q) {
            const float *r = slot + ((size_t)q * G + g) * rec;
            const float w = r[HD] == -INFINITY ? 0.0f : expf(r[HD] - M);
            L += w * r[HD + 1];
            O += w * r[dd];
        }
        float *dst = b.part + ((size_t)(kvh * G + g) * d.max_splits + sp) * rec;
        dst[dd] = O;
        if (dd == 0) dst[HD] = M, dst[HD + 1] = L;
    }
}

template <int HD>
void launch_attention(int G, dim3 grid, size_t lds, hipStream_t s, const LlmDims &d, const float *qn,
                      const float *kn, _Float16 *kc, _Float16 *vc, const LlmBuffers &b) {
    switch (G) {
        case 1: hipLaunchKernelGGL((k_attention<HD, 1>), grid, dim3(NT), lds, s, d, qn, kn, kc, vc, b); break;
        case 2: hipLaunchKernelGGL((k_attention<HD, 2>), grid, dim3(NT), lds, s, d, qn, kn, kc, vc, b); break;
        case 3: hipLaunchKernelGGL((k_attention<HD, 3>), grid, dim3(NT), lds, s, d, qn, kn, kc, vc, b); break;
        case 4: hipLaunchKernelGGL((k_attention<HD, 4>), grid, dim3(NT), lds, s, d, qn, kn, kc, vc, b); break;
        case 8: hipLaunchKernelGGL((k_attention<HD, 8>), grid, dim3(NT), lds, s, d, qn, kn, kc, vc, b); break;
        default: break;
    }
}

// Split combine of the attention partials + re-quantization of the attention output
// (one workgroup per 256 outputs = one Q8_K block / eight Q8_0 blocks) -> global blob.
__global__ __launch_bounds__(NT) void k_attn_combine(LlmDims d, int kquant, LlmBuffers b) {
    __shared__ float xs[NT];
    __shared__ __attribute__((aligned(16))) int8_t qs[NT];
    __shared__ float dd[8];
    __shared__ int16_t bs[16];
    const int K = d.n_head * d.hd;
    const int pos = b.st->pos;
    const int nsp = pos / d.split + 1;
    const int rec = d.hd + 2;
    const int e = blockIdx.x * NT + threadIdx.x;
    const int ec = e < K ? e : K - 1;
    const int h = ec / d.hd, dd_ = ec - h * d.hd;
    const float *base = b.part + (size_t)h * d.max_splits * rec;
    float M = -INFINITY;
    for (int sp = 0; sp < nsp; ++sp) M = fmaxf(M, base[(size_t)sp * rec + d.hd]);
    float L = 0.0f, O = 0.0f;
    for (int sp = 0; sp < nsp; ++sp) {
        const float *r = base + (size_t)sp * rec;
        const float w = expf(r[d.hd] - M);
        L += w * r[d.hd + 1];
        O += w * r[dd_];
    }
    if (e >= K) O = 0.0f, L = 1.0f;
    xs[threadIdx.x] = O / L;
    __syncthreads();
    ActL a{qs, dd, bs};
    quantize(xs, NT, kquant != 0, a);
    const Smem gs = carve((char *)b.act2, K);
    if (threadIdx.x < NT / 4 && blockIdx.x * NT + 4 * threadIdx.x < K)
        ((int *)gs.a.qs)[blockIdx.x * (NT / 4) + threadIdx.x] = ((const int *)qs)[threadIdx.x];
    if (kquant) {
        if (threadIdx.x == 0) gs.a.d[blockIdx.x] = dd[0];
        if (threadIdx.x < 16) gs.a.bs[blockIdx.x * 16 + threadIdx.x] = bs[threadIdx.x];
    } else if (threadIdx.x < 8 && blockIdx.x * NT + 32 * threadIdx.x < K) {
        gs.a.d[blockIdx.x * 8 + threadIdx.x] = dd[threadIdx.x];
    }
}

template <int P, int XV>
__global__ __launch_bounds__(NT) void k_attn_out(LlmDims d, QMat wo, LlmBuffers b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_head * d.hd;
    const Smem s = carve(smem, K);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int rows[2];
    const int r0 = blockIdx.x * RES_ROWS + wave * 2;
    rows[0] = r0 < wo.rows ? r0 : -1;
    rows[1] = r0 + 1 < wo.rows ? r0 + 1 : -1;
    Frag pre[2][P];
    preload<2, P>(wo, rows, pre);
    act_from_global(b.act2, K, s);
    float o[2];
    finish_rows<2, P>(wo, rows, pre, s.a, o);
    if (lane == 0) {
        if (rows[0] >= 0) b.x[rows[0]] = o[0] + b.x[rows[0]];
        if (rows[1] >= 0) b.x[rows[1]] = o[1] + b.x[rows[1]];
    }
}

__device__ inline float silu_f(float x) { return x / (1.0f + expf(-x)); }

template <int P, int XV>
__global__ __launch_bounds__(NT) void k_ffn_in(LlmDims d, const float *norm_w, QMat gate, QMat up, LlmBuffers b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    XRegs<XV> xr;
    load_x(b.x, K, xr);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int rows[2];
    const int r0 = blockIdx.x * FFN_PAIRS + wave * 2;
    rows[0] = r0 < gate.rows ? r0 : -1;
    rows[1] = r0 + 1 < gate.rows ? r0 + 1 : -1;
    Frag pg[2][P], pu[2][P];
    preload<2, P>(gate, rows, pg);
    preload<2, P>(up, rows, pu);
    rmsnorm_quant(xr, norm_w, K, d.eps, gate.type != 8, s);
    float g[2], u[2];
    finish_rows<2, P>(gate, rows, pg, s.a, g);
    finish_rows<2, P>(up, rows, pu, s.a, u);
    if (lane == 0) {
        if (rows[0] >= 0) b.h[rows[0]] = silu_f(g[0]) * u[0];
        if (rows[1] >= 0) b.h[rows[1]] = silu_f(g[1]) * u[1];
    }
}

template <int P, int XV>
__global__ __launch_bounds__(NT) void k_ffn_down(LlmDims d, QMat down, LlmBuffers b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_ff;
    const Smem s = carve(smem, K);
    XRegs<XV> xr;
    load_x(b.h, K, xr);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int rows[2];
    const int r0 = blockIdx.x * RES_ROWS + wave * 2;
    rows[0] = r0 < down.rows ? r0 : -1;
    rows[1] = r0 + 1 < down.rows ? r0 + 1 : -1;
    Frag pre[2][P];
    preload<2, P>(down, rows, pre);
    plain_quant(xr, K, down.type != 8, s);
    float o[2];
    finish_rows<2, P>(down, rows, pre, s.a, o);
    if (lane == 0) {
        if (rows[0] >= 0) b.x[rows[0]] = o[0] + b.x[rows[0]];
        if (rows[1] >= 0) b.x[rows[1]] = o[1] + b.x[rows[1]];
    }
}

// final RMSNorm + re-quantization once per step -> global (read by every lm_head block)
template <int P, int XV>
__global__ __launch_bounds__(NT) void k_final_norm(LlmDims d, const float *norm_w, int kquant, LlmBuffers b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    XRegs<XV> xr;
    load_x(b.x, K, xr);
    rmsnorm_quant(xr, norm_w, K, d.eps, kquant != 0, s);
    const Smem gs = carve((char *)b.act, K);
    for (int i = threadIdx.x; i < K / 4; i += NT) ((int *)gs.a.qs)[i] = ((const int *)s.a.qs)[i];
    for (int i = threadIdx.x; i < K / 32; i += NT) gs.a.d[i] = s.a.d[i];
    for (int i = threadIdx.x; i < K / 16; i += NT) gs.a.bs[i] = s.a.bs[i];
}

__device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// same counter-based Gumbel noise as oracle/llm_ref.c mo_gumbel
__device__ inline float gumbel(uint64_t seed, int step, int idx) {
    const uint64_t h = mix64(seed ^ mix64(((uint64_t)(uint32_t)step << 32) | (uint32_t)idx));
    const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
    return -logf(-logf(u));
}

template <int P>
__global__ __launch_bounds__(NT) void k_lm_head(LlmDims d, QMat lm, SampleCfg sc, LlmBuffers b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float bs_[NWAVE];
    __shared__ int bi_[NWAVE];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int NG = LM_ROWS / (NWAVE * 4);
    const int rbase = blockIdx.x * LM_ROWS + wave * (LM_ROWS / NWAVE);
    int rows[NG][4];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) rows[g][r] = rbase + g * 4 + r < lm.rows ? rbase + g * 4 + r : -1;
    // lm_head rows are one pass at K <= 2048: load two groups ahead of the prologue
    Frag f0[4][P], f1[4][P];
    preload<4, P>(lm, rows[0], f0);
    preload<4, P>(lm, rows[1], f1);
    act_from_global(b.act, K, s);
    const int step = b.st->step;
    const uint64_t seed = ((uint64_t)sc.seed_hi << 32) | sc.seed_lo;
    float best = -INFINITY;
    int bi = INT_MAX;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        float o[4];
        if (g % 2 == 0) {
            finish_rows<4, P>(lm, rows[g], f0, s.a, o);
            if (g + 2 < NG) preload<4, P>(lm, rows[g + 2], f0);
        } else {
            finish_rows<4, P>(lm, rows[g], f1, s.a, o);
            if (g + 2 < NG) preload<4, P>(lm, rows[g + 2], f1);
        }
        if (lane == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = rows[g][r];
                if (row < 0) continue;
                b.logits[row] = o[r];
                if (row >= sc.lo && row < sc.hi) {
                    const float v = sc.temp > 0.0f ? o[r] / sc.temp + gumbel(seed, step, row) : o[r];
                    if (v > best || (v == best && row < bi)) best = v, bi = row;
                }
            }
        }
    }
    if (lane == 0) bs_[wave] = best, bi_[wave] = bi;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < NWAVE; ++w)
            if (bs_[w] > best || (bs_[w] == best && bi_[w] < bi)) best = bs_[w], bi = bi_[w];
        b.smp[2 * blockIdx.x] = best;
        b.smp[2 * blockIdx.x + 1] = __int_as_float(bi);
    }
}

__device__ float dequant_elem(const QMat &W, int row, int e) {
    if (W.type == 12) {
        const int nsb = W.k >> 8, sb = e >> 8, c = e & 255, j = c >> 6, w = c & 63, hi = w >> 5, l = w & 31;
        const uint8_t q = W.p0[(size_t)row * (W.k / 2) + sb * 128 + 32 * j + l];
        const uint4 hd = ld16(W.p1 + ((size_t)row * nsb + sb) * 16);
        int sc, m;
        scale_min_k4(2 * j + hi, hd, sc, m);
        const float d1 = h2f(hd.x & 0xFFFF) * sc, m1 = h2f(hd.x >> 16) * m;
        return d1 * (float)(hi ? (q >> 4) : (q & 0xF)) - m1;
    } else if (W.type == 14) {
        const int nsb = W.k >> 8, sb = e >> 8, c = e & 255, n = c >> 7, w = c & 127, g = w >> 5, l = w & 31;
        const uint8_t ql = W.p0[(size_t)row * (W.k / 2) + sb * 128 + 64 * n + l + 32 * (g & 1)];
        const uint8_t qh = W.p1[(size_t)row * (W.k / 4) + sb * 64 + 32 * n + l];
        const int q = (int)((g < 2 ? (ql & 0xF) : (ql >> 4)) | (((qh >> (2 * g)) & 3) << 4)) - 32;
        const int sc = ((const int8_t *)W.p2)[(size_t)row * (W.k / 16) + sb * 16 + (c >> 4)];
        const float dd = h2f(((const uint16_t *)W.p3)[(size_t)row * nsb + sb]);
        return dd * (float)sc * (float)q;
    } else {
        const int nb = W.k >> 5;
        const int8_t q = ((const int8_t *)W.p0)[(size_t)row * W.k + e];
        return (float)q * h2f(((const uint16_t *)W.p1)[(size_t)row * nb + (e >> 5)]);
    }
}

__global__ __launch_bounds__(NT) void k_sample(LlmDims d, SampleCfg sc, QMat emb, int nblk, LlmBuffers b) {
    __shared__ float bs_[NT];
    __shared__ int bi_[NT];
    __shared__ int tok_s;
    const int tid = threadIdx.x;
    const int step = b.st->step;
    float best = -INFINITY;
    int bi = INT_MAX;
    for (int i = tid; i < nblk; i += NT) {
        const float v = b.smp[2 * i];
        const int ix = __float_as_int(b.smp[2 * i + 1]);
        if (v > best || (v == best && ix < bi)) best = v, bi = ix;
    }
    bs_[tid] = best, bi_[tid] = bi;
    __syncthreads();
    for (int o = NT / 2; o > 0; o >>= 1) {
        if (tid < o) {
            const float v = bs_[tid + o];
            const int ix = bi_[tid + o];
            if (v > bs_[tid] || (v == bs_[tid] && ix < bi_[tid])) bs_[tid] = v, bi_[tid] = ix;
        }
        __syncthreads();
    }
    if (tid == 0) {
        int tok = bi_[0];
        if (tok == INT_MAX) tok = sc.lo;
        if (sc.force && step < sc.n_force && sc.force[step] >= 0) tok = sc.force[step];
        tok_s = tok;
    }
    __syncthreads();
    const int tok = tok_s;
    for (int e = tid; e < d.n_embd; e += NT) b.x[e] = dequant_elem(emb, tok, e);
    if (tid == 0) {
        if (step < sc.max_steps) sc.out_tokens[step] = tok;
        if (tok == sc.eos0 || tok == sc.eos1) b.st->done = 1;
        b.st->token = tok;
        b.st->pos = b.st->pos + 1;
        b.st->step = step + 1;
    }
}

__global__ void k_embed(LlmDims d, QMat emb, LlmBuffers b) {
    const int tok = b.st->token;
    for (int e = threadIdx.x; e < d.n_embd; e += blockDim.x) b.x[e] = dequant_elem(emb, tok, e);
}

}  // namespace

int lm_head_blocks(const LlmDims &d) { return (d.n_vocab + LM_ROWS - 1) / LM_ROWS; }

void launch_embed_token(const LlmDims &d, const QMat &tok_embd, const LlmBuffers &b, hipStream_t s) {
    hipLaunchKernelGGL(k_embed, dim3(1), dim3(NT), 0, s, d, tok_embd, b);
}

inline int pick_p(int K) { return (K + 2047) / 2048 <= 1 ? 1 : 3; }
inline int pick_xv(int K) {
    const int v = (K + 1023) / 1024;
    return v <= 1 ? 1 : (v <= 2 ? 2 : (v <= 6 ? 6 : 12));
}

// Calls F.template operator()<P, XV>() with P = passes preloaded, XV = float4 x-registers.
template <class F>
void dispatch_px(int K, F &&f) {
    const int p = pick_p(K), xv = pick_xv(K);
#define PX(PP, XX) \
    if (p == PP && xv == XX) return f.template operator()<PP, XX>();
    PX(1, 1) PX(1, 2) PX(1, 6) PX(1, 12) PX(3, 1) PX(3, 2) PX(3, 6) PX(3, 12)
#undef PX
}

// Launch one kernel of the step: which = 0 attn_in, 1 attention, 2 attn_out (with its
// combine kernel in front), 3 ffn_in, 4 ffn_down (layer il), 5 final_norm, 6 lm_head,
// 7 sample.
void launch_step_kernel(int which, const LlmDims &d, const LayerW *layers, int il, _Float16 *kcache,
                        _Float16 *vcache, const float *out_norm, const QMat &lm, const QMat &tok_embd,
                        const LlmBuffers &b, const SampleCfg &sc, hipStream_t s) {
    const size_t layer_kv = (size_t)d.n_kv * d.n_ctx * d.hd;
    const int G = d.n_head / d.n_kv;
    const int ns = NT / (d.hd / 8);
    const size_t att_lds = (size_t)ns * G * (d.hd + 2) * 4;
    const int nblk = lm_head_blocks(d);
    switch (which) {
        case 0: {
            const LayerW &L = layers[il];
            const int qkv_rows = L.wq.rows + L.wk.rows + L.wv.rows;
            dispatch_px(d.n_embd, [&]<int P, int XV>() {
                hipLaunchKernelGGL((k_attn_in<P, XV>), dim3((qkv_rows + QKV_ROWS - 1) / QKV_ROWS), dim3(NT),
                                   smem_bytes(d.n_embd), s, d, L.attn_norm, L.wq, L.wk, L.wv, b);
            });
            break;
        }
        case 1: {
            const LayerW &L = layers[il];
            if (d.hd == 128)
                launch_attention<128>(G, dim3(d.max_splits, d.n_kv), att_lds, s, d, L.q_norm, L.k_norm,
                                      kcache + il * layer_kv, vcache + il * layer_kv, b);
            else
                launch_attention<64>(G, dim3(d.max_splits, d.n_kv), att_lds, s, d, L.q_norm, L.k_norm,
                                     kcache + il * layer_kv, vcache + il * layer_kv, b);
            break;
        }
        case 2: {
            const LayerW &L = layers[il];
            const int K = d.n_head * d.hd;
            hipLaunchKernelGGL(k_attn_combine, dim3((K + NT - 1) / NT), dim3(NT), 0, s, d, L.wo.type != 8 ? 1 : 0, b);
            dispatch_px(K, [&]<int P, int XV>() {
                hipLaunchKernelGGL((k_attn_out<P, XV>), dim3((L.wo.rows + RES_ROWS - 1) / RES_ROWS), dim3(NT),
                                   smem_bytes(K), s, d, L.wo, b);
            });
            break;
        }
        case 3: {
            const LayerW &L = layers[il];
            dispatch_px(d.n_embd, [&]<int P, int XV>() {
                hipLaunchKernelGGL((k_ffn_in<P, XV>), dim3((L.gate.rows + FFN_PAIRS - 1) / FFN_PAIRS), dim3(NT),
                                   smem_bytes(d.n_embd), s, d, L.ffn_norm, L.gate, L.up, b);
            });
            break;
        }
        case 4: {
            const LayerW &L = layers[il];
            dispatch_px(d.n_ff, [&]<int P, int XV>() {
                hipLaunchKernelGGL((k_ffn_down<P, XV>), dim3((L.down.rows + RES_ROWS - 1) / RES_ROWS), dim3(NT),
                                   smem_bytes(d.n_ff), s, d, L.down, b);
            });
            break;
        }
        case 5:
            dispatch_px(d.n_embd, [&]<int P, int XV>() {
                hipLaunchKernelGGL((k_final_norm<P, XV>), dim3(1), dim3(NT), smem_bytes(d.n_embd), s, d, out_norm,
                                   lm.type != 8 ? 1 : 0, b);
            });
            break;
        case 6:
            if (pick_p(d.n_embd) == 1)
                hipLaunchKernelGGL(k_lm_head<1>, dim3(nblk), dim3(NT), smem_bytes(d.n_embd), s, d, lm, sc, b);
            else
                hipLaunchKernelGGL(k_lm_head<3>, dim3(nblk), dim3(NT), smem_bytes(d.n_embd), s, d, lm, sc, b);
            break;
        case 7: hipLaunchKernelGGL(k_sample, dim3(1), dim3(NT), 0, s, d, sc, tok_embd, nblk, b); break;
        default: break;
    }
}

void launch_decode_step(const LlmDims &d, const LayerW *layers, int n_layer, _Float16 *kcache,
                        _Float16 *vcache, const float *out_norm, const QMat &lm, const QMat &tok_embd,
                        const LlmBuffers &b, const SampleCfg &sc, hipStream_t s) {
    for (int il = 0; il < n_layer; ++il)
        for (int k = 0; k < 5; ++k) launch_step_kernel(k, d, layers, il, kcache, vcache, out_norm, lm, tok_embd, b, sc, s);
    for (int k = 5; k < 8; ++k) launch_step_kernel(k, d, layers, 0, kcache, vcache, out_norm, lm, tok_embd, b, sc, s);
}

}  // namespace mio

// ------------------------------------------------------------------ parity entry point
namespace mio {
namespace {
template <int P, int XV>
__global__ __launch_bounds__(NT) void k_debug_matvec(QMat W, const float *x, float *y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = W.k;
    const Smem s = carve(smem, K);
    XRegs<XV> xr;
    load_x(x, K, xr);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int rows[2];
    const int r0 = blockIdx.x * RES_ROWS + wave * 2;
    rows[0] = r0 < W.rows ? r0 : -1;
    rows[1] = r0 + 1 < W.rows ? r0 + 1 : -1;
    Frag pre[2][P];
    preload<2, P>(W, rows, pre);
    plain_quant(xr, K, W.type != 8, s);
    float o[2];
    finish_rows<2, P>(W, rows, pre, s.a, o);
    if (lane == 0) {
        if (rows[0] >= 0) y[rows[0]] = o[0];
        if (rows[1] >= 0) y[rows[1]] = o[1];
    }
}
}  // namespace

void launch_debug_matvec(const QMat &W, const float *x, float *y, hipStream_t s) {
    dispatch_px(W.k, [&]<int P, int XV>() {
        hipLaunchKernelGGL((k_debug_matvec<P, XV>), dim3((W.rows + RES_ROWS - 1) / RES_ROWS), dim3(NT), smem_bytes(W.k),
                           s, W, x, y);
    });
}
}  // namespace mio
