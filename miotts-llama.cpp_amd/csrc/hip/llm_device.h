// Device-side building blocks shared by the decode-step kernels (llm_kernels.hip) and
// the batched prompt prefill (llm_prefill.hip): DPP cross-lane reductions, ggml activation
// quantizers (Q8_K / Q8_0), the split-layout weight fragments and their integer block dots,
// and the streaming-rows matvec engine. Included by exactly those two translation units;
// everything lives in an anonymous namespace.
#pragma once

#include <cfloat>
#include <climits>
#include <type_traits>

#include "llm_kernels.h"

#pragma clang fp contract(off)

// Thread index used by every helper below.
#ifndef MIO_TIDX
#define MIO_TIDX threadIdx.x
#endif

namespace mio {
namespace {
// Diagnostics (checkpoint trace, step timeline) compile into a kernel only where kDiag is
// true: the decode kernels are instantiated twice (template flag DG, a local kDiag shadowing
// this default) and the step graph uses the DG = false ones, whose kernel-argument loads
// then issue together at entry (a diagnostic branch on a pointer argument serialized them
// into several scalar-load round trips before the first weight load).
constexpr bool kDiag = true;
// Checkpoint timestamps (s_memtime) of workgroup 0 / thread 0, only when b.trace is set
// (mio_hip_llm_trace_kernel); a uniform branch otherwise.
#define MIO_TRACE(bufs, k)                                                                    \
    do {                                                                                      \
        if (kDiag && (bufs).trace && blockIdx.x == 0 && blockIdx.y == 0 && MIO_TIDX == 0) { \
            asm volatile("" ::: "memory");                                                    \
            (bufs).trace[k] = __builtin_readcyclecounter();                                   \
            if ((k) == 0 || (k) == 15) (bufs).trace[16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                     \
    } while (0)

// Step timeline (diagnostic, mio_hip_llm_timeline): per workgroup of each launch {start,
// mark 1, mark 2, diagnostic marks 3-6, end}, s_memrealtime ticks (100 MHz), plain stores to
// slot [seq][wg][8] (wg < 512). Marks: matvec kernels 1 = weight loads issued, 2 = activations quantized;
// attention 1 = K/V loads issued, 2 = heads prepared; sampler 1 = token chosen.
#define MIO_TL_SLOT(bufs) ((bufs).tl + 8 * ((size_t)(bufs).seq * kTlSlots + ((blockIdx.x + blockIdx.y * gridDim.x) & (kTlSlots - 1))))
#define MIO_TL_AT(bufs, k)                                                                      \
    do {                                                                                        \
        if (kDiag && (bufs).tl && MIO_TIDX == 0) MIO_TL_SLOT(bufs)[k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#ifdef MIO_TL_DIAG
// diagnostic builds: mark 6 = the LAST wave's first instruction (wave launch skew)
#define MIO_TL_BEGIN(bufs)                                                                     \
    do {                                                                                       \
        MIO_TL_AT(bufs, 0);                                                                    \
        if (kDiag && (bufs).tl && MIO_TIDX == blockDim.x - 64) MIO_TL_SLOT(bufs)[6] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define MIO_TL_BEGIN(bufs) MIO_TL_AT(bufs, 0)
#endif
#ifdef MIO_TL_WAVES
#define MIO_TL_MARK(bufs, k)
#define MIO_TL_END(bufs)
#else
#define MIO_TL_MARK(bufs, k) MIO_TL_AT(bufs, k)
#define MIO_TL_END(bufs) MIO_TL_AT(bufs, 7)
#endif
// -DMIO_TL_DIAG: the prologue helpers also stamp marks 3-5 (activation consumed, reduced,
// staged; diagnostic builds only)
// and mark 1 becomes wave MIO_DIAG_WAVE's "activation consumed" (wave skew)
#ifndef MIO_DIAG_WAVE
#define MIO_DIAG_WAVE 7
#endif
#ifdef MIO_TL_DIAG
#define MIO_TL_DIAGSLOT(bufs) ((kDiag && (bufs).tl) ? MIO_TL_SLOT(bufs) : nullptr)
#define MIO_TL_MARK1(bufs)
#else
#define MIO_TL_DIAGSLOT(bufs) nullptr
#define MIO_TL_MARK1(bufs) MIO_TL_MARK(bufs, 1)
#endif
// stamp after value v is available (the empty asm consumes it; the timer read cannot move
// above a volatile asm)
#ifdef MIO_TL_WAVES
#define MIO_DIAG_STAMP(diag, k, v)
#else
#define MIO_DIAG_STAMP(diag, k, v)                                                   \
    do {                                                                             \
        if ((diag) && MIO_TIDX == 0) {                                            \
            asm volatile("" ::"v"(v));                                               \
            (diag)[k] = __builtin_amdgcn_s_memrealtime();                            \
        }                                                                            \
    } while (0)
#endif

constexpr int NT = 256;        // threads of the attention / sampler kernels
constexpr int NWAVE = NT / 64;
constexpr int MT = 512;        // threads of a streaming matvec workgroup
constexpr int MW = MT / 64;
constexpr int ATT_CHUNK = kAttChunk;
__host__ __device__ constexpr int part_rec(int hd) { return hd + 4; }  // partial record {O[hd], m, l, pad}

__device__ __forceinline__ float h2f(uint32_t bits16) {
    const uint16_t b = (uint16_t)bits16;
    return (float)__builtin_bit_cast(_Float16, b);
}
__device__ __forceinline__ float f16r(float f) { return (float)(_Float16)f; }
__device__ __forceinline__ int sdot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }
__device__ __forceinline__ uint4 ld16(const uint8_t *p) { return *reinterpret_cast<const uint4 *>(p); }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations,
// not for its vector memory operations. __syncthreads() carries a workgroup release fence,
// which compiles to s_waitcnt vmcnt(0): in a prologue that waits for the whole weight group
// in flight (and, in attention, for the K/V row stores) before the barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ------------------------------------------------------------------ cross-lane (DPP)
// Cross-lane sums by DPP (gfx9 row_shr / row_bcast), never through LDS.
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, RM, 0xF, false));
}
constexpr int ROW_SHR1 = 0x111, ROW_SHR2 = 0x112, ROW_SHR4 = 0x114, ROW_SHR8 = 0x118;
constexpr int ROW_BCAST15 = 0x142, ROW_BCAST31 = 0x143;

// wave-wide reductions to lane 63 (row_shr prefix within rows, then row_bcast), returned
// wave-uniform. `id` is the identity of the operation (what out-of-row lanes contribute).
__device__ __forceinline__ float wave_max_f(float v, float id) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), ROW_SHR1, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), ROW_SHR2, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), ROW_SHR4, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), ROW_SHR8, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), ROW_BCAST15, 0xA, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), ROW_BCAST31, 0xC, 0xF, false)));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ int wave_min_i(int v) {
    const int id = INT_MAX;
    v = min(v, __builtin_amdgcn_update_dpp(id, v, ROW_SHR1, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(id, v, ROW_SHR2, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(id, v, ROW_SHR4, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(id, v, ROW_SHR8, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(id, v, ROW_BCAST15, 0xA, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(id, v, ROW_BCAST31, 0xC, 0xF, false));
    return __builtin_amdgcn_readlane(v, 63);
}
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ double dpp_d(double v) {
    const int2 p = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(0, p.x, CTRL, RM, 0xF, false);
    r.y = __builtin_amdgcn_update_dpp(0, p.y, CTRL, RM, 0xF, false);
    return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<ROW_SHR1>(v);
    v += dpp_d<ROW_SHR2>(v);
    v += dpp_d<ROW_SHR4>(v);
    v += dpp_d<ROW_SHR8>(v);
    v += dpp_d<ROW_BCAST15, 0xA>(v);
    v += dpp_d<ROW_BCAST31, 0xC>(v);
    const int2 p = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(p.x, 63);
    r.y = __builtin_amdgcn_readlane(p.y, 63);
    return __builtin_bit_cast(double, r);
}
// all-reduce (max) within aligned 8-lane groups; every lane gets the result
__device__ __forceinline__ float group8_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]
    v = fmaxf(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]
    v = fmaxf(v, dpp_f<0x141>(v));  // row_half_mirror
    return v;
}
// all-reduce (sum) within aligned 4-lane groups
__device__ __forceinline__ int quad_sum_i(int v) {
    v += dpp_i<0xB1>(v);
    v += dpp_i<0x4E>(v);
    return v;
}

// ------------------------------------------------------------------ activation in LDS
struct ActL {
    int8_t *qs;
    float *d;
    int16_t *bs;
};

struct Smem {
    ActL a;
    double *red; // [16]
};

// LDS layout: qs [2K bytes: int8 codes (Q8_0 / Q8_K) or bf16 values (BF16 weights)] |
// d f32[K/32+8] | bs i16[K/16+8] | red
__host__ __device__ inline size_t smem_bytes(int K) {
    return (size_t)K * 2 + (size_t)(K / 32 + 8) * 4 + (size_t)(K / 16 + 8) * 2 + 128;
}

__device__ inline Smem carve(char *base, int K) {
    Smem s;
    s.a.qs = (int8_t *)base;
    s.a.d = (float *)(base + (size_t)K * 2);
    s.a.bs = (int16_t *)(base + (size_t)K * 2 + (size_t)(K / 32 + 8) * 4);
    s.red = (double *)(base + smem_bytes(K) - 128);
    return s;
}

// A multi-token activation record (prefill / batched launches, llm_prefill.hip): act[t] =
// {qs i8[K] | d f32[K/32+8] | bs i16[K/16+8]}, 16-B aligned, nt of them back to back.
__host__ __device__ inline size_t act_bytes(int K) {
    return ((size_t)K + (size_t)(K / 32 + 8) * 4 + (size_t)(K / 16 + 8) * 2 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t act_base(int) { return 0; }
__device__ inline Smem carve_t(char *base, int K, int t) {
    Smem s;
    s.red = nullptr;
    char *a = base + act_base(K) + act_bytes(K) * t;
    s.a.qs = (int8_t *)a;
    s.a.d = (float *)(a + K);
    s.a.bs = (int16_t *)(a + K + (size_t)(K / 32 + 8) * 4);
    return s;
}

// Workgroup sum (8 waves). No trailing barrier: every caller writes `red` again only
// after a later workgroup barrier (the quantizer's closing barrier).
__device__ double block_sum(double v, double *red) {
    v = wave_sum_d(v);
    if ((MIO_TIDX & 63) == 0) red[MIO_TIDX >> 6] = v;
    lds_barrier();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < MW; ++w) t += red[w];
    return t;
}

// quantize_row_q8_K_ref semantics for superblock b held as 4 values per lane (lane l:
// elements 4l .. 4l+3), am = the superblock's largest |x| (wave-uniform): iscale =
// -127/max_signed with max_signed the first element of largest |x|, nearest-even, clamp
// 127, bsums. Its first position comes from a ballot of the lanes holding it (the lowest
// such lane, the lowest of its 4 values); the signed value straight from that lane.
__device__ __forceinline__ void q8k_store(const float (&v)[4], float am, int b, const ActL &a) {
    const int lane = MIO_TIDX & 63;
    int q[4] = {0, 0, 0, 0};
    float dd = 0.0f;
    if (am > 0.0f) {
        float sel = 0.0f;
        bool has = false;
#pragma unroll
        for (int i = 3; i >= 0; --i)
            if (fabsf(v[i]) == am) sel = v[i], has = true;
        const int src = __builtin_ctzll(__ballot(has));
        const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), src));
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
    const int sm = quad_sum_i(q[0] + q[1] + q[2] + q[3]);
    if ((lane & 3) == 0) a.bs[b * 16 + (lane >> 2)] = (int16_t)sm;
    if (lane == 0) a.d[b] = dd;
}
__device__ __forceinline__ float abs_max4(const float (&v)[4]) {
    return wave_max_f(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))), 0.0f);
}

// quantize_row_q8_0_ref semantics (d = amax/127 stored as f16, q = roundf(x * 1/d)) of
// block b held by the 8-lane group of this lane (4 values per lane, lane & 7 = position)
__device__ __forceinline__ void q80_store(const float (&v)[4], int b, bool ok, const ActL &a) {
    const int lane = MIO_TIDX & 63;
    float am = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) am = fmaxf(am, fabsf(v[i]));
    am = group8_max(am);
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

// MIO_X_FIRST=1: a matvec launch waits for its activation loads before issuing any weight
// load (the activation is the critical path; queued behind the chip's first weight burst it
// arrives late). Memory clobber: no load moves across it.
#ifndef MIO_X_FIRST
#define MIO_X_FIRST 0
#endif
// MIO_X_FIRST=2: every wave issues its activation loads before any wave issues weights (a
// bare s_barrier, no waitcnt): the CU's memory queue then holds all activation requests
// ahead of the weight burst, so no wave's activation waits behind other waves' weights.
__device__ __forceinline__ void x_gate() {
#if MIO_X_FIRST == 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#elif MIO_X_FIRST == 2
    asm volatile("s_barrier" ::: "memory");
#endif
}

// ------------------------------------------------------------------ prologue registers
// x (and the norm weight) as float4 per thread, loaded before any weight load.
template <int XV>
struct XRegs {
    float4 v[XV];
    float4 w[XV];
};

// Placed after a launch's first weight loads: nothing computed from x (or the norm weight)
// may be hoisted above them, so the wait for x is never issued before the weight stream is
// (measured 0.813 -> 0.801 ms/token together with the attention kernel's argument
// ordering; forcing every kernel argument into the first scalar round trip was slower).
template <int XV>
__device__ __forceinline__ void x_after_weights(XRegs<XV> &xr) {
#pragma unroll
    for (int i = 0; i < XV; ++i)
        asm volatile("" : "+v"(xr.v[i].x), "+v"(xr.v[i].y), "+v"(xr.v[i].z), "+v"(xr.v[i].w), "+v"(xr.w[i].x),
                     "+v"(xr.w[i].y), "+v"(xr.w[i].z), "+v"(xr.w[i].w));
}

// XAUX = 16 (sc1): x was stored write-through by another workgroup of the same launch
template <int XV, int XAUX = 0>
__device__ inline void load_x(const float *x, const float *w, int K, XRegs<XV> &xr) {
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x), 0, x ? K * 4 : 0, 0x00020000);
    const auto rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(w), 0, w ? K * 4 : 0, 0x00020000);
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rx, e * 4, 0, XAUX);
        const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rw, e * 4, 0, 0);
        xr.v[i] = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
        xr.w[i] = make_float4(__uint_as_float(c.x), __uint_as_float(c.y), __uint_as_float(c.z), __uint_as_float(c.w));
    }
}

// Activation kind of a weight type (ggml's vec_dot_type): 0 Q8_0 (Q8_0 weights), 1 Q8_K
// (Q4_K / Q6_K), 2 BF16 (BF16 weights: the activation rounded to bf16, ggml_fp32_to_bf16).
__host__ __device__ constexpr int akind(int T) { return T == 30 ? 2 : (T == 8 ? 0 : 1); }

// ggml_compute_fp32_to_bf16: round to nearest even, NaN kept quiet
__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 64u;
    return (u + (0x7fffu + ((u >> 16) & 1u))) >> 16;
}

// Quantization straight from the registers a prologue loaded: thread t holds elements
// e = (t + i*MT) * 4 .. +3, i.e. wave w lane l holds 256 w + 4 l + 2048 i — exactly superblock
// w + 8 i at lane offset 4 l (quant_q8k's layout) and, for Q8_0, block 8 w + (l >> 3) + 64 i
// at position 4 (l & 7) (quant_q80's layout). So the LDS staging row and its barrier of the
// staged quantizer are not needed; the records are the same bits. One barrier at the end
// makes them visible to every wave. ak = akind(weight type); BF16 stores the rounded values
// (2 bytes each) at a.qs + 2e.
template <int XV>
__device__ __forceinline__ void quant_regs(const float4 (&v)[XV], int K, int ak, const ActL &a) {
    const int lane = MIO_TIDX & 63, wave = __builtin_amdgcn_readfirstlane(MIO_TIDX >> 6);
    if (ak == 1) {
        const int nsb = K >> 8;
#pragma unroll
        for (int j = 0; j < XV; ++j) {
            const int b = wave + MW * j;
            if (b >= nsb) break;
            const float vv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
            q8k_store(vv, abs_max4(vv), b, a);
        }
    } else if (ak == 2) {
#pragma unroll
        for (int j = 0; j < XV; ++j) {
            const int e = (MIO_TIDX + j * MT) * 4;
            if (e < K)
                *reinterpret_cast<uint2 *>(a.qs + 2 * e) =
                    make_uint2(f32_to_bf16(v[j].x) | (f32_to_bf16(v[j].y) << 16),
                               f32_to_bf16(v[j].z) | (f32_to_bf16(v[j].w) << 16));
        }
    } else {
        const int nb = K / 32;
#pragma unroll
        for (int j = 0; j < XV; ++j) {
            const int b = wave * 8 + MW * 8 * j + (lane >> 3);
            const float vv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
            q80_store(vv, b, b < nb, a);
        }
    }
    lds_barrier();
}

// ggml: mean = sum / ne00 in double; a power-of-two K divides exactly by a multiply
__device__ __forceinline__ float rms_scale(double tot, int K, float eps) {
    const float mean = (float)((K & (K - 1)) == 0 ? tot * (1.0 / K) : tot / K);
    return 1.0f / sqrtf(mean + eps);
}

// ggml_rms_norm + mul(weight): xs = (x * 1/sqrtf(mean(x^2) + eps)) * w, then quantize.
template <int XV>
__device__ void rmsnorm_quant(const XRegs<XV> &xr, int K, float eps, int kquant, const Smem &s,
                              unsigned long long *diag = nullptr) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        if (e < K) {
            const float4 v = xr.v[i];
            acc += (double)(v.x * v.x);
            acc += (double)(v.y * v.y);
            acc += (double)(v.z * v.z);
            acc += (double)(v.w * v.w);
        }
    }
#ifdef MIO_TL_WAVES
    // wave-arrival diagnostic: slot w = wave w's activation consumed (w = 1..7; slot 7
    // replaces the end mark)
    if (diag && (MIO_TIDX & 63) == 0 && MIO_TIDX > 0) {
        asm volatile("" ::"v"(acc));
        diag[MIO_TIDX >> 6] = __builtin_amdgcn_s_memrealtime();
    }
    if (diag && MIO_TIDX == 0) {
        asm volatile("" ::"v"(acc));
        diag[0] = __builtin_amdgcn_s_memrealtime() - 0;  // wave 0 stays the start reference
    }
#else
    MIO_DIAG_STAMP(diag, 3, acc);  // activation consumed (arrived)
    if (diag && MIO_TIDX == MIO_DIAG_WAVE * 64) {  // ... by wave MIO_DIAG_WAVE (default: the last)
        asm volatile("" ::"v"(acc));
        diag[1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const double tot = block_sum(acc, s.red);
    MIO_DIAG_STAMP(diag, 4, tot);  // reduced over the workgroup
    const float scale = rms_scale(tot, K, eps);
    float4 y[XV];
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const float4 v = xr.v[i], ww = xr.w[i];
        float t;
        t = v.x * scale, y[i].x = t * ww.x;
        t = v.y * scale, y[i].y = t * ww.y;
        t = v.z * scale, y[i].z = t * ww.z;
        t = v.w * scale, y[i].w = t * ww.w;
    }
    MIO_DIAG_STAMP(diag, 5, scale);  // normalized activation in registers
    quant_regs<XV>(y, K, kquant, s.a);
}

template <int XV>
__device__ inline void plain_quant(const XRegs<XV> &xr, int K, int kquant, const Smem &s,
                                   unsigned long long *diag = nullptr) {
    MIO_DIAG_STAMP(diag, 5, 0);  // activation arrived
    quant_regs<XV>(xr.v, K, kquant, s.a);
}

// ------------------------------------------------------------------ lfm2 gated short conv
// llama.cpp build_shortconv_block + ggml_ssm_conv (d_conv = kConvL = 3) for one token:
// bcx = in_proj(norm x) = B | C | X, bx = B * X, y = C * conv with, per channel e,
// conv = ((0 + x[p-2] w[e][0]) + x[p-1] w[e][1]) + bx w[e][2] (ggml's f32 sum from 0 over the
// window in order), x[q] = the bx of position q, 0 before the sequence start. A window input
// comes from a ring row of bx values, or from the bcx row of an earlier token of the same
// launch (B * X recomputed: the same f32 product), or is absent (zeros).
struct ConvPrev {
    const float *p;  // null: zeros
    int bcx;         // 1: p is a bcx row (3 K floats), 0: a bx row (K floats)
};
template <int XV>
struct ConvRegs {
    float4 b[XV], c[XV], x[XV], p1[XV], p2[XV], w[XV][3];
};
__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 mul4(float4 a, float4 b) {
    return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float4 conv_prev4(const ConvPrev &pv, int K, int e) {
    if (!pv.p) return make_float4(0.f, 0.f, 0.f, 0.f);
    if (!pv.bcx) return ld4(pv.p + e);
    return mul4(ld4(pv.p + e), ld4(pv.p + 2 * K + e));
}
template <int XV>
__device__ inline void conv_load(const float *bcx, const ConvPrev &p1, const ConvPrev &p2, const float *conv_w, int K,
                                 ConvRegs<XV> &r) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        if (e < K) {
            r.b[i] = ld4(bcx + e), r.c[i] = ld4(bcx + K + e), r.x[i] = ld4(bcx + 2 * K + e);
            r.p1[i] = conv_prev4(p1, K, e), r.p2[i] = conv_prev4(p2, K, e);
#pragma unroll
            for (int j = 0; j < 3; ++j) r.w[i][j] = ld4(conv_w + (size_t)e * kConvL + 4 * j);
        }
    }
}
// the conv output (and, when bx_out is set, this token's bx row into it), re-quantized from
// registers as the out_proj activation
template <int XV>
__device__ inline void conv_quant(const ConvRegs<XV> &r, int K, int kquant, const Smem &s, float *bx_out,
                                  unsigned long long *diag = nullptr) {
    float4 y[XV];
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        y[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < K) {
            const float4 bx = mul4(r.b[i], r.x[i]);
            const float v2[4] = {r.p2[i].x, r.p2[i].y, r.p2[i].z, r.p2[i].w};
            const float v1[4] = {r.p1[i].x, r.p1[i].y, r.p1[i].z, r.p1[i].w};
            const float v0[4] = {bx.x, bx.y, bx.z, bx.w};
            const float c[4] = {r.c[i].x, r.c[i].y, r.c[i].z, r.c[i].w};
            // taps of channels e..e+3: w[e + j][t] = flat[(e + j) * 3 + t] = 12 consecutive floats
            const float w[12] = {r.w[i][0].x, r.w[i][0].y, r.w[i][0].z, r.w[i][0].w, r.w[i][1].x, r.w[i][1].y,
                                 r.w[i][1].z, r.w[i][1].w, r.w[i][2].x, r.w[i][2].y, r.w[i][2].z, r.w[i][2].w};
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float acc = 0.0f;
                acc = acc + v2[j] * w[j * 3 + 0];
                acc = acc + v1[j] * w[j * 3 + 1];
                acc = acc + v0[j] * w[j * 3 + 2];
                o[j] = c[j] * acc;
            }
            y[i] = make_float4(o[0], o[1], o[2], o[3]);
            if (bx_out) *reinterpret_cast<float4 *>(bx_out + e) = bx;
        }
    }
    MIO_DIAG_STAMP(diag, 5, 0);
    quant_regs<XV>(y, K, kquant, s.a);
}
// keeps the conv operands' use below the first weight loads (x_after_weights)
template <int XV>
__device__ __forceinline__ void conv_after_weights(ConvRegs<XV> &r) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        asm volatile("" : "+v"(r.b[i].x), "+v"(r.b[i].y), "+v"(r.b[i].z), "+v"(r.b[i].w));
        asm volatile("" : "+v"(r.x[i].x), "+v"(r.x[i].y), "+v"(r.x[i].z), "+v"(r.x[i].w));
    }
}

// ------------------------------------------------------------------ typed row dots
// exact integer sum of each 8-lane group, valid in lanes 8k+7
__device__ __forceinline__ int sum8_i(int v) {
    v += dpp_i<ROW_SHR1>(v);
    v += dpp_i<ROW_SHR2>(v);
    v += dpp_i<ROW_SHR4>(v);
    return v;
}
__device__ __forceinline__ float sum8_f(float v) {
    v += dpp_f<ROW_SHR1>(v);
    v += dpp_f<ROW_SHR2>(v);
    v += dpp_f<ROW_SHR4>(v);
    return v;
}
// sum of the values held in lanes 8k+7 (k = 0..7), returned wave-uniform
__device__ __forceinline__ float sum_lanes7(float v) {
    v += dpp_f<ROW_SHR8>(v);
    v += dpp_f<ROW_BCAST15, 0xA>(v);
    v += dpp_f<ROW_BCAST31, 0xC>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

constexpr uint32_t M4 = 0x0F0F0F0Fu, M2 = 0x03030303u;

// One unit's weight registers.
//   Q4_K: a = 16 B of nibbles, c = dword (lane & 3) of the superblock header {d, dmin,
//         4 x 24-bit scale pairs}
//   Q6_K: a = 16 B of ql, b = 16 B of qh, c = the lane's two int8 sub-block scales, e = d
//   Q8_0: a, b = the lane's 32 codes, e = d
//   BF16: a, b, a2, b2 = the lane's 32 weights (bf16 pairs), one contiguous KB per register
//         over the wave (weights pass*2048 + 512 i + 8 l .. +8 for register i = a, b, a2, b2)
struct Frag {
    uint4 a, b;
    uint32_t c, e;
    uint4 a2, b2;
};

// One unit's activation registers (the lane's 32 int8 values, two bsums, the scale).
struct ALane {
    int4 lo, hi;
    int b0, b1;
    float d;
    int4 lo2, hi2;  // BF16: the activations of registers a2, b2
};

// Lane mapping per pass: K-quants - 8 superblocks x 8 lanes (lane>>3 = superblock,
// lane&7 = 16-byte piece); Q8_0 - 64 blocks, one per lane (32 codes = two 16-B loads).
// `row` is wave-uniform, so the row base address is scalar. Loads are unconditional
// (indices past K are clamped to the row's last block and their terms zeroed in
// dot_frag): no branches around loads, so vmcnt accounting stays exact and raw data is
// only converted where it is consumed.
// Raw buffer loads: descriptor from the (uniform) base and its exact byte size, the row
// offset in an SGPR (soffset), the lane's constant byte offset in voffset - no per-load
// address VALU; lanes past the end read 0 (range-checked).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)min(bytes, 0x7FFFFFF0u), 0x00020000);
}
// Cache policy of the weight stream (buffer-load aux bits; 2 = nt): weights are read once per
// step by one CU, so they should not evict what the launch chain re-reads (kernel arguments,
// activations, K/V rows) from L2 / Infinity Cache.
#ifndef MIO_WEIGHT_AUX
#define MIO_WEIGHT_AUX 2
#endif
// policy of the output matrix stream (lm_head): A/B knob
#ifndef MIO_LM_AUX
#define MIO_LM_AUX MIO_WEIGHT_AUX
#endif
// policy of the small per-layer streams (attn_in q|k|v, attn_out o): A/B knob
#ifndef MIO_SMALL_AUX
#define MIO_SMALL_AUX MIO_WEIGHT_AUX
#endif
template <int AUX = MIO_WEIGHT_AUX>
__device__ __forceinline__ uint4 bld16(const uint8_t *base, uint32_t bytes, uint32_t voff, uint32_t soff) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base, bytes), voff, soff, AUX);
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <int AUX = MIO_WEIGHT_AUX>
__device__ __forceinline__ uint32_t bld4(const uint8_t *base, uint32_t bytes, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(rsrc(base, bytes), voff, soff, AUX);
}
template <int AUX = MIO_WEIGHT_AUX>
__device__ __forceinline__ uint32_t bld2(const uint8_t *base, uint32_t bytes, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b16(rsrc(base, bytes), voff, soff, AUX);
}

template <int T, int AUX = MIO_WEIGHT_AUX>
__device__ __forceinline__ Frag load_frag(const QMat W, int row, int pass) {
    const int lane = MIO_TIDX & 63;
    // the row is wave-uniform; readfirstlane lets the compiler keep it (and the soffset) in
    // SGPRs - without it every load became a waterfall loop over a VGPR soffset
    const uint32_t R = (uint32_t)W.rows,
                   r = (uint32_t)__builtin_amdgcn_readfirstlane(min(max(row, 0), W.rows - 1));
    Frag f;
    if constexpr (T == 12) {
        const int nsb = W.k >> 8, sb = min(pass * 8 + (lane >> 3), nsb - 1), pc = lane & 7;
        const uint32_t qb = (uint32_t)(W.k / 2), hb = (uint32_t)nsb * 16;
        f.a = bld16<AUX>(W.p0, R * qb, sb * 128 + pc * 16, r * qb);
        // header dword (lane & 3) only: both quads of the superblock's 8 lanes hold all four,
        // broadcast by DPP in dot_frag (a quarter of the load-return traffic of 16 B per lane)
        f.c = bld4<AUX>(W.p1, R * hb, sb * 16 + 4 * (pc & 3), r * hb);
        f.b = make_uint4(0, 0, 0, 0);
        f.e = 0;
    } else if constexpr (T == 14) {
        const int nsb = W.k >> 8, sb = min(pass * 8 + (lane >> 3), nsb - 1), pc = lane & 7;
        const uint32_t lb = (uint32_t)(W.k / 2), hb = (uint32_t)(W.k / 4), sbb = (uint32_t)(W.k / 16),
                       db = (uint32_t)nsb * 2;
        f.a = bld16<AUX>(W.p0, R * lb, sb * 128 + pc * 16, r * lb);
        f.b = bld16<AUX>(W.p1, R * hb, sb * 64 + 32 * (pc >> 2) + 16 * (pc & 1), r * hb);
        f.c = bld2<AUX>(W.p2, R * sbb, sb * 16 + 2 * pc, r * sbb);
        f.e = bld2<AUX>(W.p3, R * db, sb * 2, r * db);
    } else if constexpr (T == 30) {
        // element offsets clamped into the row (past K: another valid piece, zeroed in dot_frag)
        const uint32_t rb = (uint32_t)W.k * 2;
        auto off = [&](int i) { return (uint32_t)min(pass * 2048 + 512 * i + 8 * lane, W.k - 8) * 2u; };
        f.a = bld16<AUX>(W.p0, R * rb, off(0), r * rb);
        f.b = bld16<AUX>(W.p0, R * rb, off(1), r * rb);
        f.a2 = bld16<AUX>(W.p0, R * rb, off(2), r * rb);
        f.b2 = bld16<AUX>(W.p0, R * rb, off(3), r * rb);
        f.c = 0;
        f.e = 0;
    } else {
        const int nb = W.k >> 5, b = min(pass * 64 + lane, nb - 1);
        const uint32_t qb = (uint32_t)W.k, db = (uint32_t)nb * 2;
        f.a = bld16<AUX>(W.p0, R * qb, 32 * b, r * qb);
        f.b = bld16<AUX>(W.p0, R * qb, 32 * b + 16, r * qb);
        f.c = 0;
        f.e = bld2<AUX>(W.p1, R * db, 2 * b, r * db);
    }
    return f;
}

template <int T>
__device__ __forceinline__ ALane load_alane(const ActL &a, int K, int pass) {
    const int lane = MIO_TIDX & 63;
    ALane r;
    if constexpr (T == 12 || T == 14) {
        const int nsb = K >> 8, sb = pass * 8 + (lane >> 3), pc = lane & 7;
        const int sbc = sb < nsb ? sb : 0;
        int e, e2;
        if constexpr (T == 12) {
            e = sbc * 256 + 64 * (pc >> 1) + 16 * (pc & 1);
            e2 = e + 32;
        } else {
            const int n = pc >> 2, qq = pc & 3;
            e = sbc * 256 + 128 * n + 32 * (qq >> 1) + 16 * (qq & 1);
            e2 = e + 64;
        }
        r.lo = *reinterpret_cast<const int4 *>(a.qs + e);
        r.hi = *reinterpret_cast<const int4 *>(a.qs + e2);
        r.b0 = a.bs[e >> 4];
        r.b1 = a.bs[e2 >> 4];
        r.d = a.d[sbc];
    } else if constexpr (T == 30) {
        auto at = [&](int i) {
            const int e = min(pass * 2048 + 512 * i + 8 * lane, K - 8);
            return *reinterpret_cast<const int4 *>(a.qs + 2 * e);
        };
        r.lo = at(0), r.hi = at(1), r.lo2 = at(2), r.hi2 = at(3);
        r.b0 = r.b1 = 0;
        r.d = 0.0f;
    } else {
        const int nb = K >> 5, b = pass * 64 + lane, bc = b < nb ? b : 0;
        r.lo = *reinterpret_cast<const int4 *>(a.qs + 32 * bc);
        r.hi = *reinterpret_cast<const int4 *>(a.qs + 32 * bc + 16);
        r.b0 = r.b1 = 0;
        r.d = a.d[bc];
    }
    return r;
}

// This lane's partial of the row dot for one pass. K-quants: the per-superblock integer
// sums are reduced exactly over the superblock's 8 lanes (ggml vec_dot semantics) and the
// superblock's float term is valid in lane 8k+7; Q8_0: every lane holds one block's term.
// Lanes whose superblock / block lies past K have zero codes and zero scales -> 0.
template <int T>
__device__ __forceinline__ float dot_frag(const Frag &f, const ALane &al, int K, int pass) {
    const int lane = MIO_TIDX & 63;
    if constexpr (T == 12) {
        const int jj = (lane & 7) >> 1;
        uint4 h;  // the superblock header {d|dmin, scale/min words} from the quad's four dwords
        h.x = (uint32_t)dpp_i<0x00>((int)f.c);
        h.y = (uint32_t)dpp_i<0x55>((int)f.c);
        h.z = (uint32_t)dpp_i<0xAA>((int)f.c);
        h.w = (uint32_t)dpp_i<0xFF>((int)f.c);
        const uint32_t wlo = jj < 2 ? h.y : (jj == 2 ? h.z : h.w);
        const uint32_t whi = jj < 2 ? h.z : h.w;
        const uint32_t F = __builtin_amdgcn_alignbit(whi, wlo, (24 * jj) & 31);
        const int sc0 = F & 63, m0 = (F >> 6) & 63, sc1 = (F >> 12) & 63, m1 = (F >> 18) & 63;
        int dlo = 0, dhi = 0;
        dlo = sdot4((int)(f.a.x & M4), al.lo.x, dlo);
        dlo = sdot4((int)(f.a.y & M4), al.lo.y, dlo);
        dlo = sdot4((int)(f.a.z & M4), al.lo.z, dlo);
        dlo = sdot4((int)(f.a.w & M4), al.lo.w, dlo);
        dhi = sdot4((int)((f.a.x >> 4) & M4), al.hi.x, dhi);
        dhi = sdot4((int)((f.a.y >> 4) & M4), al.hi.y, dhi);
        dhi = sdot4((int)((f.a.z >> 4) & M4), al.hi.z, dhi);
        dhi = sdot4((int)((f.a.w >> 4) & M4), al.hi.w, dhi);
        int isum = __mul24(sc0, dlo) + __mul24(sc1, dhi);
        int imin = __mul24(m0, al.b0) + __mul24(m1, al.b1);
        isum = sum8_i(isum);
        imin = sum8_i(imin);
        const float d = h2f(h.x & 0xFFFF) * al.d;
        const float dmin = h2f(h.x >> 16) * al.d;
        float v = d * (float)isum;
        v = v - dmin * (float)imin;
        return pass * 8 + (lane >> 3) < (K >> 8) ? v : 0.0f;
    } else if constexpr (T == 14) {
        // high 2 bits of the low-nibble codes sit at bit 2*gl of each qh byte, of the
        // high-nibble codes at bit 2*gl+4 (gl = (lane&3)>>1); move them to bits 4-5
        const int shl = 2 * ((lane & 3) >> 1);
        auto lo = [&](uint32_t l, uint32_t h) { return (int)((l & M4) | ((h << (4 - shl)) & 0x30303030u)); };
        auto hi = [&](uint32_t l, uint32_t h) { return (int)(((l >> 4) & M4) | ((h >> shl) & 0x30303030u)); };
        int dlo = 0, dhi = 0;
        dlo = sdot4(lo(f.a.x, f.b.x), al.lo.x, dlo);
        dlo = sdot4(lo(f.a.y, f.b.y), al.lo.y, dlo);
        dlo = sdot4(lo(f.a.z, f.b.z), al.lo.z, dlo);
        dlo = sdot4(lo(f.a.w, f.b.w), al.lo.w, dlo);
        dhi = sdot4(hi(f.a.x, f.b.x), al.hi.x, dhi);
        dhi = sdot4(hi(f.a.y, f.b.y), al.hi.y, dhi);
        dhi = sdot4(hi(f.a.z, f.b.z), al.hi.z, dhi);
        dhi = sdot4(hi(f.a.w, f.b.w), al.hi.w, dhi);
        const int sa = (int)(int8_t)(f.c & 0xFF), sb = (int)(int8_t)(f.c >> 8);
        int isum = __mul24(sa, dlo - 32 * al.b0) + __mul24(sb, dhi - 32 * al.b1);
        isum = sum8_i(isum);
        const float d = h2f(f.e) * al.d;
        const float v = d * (float)isum;
        return pass * 8 + (lane >> 3) < (K >> 8) ? v : 0.0f;
    } else if constexpr (T == 30) {
        // ggml_vec_dot_bf16 on the bf16-rounded activation: products of bf16 pairs are exact
        // in f32; 8 weights per register, summed by v_dot2 in register order (pieces past K
        // zeroed on both sides)
        typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
        float acc = 0.0f;
        auto dot8 = [&](const uint4 &w, const int4 &x, int i) {
            const bool ok = pass * 2048 + 512 * i + 8 * lane < K;
            const uint4 ww = ok ? w : make_uint4(0, 0, 0, 0);
            const uint4 xx = ok ? make_uint4((uint32_t)x.x, (uint32_t)x.y, (uint32_t)x.z, (uint32_t)x.w)
                                : make_uint4(0, 0, 0, 0);
            acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, ww.x), __builtin_bit_cast(bf2, xx.x), acc, false);
            acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, ww.y), __builtin_bit_cast(bf2, xx.y), acc, false);
            acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, ww.z), __builtin_bit_cast(bf2, xx.z), acc, false);
            acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, ww.w), __builtin_bit_cast(bf2, xx.w), acc, false);
        };
        dot8(f.a, al.lo, 0);
        dot8(f.b, al.hi, 1);
        dot8(f.a2, al.lo2, 2);
        dot8(f.b2, al.hi2, 3);
        return acc;
    } else {
        int s = 0;
        s = sdot4((int)f.a.x, al.lo.x, s);
        s = sdot4((int)f.a.y, al.lo.y, s);
        s = sdot4((int)f.a.z, al.lo.z, s);
        s = sdot4((int)f.a.w, al.lo.w, s);
        s = sdot4((int)f.b.x, al.hi.x, s);
        s = sdot4((int)f.b.y, al.hi.y, s);
        s = sdot4((int)f.b.z, al.hi.z, s);
        s = sdot4((int)f.b.w, al.hi.w, s);
        const float v = (float)s * (h2f(f.e) * al.d);
        return pass * 64 + lane < (K >> 5) ? v : 0.0f;
    }
}

// Row total of the per-lane partials (accumulated over the row's passes), wave-uniform.
template <int T>
__device__ __forceinline__ float row_total(float acc) {
    if constexpr (T == 8 || T == 30) acc = sum8_f(acc);
    return sum_lanes7(acc);
}

// ------------------------------------------------------------------ streaming rows
// NP passes per row (1, 3 or 6); U units per register group; NP <= 3 keeps the lane's
// activation slices in registers for the whole stream. SU > 0: the wave's whole share (at
// most SU units, host-checked) is ONE group of SU units, issued before the prologue - a
// launch whose waves own only a row or two issues no duplicate (clamped) loads; every
// vector memory instruction costs the CU's address path ~16 cycles however few bytes it
// moves, and a launch's first loads are issued in one burst.
template <int NP, int SU = 0>
struct Cfg {
    static constexpr int U = SU ? SU : (NP == 1 ? 4 : 3);
    static constexpr int NG = SU ? 1 : 2;
    static constexpr bool AREG = NP <= 3;
};

// Loads units [u0, u0 + U) (clamped into [0, n): loads are never skipped, so the
// compiler's in-order vmcnt accounting stays exact). Unit u -> row lo + u/(NP*NM),
// matrix (u/NP)%NM, pass u%NP. With NM == 1, rows >= split come from W1 (row - split):
// two matrices of one type streamed as one row space (q|k).
template <int T, int NP, int NM, int SU = 0, int AUX = MIO_WEIGHT_AUX>
__device__ __forceinline__ void load_group(const QMat W0, const QMat W1, int lo, int n, int u0,
                                           Frag (&f)[Cfg<NP, SU>::U], int split = INT_MAX) {
#pragma unroll
    for (int j = 0; j < Cfg<NP, SU>::U; ++j) {
        // wave-uniform (readfirstlane: the compiler cannot prove it through wave_range's
        // VALU divisions, and a VGPR unit index turns matrix selection into waterfall loops)
        const int u = __builtin_amdgcn_readfirstlane(max(0, min(u0 + j, n - 1)));
        const int p = u % NP, m = (u / NP) % NM, i = u / (NP * NM);
        if constexpr (NM == 1) {
            const int r = __builtin_amdgcn_readfirstlane(lo + i);
            f[j] = load_frag<T, AUX>(r >= split ? W1 : W0, r >= split ? r - split : r, p);
        } else {
            f[j] = load_frag<T, AUX>(m ? W1 : W0, lo + i, p);
        }
    }
}

// Streams rows [lo, hi) (wave-uniform) of W0 (and W1 when NM == 2: row pairs, e.g.
// gate/up); calls epi(row, dot0, dot1) once per row with wave-uniform values. A and B hold
// the first two groups (units [0, U) and [U, 2U)), issued by the caller before its
// prologue; groups then alternate between A and B, one group in flight while the other is
// reduced (no register copies).
template <int T, int NP, int NM, int SU = 0, int AUX = MIO_WEIGHT_AUX, class Epi>
__device__ __forceinline__ void stream_rows(const QMat W0, const QMat W1, int lo, int hi, Frag (&A)[Cfg<NP, SU>::U],
                                            Frag (&B)[Cfg<NP, SU>::U], const ActL &a, Epi &&epi, int split = INT_MAX,
                                            unsigned long long *trace = nullptr) {
    constexpr int U = Cfg<NP, SU>::U;
    const int K = W0.k;
    const int n = (hi - lo) * NM * NP;
    if (n <= 0) return;
    ALane al[Cfg<NP, SU>::AREG ? NP : 1];
    if constexpr (Cfg<NP, SU>::AREG) {
#pragma unroll
        for (int p = 0; p < NP; ++p) al[p] = load_alane<T>(a, K, p);
    }
    float acc = 0.0f, g = 0.0f;
    auto consume = [&](const Frag (&F)[U], int u0) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int u = u0 + j;
            if (u < n) {
                int p;
                ALane av;
                if constexpr (NP == 1) {
                    p = 0;
                    av = al[0];
                } else if constexpr (NP == U) {
                    p = j;
                    av = al[j];
                } else {
                    p = u % NP;
                    av = load_alane<T>(a, K, p);
                }
                acc += dot_frag<T>(F[j], av, K, p);
                if (p == NP - 1) {
                    const float v = row_total<T>(acc);
                    acc = 0.0f;
                    const int i = u / (NP * NM);
                    if constexpr (NM == 1) {
                        epi(lo + i, v, 0.0f);
                    } else {
                        if ((u / NP) % NM == 0)
                            g = v;
                        else
                            epi(lo + i, g, v);
                    }
                }
            }
        }
    };
    for (int u0 = 0;;) {
        consume(A, u0);
        if (trace && u0 == 0 && blockIdx.x == 0 && MIO_TIDX == 0) trace[3] = __builtin_readcyclecounter();
        if constexpr (Cfg<NP, SU>::NG == 1) break;
        u0 += U;
        if (u0 >= n) break;
        load_group<T, NP, NM, SU, AUX>(W0, W1, lo, n, u0 + U, A, split);
        consume(B, u0);
        u0 += U;
        if (u0 >= n) break;
        load_group<T, NP, NM, SU, AUX>(W0, W1, lo, n, u0 + U, B, split);
    }
}

// The first group(s) of a wave's stream (before the prologue).
template <int T, int NP, int NM, int SU = 0, int AUX = MIO_WEIGHT_AUX>
__device__ __forceinline__ void load_first(const QMat W0, const QMat W1, int lo, int hi, Frag (&A)[Cfg<NP, SU>::U],
                                           Frag (&B)[Cfg<NP, SU>::U], int split = INT_MAX) {
    const int n = (hi - lo) * NM * NP;
    load_group<T, NP, NM, SU, AUX>(W0, W1, lo, n, 0, A, split);
    if constexpr (Cfg<NP, SU>::NG == 2) load_group<T, NP, NM, SU, AUX>(W0, W1, lo, n, Cfg<NP, SU>::U, B, split);
}

// Rows [0, R) over G workgroups: workgroup b owns [R*b/G, R*(b+1)/G), wave w a contiguous
// eighth of that (wave-uniform, held in scalar registers). R*G < 2^31.
__device__ inline void wave_range(int R, int &lo, int &hi, int b, int G) {
    const int w = __builtin_amdgcn_readfirstlane(MIO_TIDX >> 6);
    const int ra = (R * b) / G, rb = (R * (b + 1)) / G;
    lo = ra + (rb - ra) * w / MW;
    hi = ra + (rb - ra) * (w + 1) / MW;
}
// the same over NW row waves: wave w (w0 <= w < w0 + NW) owns its share; other waves none
__device__ inline void wave_range_n(int R, int &lo, int &hi, int b, int G, int w0, int NW) {
    const int w = __builtin_amdgcn_readfirstlane(MIO_TIDX >> 6) - w0;
    const int ra = (R * b) / G, rb = (R * (b + 1)) / G;
    if (w < 0 || w >= NW) {
        lo = hi = ra;
        return;
    }
    lo = ra + (rb - ra) * w / NW;
    hi = ra + (rb - ra) * (w + 1) / NW;
}
__device__ inline void wave_range(const LlmDims &d, int R, int &lo, int &hi) {
    wave_range(R, lo, hi, blockIdx.x, matvec_grid_n(d.n_wg, R));
}


// ------------------------------------------------------------------ embedding rows
__device__ float dequant_elem(const QMat &W, int row, int e) {
    if (W.type == 12) {
        const int nsb = W.k >> 8, sb = e >> 8, c = e & 255, j = c >> 6, w = c & 63, hi = w >> 5, l = w & 31;
        const uint8_t q = W.p0[(size_t)row * (W.k / 2) + sb * 128 + 32 * j + l];
        const uint8_t *hd = W.p1 + ((size_t)row * nsb + sb) * 16;
        const uint32_t F = (uint32_t)hd[4 + 3 * j] | ((uint32_t)hd[5 + 3 * j] << 8) | ((uint32_t)hd[6 + 3 * j] << 16);
        const int sc = (F >> (12 * hi)) & 63, m = (F >> (12 * hi + 6)) & 63;
        const float d1 = h2f(hd[0] | (hd[1] << 8)) * sc, m1 = h2f(hd[2] | (hd[3] << 8)) * m;
        return d1 * (float)(hi ? (q >> 4) : (q & 0xF)) - m1;
    } else if (W.type == 14) {
        const int nsb = W.k >> 8, sb = e >> 8, c = e & 255, n = c >> 7, w = c & 127, g = w >> 5, l = w & 31;
        const uint8_t ql = W.p0[(size_t)row * (W.k / 2) + sb * 128 + 64 * n + l + 32 * (g & 1)];
        const uint8_t qh = W.p1[(size_t)row * (W.k / 4) + sb * 64 + 32 * n + l];
        const int q = (int)((g < 2 ? (ql & 0xF) : (ql >> 4)) | (((qh >> (2 * g)) & 3) << 4)) - 32;
        const int is = c >> 4, sn = is >> 3, sw = is & 7;
        const int sc = ((const int8_t *)W.p2)[(size_t)row * (W.k / 16) + sb * 16 + 2 * (4 * sn + (sw & 3)) + (sw >> 2)];
        const float dd = h2f(((const uint16_t *)W.p3)[(size_t)row * nsb + sb]);
        return dd * (float)sc * (float)q;
    } else if (W.type == 30) {
        const uint16_t h = ((const uint16_t *)W.p0)[(size_t)row * W.k + e];
        return __uint_as_float((uint32_t)h << 16);
    } else {
        const int nb = W.k >> 5;
        const int8_t q = ((const int8_t *)W.p0)[(size_t)row * W.k + e];
        return (float)q * h2f(((const uint16_t *)W.p1)[(size_t)row * nb + (e >> 5)]);
    }
}

constexpr int ST = 1024;  // sampler / embedding threads (n_embd <= 4 * ST)

__device__ inline void embed_row(const QMat &emb, int tok, int n, float *x) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = MIO_TIDX + i * ST;
        v[i] = e < n ? dequant_elem(emb, tok, e) : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = MIO_TIDX + i * ST;
        if (e < n) x[e] = v[i];
    }
}


// ------------------------------------------------------------------ host-side grids
// attn_in grid: q|k rows on the first g_qk workgroups, v rows on the rest
inline void attn_in_grid(const LlmDims &d, const LayerW &L, int &G, int &g_qk) {
    const int rows = L.wq.rows + L.wk.rows + L.wv.rows, qk = L.wq.rows + L.wk.rows;
    G = matvec_grid(d, rows);
    g_qk = (G * qk + rows / 2) / rows;
    g_qk = g_qk < 1 ? 1 : (g_qk > G - 1 ? G - 1 : g_qk);
}


// ------------------------------------------------------------------ attention helpers
// all-reduce over aligned groups of LP (8 or 16) lanes, by DPP; every lane of a group gets
// the bitwise-same sum
template <int LP>
__device__ __forceinline__ float group_sum(float v) {
    v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);  // row_half_mirror
    if constexpr (LP == 16) v += dpp_f<0x140>(v);  // row_mirror
    return v;
}

__device__ inline float silu_f(float x) { return x / (1.0f + expf(-x)); }

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



// ------------------------------------------------------------------ sampler
// Position of the token being decoded (StepState: the sampler of the previous step may still
// be pending, then the token sits one past st->pos; a full context keeps the last slot).
__device__ __forceinline__ int cur_pos(const StepState *st, const LlmDims &d) {
    return min(st->pos + st->pending, d.n_ctx - 1);
}

// An end token was sampled: the rest of the step and every later step return at entry (the
// reference breaks before the next llama_decode, test-to-speech.cpp:168-170). The matvec
// launches read the flag with a VECTOR load issued in front of their activation loads:
// vmcnt retires in order, so the wait for x covers it and a decoding step pays no extra
// round trip (a scalar load of the flag behind the weight group cost 82 us per 1.7B token).
template <class B>
__device__ __forceinline__ uint32_t done_issue(const B &b) {
    return __builtin_amdgcn_raw_buffer_load_b32(rsrc(&b.st->done, 4), 0, 0, 0);
}
__device__ __forceinline__ bool done_now(uint32_t v) { return __builtin_amdgcn_readfirstlane(v) != 0; }
// An end token was sampled: besides StepState.done (which the step's own launches read), one
// system-scope vector store to the host's mapped word, so the host stops enqueuing steps
// without a blocking poll (once per utterance, over PCIe)
__device__ __forceinline__ void signal_host_done(const SampleCfg &sc) {
    if (sc.host_done) __hip_atomic_store(sc.host_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The pending sample's token: Gumbel-max winner (ties -> lowest id) over the lm_head
// workgroups' partials {smp[2i] value, smp[2i+1] id bits}, sc.lo when no id was allowed, the
// forced token of this step if any. Whole workgroup of NTH threads (multiple of 64, <= 1024);
// every thread returns the same token (the winner is order-independent: a total order).
template <int NTH>
__device__ int sample_token(const float *smp, int nblk, const SampleCfg &sc, int step, float *rs, int *ri) {
    const int tid = MIO_TIDX, lane = tid & 63, wave = tid >> 6;
    float best = -INFINITY;
    int bi = INT_MAX;
    const bool forced = sc.force && step < sc.n_force;
    const int ft = forced ? sc.force[step] : -1;
    for (int i = tid; i < nblk; i += NTH) {
        const float v = smp[2 * i];
        const int ix = __float_as_int(smp[2 * i + 1]);
        if (v > best || (v == best && ix < bi)) best = v, bi = ix;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float v = __shfl_xor(best, o);
        const int ix = __shfl_xor(bi, o);
        if (v > best || (v == best && ix < bi)) best = v, bi = ix;
    }
    if (lane == 0) rs[wave] = best, ri[wave] = bi;
    lds_barrier();
    best = rs[0], bi = ri[0];
    for (int w = 1; w < NTH / 64; ++w)
        if (rs[w] > best || (rs[w] == best && ri[w] < bi)) best = rs[w], bi = ri[w];
    int tok = bi == INT_MAX ? sc.lo : bi;
    if (ft >= 0) tok = ft;
    return tok;
}

// Embedding row of tok in the matvec prologue's register layout (thread t: elements
// 4(t + i*MT) .. +3), the same dequantization as embed_row.
template <int XV>
__device__ inline void embed_regs(const QMat &emb, int tok, int K, XRegs<XV> &xr) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (e < K)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = dequant_elem(emb, tok, e + q);
        xr.v[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// Calls f.template operator()<NP, T>() for the matrix's pass count and weight type. BF = false:
// the int8 types only (the multi-token engine: BF16 models prefill token by token).
template <bool BF = true, class F>
void dispatch_nt(int K, int type, F &&f) {
    const int np = pick_np(K);
#define NT_CASE(NPV, TV) \
    if (np == NPV && type == TV) return f.template operator()<NPV, TV>();
    NT_CASE(1, 8) NT_CASE(1, 12) NT_CASE(1, 14) NT_CASE(3, 8) NT_CASE(3, 12) NT_CASE(3, 14)
    NT_CASE(6, 8) NT_CASE(6, 12) NT_CASE(6, 14)
    if constexpr (BF) {
        NT_CASE(1, 30) NT_CASE(3, 30) NT_CASE(6, 30)
    }
#undef NT_CASE
}


// ------------------------------------------------------------------ attention chunk sweep
// Shared by the decode step (k_attention), the batched decode (k_bt_attention) and the
// prefill (k_pf_attention), so all three produce bit-identical partial records and outputs.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

// One workgroup per (ATT_CHUNK positions, kv head [, token]): a position slot is LP lanes
// holding 8 dims each; NT = ATT_CHUNK * LP threads (at most MIO_ATT_NT), IT positions per
// slot, and the K/V rows of a chunk arrive in one load round trip per lane.
// MIO_ATT_NT: threads per attention chunk workgroup at most. 256 (4 positions per slot at
// 64-position chunks): 0.763-0.766 vs 0.775 ms per token with 512 (profiles/r04_att_nt_ab.txt);
// 128 would need the merge to cover more than one float4 of outputs per thread at G * hd = 1024
#ifndef MIO_ATT_NT
#define MIO_ATT_NT 256
#endif
template <int HD>
struct AttCfg {
    static constexpr int LP = HD / 8;                                        // lanes per slot
    static constexpr int NT = ATT_CHUNK * LP < MIO_ATT_NT ? ATT_CHUNK * LP : MIO_ATT_NT;  // threads
    static constexpr int NW = NT / 64;                                       // waves
    static constexpr int NS = NT / LP;                                       // position slots
    static constexpr int IT = ATT_CHUNK / NS;                                // positions per slot
    static constexpr int REC = part_rec(HD);
};

// Agent-scope (sc1: write-through / L1-bypassing) accesses of the chunk records handed from
// the attention workgroups of a launch to the one that merges them (attn_merge_last):
// buffer instructions on a wave-uniform base with per-lane byte offsets (aux 16 = sc1).
__device__ __forceinline__ void st1_sc1(float *base, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(base, 0x7FFFFFF0u), off, 0, 16);
}
__device__ __forceinline__ void st4_sc1(float *base, uint32_t off, float4 v) {
    u32x4 u;
    u.x = __float_as_uint(v.x), u.y = __float_as_uint(v.y), u.z = __float_as_uint(v.z), u.w = __float_as_uint(v.w);
    __builtin_amdgcn_raw_buffer_store_b128(u, rsrc(base, 0x7FFFFFF0u), off, 0, 16);
}
// One lane waits until the agent-scope counter *c reaches target (relaxed loads, s_sleep
// between polls: MI355X_MICROARCH "polling-cost"). Bounded: after ~2^16 polls (tens of ms) it
// gives up and raises *flag, so a lost signal ends the launch instead of hanging the GPU. Once
// the flag is up (an earlier wait of this run gave up: the run is already an error), every
// further wait returns after at most 1024 polls instead of spinning its full bound: a broken
// hand-off costs one bound per run, not one per launch (round 5 saw a 180-s stall that a
// per-launch timeout across a 40-step batch would explain).
// Hand-off rule for every caller: the bytes the signallers published are read with sc1 loads
// only (buffer / global loads with aux 16), never plain loads (MI355X_MICROARCH, replica row).
__device__ __forceinline__ void wait_count(int *c, int target, int *flag) {
    auto *p = (__attribute__((address_space(1))) int *)c;
    auto *f = (__attribute__((address_space(1))) int *)flag;
    for (int it = 0; it < (1 << 16); ++it) {
        if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
        if ((it & 1023) == 1023 && __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld4_sc1(const float *base, uint32_t off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base, 0x7FFFFFF0u), off, 0, 16);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ float2 ld2_sc1(const float *base, uint32_t off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc(base, 0x7FFFFFF0u), off, 0, 16);
    return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}

// Online-softmax merge of nch chunk partial records {O[hd], m, l} for the 4 outputs
// dd .. dd+3 of one head whose record array starts at element `head` of the wave-uniform base
// `part` (sc1 loads: records other workgroups of the launch wrote): 8 chunks' loads in flight
// per batch; a missing chunk of a batch is {m = -inf, l = 0, O = 0}, which leaves the max and
// the sums unchanged (only real chunks are loaded: every vector load instruction costs the
// CU's address path the same, used or not). The float order does not depend on which
// workgroup merges, so every path's outputs are the same bits.
// (r06 A/B: issuing the next batch's loads before merging the current one doubles the
// batch registers; k_layer_att went from 65 to 136-160 VGPRs, its roles no longer co-reside,
// and the step lost 9 %: not kept.)
__device__ __forceinline__ float4 merge_out4(const float *part, uint32_t head, int nch, int rec, int hd, int dd) {
    float M = -INFINITY, L = 0.0f;
    float4 O = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int CB = 8;  // chunks per batch of loads
    for (int c0 = 0; c0 < nch; c0 += CB) {
        float2 ml[CB];
        float4 oc[CB];
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int c = c0 + j;
            if (c < nch) {
                ml[j] = ld2_sc1(part, (head + (uint32_t)(c * rec + hd)) * 4u);
                oc[j] = ld4_sc1(part, (head + (uint32_t)(c * rec + dd)) * 4u);
            } else {
                ml[j] = make_float2(-INFINITY, 0.0f);
                oc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        float mb = M;
#pragma unroll
        for (int j = 0; j < CB; ++j) mb = fmaxf(mb, ml[j].x);
        const float a = M == -INFINITY ? 0.0f : expf(M - mb);
        L *= a;
        O.x *= a, O.y *= a, O.z *= a, O.w *= a;
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const float w = c0 + j < nch ? expf(ml[j].x - mb) : 0.0f;
            L += w * ml[j].y;
            O.x += w * oc[j].x, O.y += w * oc[j].y, O.z += w * oc[j].z, O.w += w * oc[j].w;
        }
        M = mb;
    }
    return make_float4(O.x / L, O.y / L, O.z / L, O.w / L);
}

// value of lane ^ O (O = 16 or 32 by the gfx950 permlane swaps, VALU; smaller O by bpermute)
template <int O>
__device__ __forceinline__ float xor_lane(float v) {
    const int lane = MIO_TIDX & 63;
    if constexpr (O == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(lane < 32 ? r[1] : r[0]);
    } else if constexpr (O == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        return __uint_as_float(((lane >> 4) & 1) == 0 ? r[1] : r[0]);
    } else {
        return __shfl_xor(v, O);
    }
}

// q/k head preparation by one wave (HD values at src): optional RMSNorm with weight nw
// (qwen3 attn_q_norm / attn_k_norm), RoPE on (i, i + HD/2) pairs (NEOX) or (2i, 2i+1) (NORM)
// with the ggml rope-cache cos/sin, f16 rounding (the F16 cache / ggml's f16 K operand).
// row: wave-private LDS scratch [HD]; the prepared head is left in row.
// bias (may be null): the projection bias added in f32 before anything else (qwen2,
// llama.cpp build_attn_mha's Qcur = ggml_add(Qcur, bq)).
// The loads of one head's preparation (prep_head), issued on their own so a caller can put
// them in front of its K/V row loads (vmcnt retires in order: a head load behind 8 K/V loads
// waits for all of them). val: the head's values (+ bias), w: norm weight, cs: RoPE cos/sin;
// vv (optional, the new v row of the owner's k head): value + bias.
template <int HD>
struct HeadIn {
    static constexpr int PER = HD / 64;
    float v[PER], w[PER], vv[PER];
    float2 cs[PER];
};
// AUX = 16 (sc1): src / vsrc were stored write-through by other workgroups of the same launch
template <int HD, int AUX = 0>
__device__ __forceinline__ void head_load(const float *src, const float *bias, const float *nw, const float2 *rope,
                                          const LlmDims &d, HeadIn<HD> &in, const float *vsrc = nullptr,
                                          const float *vbias = nullptr) {
    constexpr int PER = HD / 64;
    const int lane = MIO_TIDX & 63;
    auto ld = [&](const float *base, int p) {
        if constexpr (AUX == 0) return base[p];
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(base, HD * 4), p * 4, 0, AUX));
    };
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int p = lane + 64 * i;
        in.v[i] = ld(src, p);
        if (bias) in.v[i] = in.v[i] + bias[p];
        in.w[i] = d.qk_norm ? nw[p] : 1.0f;
        in.cs[i] = p < HD / 2 ? rope[p] : make_float2(0.0f, 0.0f);
        if (vsrc) {
            in.vv[i] = ld(vsrc, p);
            if (vbias) in.vv[i] = in.vv[i] + vbias[p];
        }
    }
}

// q/k head preparation by one wave from head_load's registers: optional RMSNorm with weight w
// (qwen3 attn_q_norm / attn_k_norm), RoPE on (i, i + HD/2) pairs (NEOX) or (2i, 2i+1) (NORM)
// with the ggml rope-cache cos/sin, f16 rounding (the F16 cache / ggml's f16 K operand).
// The projection bias was added in f32 before anything else (qwen2, llama.cpp build_attn_mha's
// Qcur = ggml_add(Qcur, bq)). row: wave-private LDS scratch [HD]; the prepared head is left in row.
template <int HD>
__device__ void head_prep(const HeadIn<HD> &in, const LlmDims &d, float *row) {
    constexpr int PER = HD / 64;
    const int lane = MIO_TIDX & 63;
    float v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = in.v[i];
    if (d.qk_norm) {
        double ss = 0.0;
#pragma unroll
        for (int i = 0; i < PER; ++i) ss += (double)(v[i] * v[i]);
        ss = wave_sum_d(ss);
        const float mean = (float)(ss / HD);
        const float scale = 1.0f / sqrtf(mean + d.eps);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const float t = v[i] * scale;
            v[i] = t * in.w[i];
        }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) row[lane + 64 * i] = v[i];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float o0[PER], o1[PER];
    int i0s[PER], i1s[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int p = lane + 64 * i;
        i0s[i] = -1;
        if (p < HD / 2) {
            const int i0 = d.neox ? p : 2 * p, i1 = d.neox ? p + HD / 2 : 2 * p + 1;
            const float x0 = row[i0], x1 = row[i1];
            o0[i] = x0 * in.cs[i].x - x1 * in.cs[i].y;
            o1[i] = x0 * in.cs[i].y + x1 * in.cs[i].x;
            i0s[i] = i0, i1s[i] = i1;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int i = 0; i < PER; ++i)
        if (i0s[i] >= 0) {
            row[i0s[i]] = f16r(o0[i]);
            row[i1s[i]] = f16r(o1[i]);
        }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// head_load + head_prep (HD values at src; bias may be null)
template <int HD>
__device__ void prep_head(const float *src, const float *bias, const float *nw, const float2 *rope,
                          const LlmDims &d, float *row) {
    HeadIn<HD> in;
    head_load<HD>(src, bias, nw, rope, d, in);
    head_prep<HD>(in, d, row);
}

// K/V rows of this thread's slot (positions t0 + sl + NS*it, clamped to pos), issued early.
template <int HD>
__device__ __forceinline__ void load_kv_rows(const _Float16 *kbase, const _Float16 *vbase, int t0, int pos,
                                             h8 (&kr)[AttCfg<HD>::IT], h8 (&vr)[AttCfg<HD>::IT]) {
    constexpr int LP = AttCfg<HD>::LP, NS = AttCfg<HD>::NS;
    const int lp = (MIO_TIDX & 63) % LP, sl = MIO_TIDX / LP;
#pragma unroll
    for (int it = 0; it < AttCfg<HD>::IT; ++it) {
        const int t = min(t0 + sl + NS * it, pos);
        kr[it] = *reinterpret_cast<const h8 *>(kbase + (size_t)t * HD + lp * 8);
        vr[it] = *reinterpret_cast<const h8 *>(vbase + (size_t)t * HD + lp * 8);
    }
}

// Softmax attention of the G query heads qs (LDS, prepared) over the chunk's positions
// [t0, min(t0 + ATT_CHUNK, pos + 1)) whose K/V rows are in kr/vr, in two passes like ggml's
// soft_max (scores, chunk max, exp, sums; summation order aside): every slot's scores are
// independent dot products, the max is exchanged once (lanes by butterflies, waves by LDS),
// and the slots' sums then merge by plain adds (no online rescaling). Writes the chunk's
// partial record {O[HD] = sum_t p_t v_t, m = chunk max, l = sum_t p_t} of head g to
// dst + g * g_stride (p_t = exp(s_t - m)).
template <int HD, int G>
__device__ void attend_chunk(const float (*qs)[HD], const h8 (&kr)[AttCfg<HD>::IT], const h8 (&vr)[AttCfg<HD>::IT],
                             int t0, int pos, float scale, float (*wres)[G][HD + 2], float *dst, size_t g_stride,
                             unsigned long long *trace = nullptr, unsigned long long *diag = nullptr) {
    constexpr int LP = AttCfg<HD>::LP, NS = AttCfg<HD>::NS, IT = AttCfg<HD>::IT, NT = AttCfg<HD>::NT,
                  NW = AttCfg<HD>::NW;
    __shared__ float wmax[NW][G];
    const int tid = MIO_TIDX, lane = tid & 63, wave = tid >> 6;
    const int lp = lane % LP, sl = tid / LP;
    auto mark = [&](int k) {  // checkpoints of mio_hip_llm_trace_kernel (diagnostic)
        if (trace && blockIdx.x == 0 && blockIdx.y == 0 && MIO_TIDX == 0) {
            asm volatile("" ::: "memory");
            trace[k] = __builtin_readcyclecounter();
        }
    };
    float qv[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) qv[g][i] = qs[g][lp * 8 + i];
    // pass 1: scores (valid positions <= pos) and this thread's running max per head
    float sc[IT][G], mx[G];
#pragma unroll
    for (int g = 0; g < G; ++g) mx[g] = -INFINITY;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const bool valid = t0 + sl + NS * it <= pos;
        float kf[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) kf[i] = (float)kr[it][i];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float sdot = 0.0f;
#pragma unroll
            for (int i = 0; i < 8; ++i) sdot = fmaf(qv[g][i], kf[i], sdot);
            sdot = group_sum<LP>(sdot);
            sc[it][g] = valid ? sdot * scale : -INFINITY;
            mx[g] = fmaxf(mx[g], sc[it][g]);
        }
    }
    // chunk max: slots of the wave (butterflies), then the waves (LDS)
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if constexpr (LP <= 8) mx[g] = fmaxf(mx[g], xor_lane<8>(mx[g]));
        mx[g] = fmaxf(mx[g], xor_lane<16>(mx[g]));
        mx[g] = fmaxf(mx[g], xor_lane<32>(mx[g]));
    }
    if (lane == 0)
#pragma unroll
        for (int g = 0; g < G; ++g) wmax[wave][g] = mx[g];
    lds_barrier();
    float M[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        M[g] = wmax[0][g];
#pragma unroll
        for (int w = 1; w < NW; ++w) M[g] = fmaxf(M[g], wmax[w][g]);
    }
    mark(3);
    MIO_DIAG_STAMP(diag, 3, M[0]);  // scores and chunk max done
    // pass 2: p = exp(s - M), sums of p and of p * v (the chunk holds position t0 <= pos,
    // so M is finite)
    float l[G], acc[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        l[g] = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[g][i] = 0.0f;
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        float vf[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) vf[i] = (float)vr[it][i];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float p = sc[it][g] == -INFINITY ? 0.0f : expf(sc[it][g] - M[g]);
            l[g] += p;
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[g][i] = fmaf(p, vf[i], acc[g][i]);
        }
    }
    // slots of the wave: plain sums (every lane of a butterfly pair ends bitwise equal)
    auto sum_step = [&](auto xl) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            l[g] += xl(l[g]);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[g][i] += xl(acc[g][i]);
        }
    };
    if constexpr (LP <= 8) sum_step([](float v) { return xor_lane<8>(v); });
    sum_step([](float v) { return xor_lane<16>(v); });
    sum_step([](float v) { return xor_lane<32>(v); });
    mark(4);
    MIO_DIAG_STAMP(diag, 4, acc[0][0]);  // wave sums done
    if (lane < LP) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int i = 0; i < 8; ++i) wres[wave][g][lp * 8 + i] = acc[g][i];
            if (lp == 0) wres[wave][g][HD] = l[g];
        }
    }
    lds_barrier();
    mark(5);
    MIO_DIAG_STAMP(diag, 5, 0);  // wave results in LDS
    // the waves -> this chunk's partial record per q head, stored write-through (sc1) for
    // the workgroup of this launch that merges the chunks (attn_merge_last)
    for (int e = tid; e < G * HD; e += NT) {
        const int g = e / HD, dd = e - g * HD;
        float O = 0.0f, L = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            O += wres[w][g][dd];
            L += wres[w][g][HD];
        }
        const uint32_t o = (uint32_t)(g * g_stride) * 4u;
        st1_sc1(dst, o + 4u * dd, O);
        if (dd == 0) st1_sc1(dst, o + 4u * HD, M[g]), st1_sc1(dst, o + 4u * (HD + 1), L);
    }
}

// ------------------------------------------------------------------ attention chunk on the matrix cores
// MIO_ATT_MFMA (default 1; 0 = the VALU attend_chunk above, for A/B builds): the chunk's
// Q.K^T and P.V on v_mfma_f32_16x16x32_f16, shared by the decode step, the batched decode and
// the prefill, so their outputs stay equal bit for bit.
//  * K and V rows are staged once per workgroup into two LDS images (one 16-B chunk per lane
//    and load; a chunk's physical slot is XOR-swizzled per row, AttM::fk / fv, so the
//    fragment reads below are bank-conflict-free);
//  * every wave computes S^T = K Q^T for the WHOLE chunk (PT x KS MFMAs: A = a 16-position K
//    tile read from the image, B = Q^T, the G heads padded to 16 columns with zeros), so the
//    chunk max and sum of each head are wave-local: no workgroup barrier after the staging;
//  * S^T's accumulator has the position on the registers and the head on the lane, so P (as
//    f16 hi + lo parts: P = hi + lo to 2^-22, the f32 probabilities to within rounding of the
//    residual) is the A operand of the P.V MFMA with no lane movement; V's 16-dim column tiles
//    come from the image by ds_read_b64_tr_b16 (4 positions x 16 dims per 16-lane group) in
//    the same permuted k order (positions 32 s + 4 h + j and 32 s + 16 + 4 h + j of lane half
//    h: cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand");
//  * wave w owns output dims [HD / 4 * w, HD / 4 * (w + 1)): DTW tiles of 16.
// Numerics: q and the cache rows are f16-exact, so every product is exact and only the f32
// summation order differs from the VALU sweep (scores by 32-dim MFMA k-steps, p.v by 32
// positions); records {O[hd] = sum p v, m, l = sum p} as attend_chunk's.
#ifndef MIO_ATT_MFMA
#define MIO_ATT_MFMA 1
#endif
// MIO_ATT_FASTEXP (default 1): p by the hardware exp (v_exp_f32 of x log2 e) instead of expf
// (0 for A/B: 0.764 vs 0.754-0.758 ms per 1.7B token, profiles/r05_att_ab.txt)
#ifndef MIO_ATT_FASTEXP
#define MIO_ATT_FASTEXP 1
#endif
typedef _Float16 h4v __attribute__((ext_vector_type(4)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <int HD>
struct AttM {
    static constexpr int NT = 256, NW = 4;
    static constexpr int CH = HD / 8;               // 16-byte chunks per K / V row
    static constexpr int VI = ATT_CHUNK * CH / NT;  // chunks of K (and of V) each thread stages
    static constexpr int PT = ATT_CHUNK / 16;       // 16-position tiles of S^T
    static constexpr int KS = HD / 32;              // 32-dim k-steps of Q.K^T
    static constexpr int PS = ATT_CHUNK / 32;       // 32-position k-steps of P.V
    static constexpr int DTW = HD / 16 / NW;        // 16-dim output tiles per wave
    static constexpr int RB = HD * 2;               // bytes per image row
    static constexpr int IMG = ATT_CHUNK * RB;      // bytes per image
    // physical chunk of logical chunk c of row r = c ^ f(r).
    // fk: the K fragment read (ds_read_b128, lane (h, i) reads chunk 4 j + h of row 16 tau + i)
    //     puts each 16-lane bank group on 16 distinct slots (HD 128: slots = chunks; HD 64: 8
    //     chunks x 2 row parities);
    // fv: the transposed read (lane 4 q + p of group h: row base + 4 h + q, dims col0 + 4 p ..)
    //     puts the 8 rows x 2 chunks of a 32-lane half on 16 distinct slots.
    // Both keep the 8-lane groups of the image stores (ds_write_b128, 8 consecutive chunks of a
    // row) on distinct banks.
    __device__ static int fk(int r) { return HD == 128 ? (r & 15) : ((r >> 1) & 7); }
    __device__ static int fv(int r) { return HD == 128 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1); }
};
static_assert(ATT_CHUNK % 32 == 0, "attention chunk: whole 32-position k-steps");

// This thread's K / V chunks of the chunk's rows t0 .. t0 + ATT_CHUNK - 1 (rows past pos read
// row pos: finite values under a zero probability), issued early.
template <int HD>
__device__ __forceinline__ void kv_issue(const _Float16 *kb, const _Float16 *vb, int t0, int pos,
                                         h8 (&kr)[AttM<HD>::VI], h8 (&vr)[AttM<HD>::VI]) {
    using A = AttM<HD>;
#pragma unroll
    for (int it = 0; it < A::VI; ++it) {
        const int c = it * A::NT + (int)MIO_TIDX, row = c / A::CH, ch = c % A::CH;
        const size_t o = (size_t)min(t0 + row, pos) * HD + ch * 8;
        kr[it] = *reinterpret_cast<const h8 *>(kb + o);
        vr[it] = *reinterpret_cast<const h8 *>(vb + o);
    }
}

// The chunks into the images; row `skip` (the position being decoded, whose cache row this
// launch writes) is staged from LDS by the wave that prepared it (kv_stage_row).
template <int HD>
__device__ __forceinline__ void kv_stage(const h8 (&kr)[AttM<HD>::VI], const h8 (&vr)[AttM<HD>::VI], int skip,
                                         char *kimg, char *vimg) {
    using A = AttM<HD>;
#pragma unroll
    for (int it = 0; it < A::VI; ++it) {
        const int c = it * A::NT + (int)MIO_TIDX, row = c / A::CH, ch = c % A::CH;
        if (row != skip) {
            *reinterpret_cast<h8 *>(kimg + row * A::RB + 16 * (ch ^ A::fk(row))) = kr[it];
            *reinterpret_cast<h8 *>(vimg + row * A::RB + 16 * (ch ^ A::fv(row))) = vr[it];
        }
    }
}

// One wave: row r of both images from the prepared f16-exact k / v values (LDS floats).
template <int HD>
__device__ __forceinline__ void kv_stage_row(const float *kn, const float *vn, int r, char *kimg, char *vimg) {
    using A = AttM<HD>;
    const int lane = MIO_TIDX & 63;
    if (lane < 2 * A::CH) {
        const bool isv = lane >= A::CH;
        const int ch = lane % A::CH;
        const float *src = (isv ? vn : kn) + ch * 8;
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (_Float16)src[e];
        char *img = isv ? vimg : kimg;
        *reinterpret_cast<h8 *>(img + r * A::RB + 16 * (ch ^ (isv ? A::fv(r) : A::fk(r)))) = v;
    }
}

// The chunk's partial records {O[HD], m, l} of the G heads qh (LDS, f16) over positions
// [t0, min(t0 + ATT_CHUNK, pos + 1)) from the staged images, stored write-through (sc1) at
// dst + g * g_stride for attn_merge_last. Whole workgroup (AttM::NT threads); the images and
// qh must be visible (a barrier after staging).
template <int HD, int G>
__device__ __forceinline__ void attend_chunk_mfma(const _Float16 (*qh)[HD], const char *kimg, const char *vimg, int t0,
                                                  int pos, float scale, float *dst, uint32_t g_stride,
                                                  unsigned long long *trace = nullptr) {
    using A = AttM<HD>;
    static_assert(G <= 16, "heads per kv head");
    const int lane = MIO_TIDX & 63, wave = MIO_TIDX >> 6, h = lane >> 4, i = lane & 15;
    auto mark = [&](int k, float v) {  // checkpoints of mio_hip_llm_trace_kernel (diagnostic)
        if (trace && blockIdx.x == 0 && blockIdx.y == 0 && MIO_TIDX == 0) {
            asm volatile("" ::"v"(v) : "memory");
            trace[k] = __builtin_readcyclecounter();
        }
    };
    // every LDS read of the chunk is issued up front (one round trip, not one per fragment):
    // the K tiles (A operand: lane (h, i) reads position 16 tau + i, dims 32 j + 8 h .. + 7) ...
    h8 kf[A::PT][A::KS];
#pragma unroll
    for (int tau = 0; tau < A::PT; ++tau)
#pragma unroll
        for (int j = 0; j < A::KS; ++j) {
            const int r = 16 * tau + i;
            kf[tau][j] = *reinterpret_cast<const h8 *>(kimg + r * A::RB + 16 * ((4 * j + h) ^ A::fk(r)));
        }
    // ... Q^T (B operand: head i's dims 32 j + 8 h .. + 7, zero past G) ...
    h8 qf[A::KS];
    const int gq = i < G ? i : G - 1;
#pragma unroll
    for (int j = 0; j < A::KS; ++j) {
        const h8 q = *reinterpret_cast<const h8 *>(&qh[gq][32 * j + 8 * h]);
        qf[j] = i < G ? q : h8{};
    }
    // ... and this wave's V^T tiles by transposed reads (lane 4 q + p of group h: row
    // 32 s + 16 r2 + 4 h + q, dims col0 + 4 p .. + 3)
    const int q4 = i >> 2, p4 = i & 3;
    h4v vb[A::PS][A::DTW][2];
#pragma unroll
    for (int s2 = 0; s2 < A::PS; ++s2)
#pragma unroll
        for (int n = 0; n < A::DTW; ++n) {
            const int lch = 2 * (wave * A::DTW + n) + (p4 >> 1);
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const int row = 32 * s2 + 16 * r2 + 4 * h + q4;
                const char *a = vimg + row * A::RB + 16 * (lch ^ A::fv(row)) + 8 * (p4 & 1);
                vb[s2][n][r2] = __builtin_bit_cast(
                    h4v, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(const_cast<char *>(a))));
            }
        }
    // S^T tiles: s[tau][e] = q_i . k(t0 + 16 tau + 4 h + e)
    f4v s[A::PT];
#pragma unroll
    for (int tau = 0; tau < A::PT; ++tau) {
        s[tau] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < A::KS; ++j) s[tau] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[tau][j], qf[j], s[tau], 0, 0, 0);
    }
    // scaled scores, positions past pos masked (only the chunk holding pos has any), and head
    // i's chunk max over this lane's 4 PT positions, then the 4 lanes (h) holding head i
    float M = -INFINITY;
    if (t0 + ATT_CHUNK - 1 <= pos) {
#pragma unroll
        for (int tau = 0; tau < A::PT; ++tau)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                s[tau][e] = s[tau][e] * scale;
                M = fmaxf(M, s[tau][e]);
            }
    } else {
#pragma unroll
        for (int tau = 0; tau < A::PT; ++tau)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool valid = t0 + 16 * tau + 4 * h + e <= pos;
                s[tau][e] = valid ? s[tau][e] * scale : -INFINITY;
                M = fmaxf(M, s[tau][e]);
            }
    }
    M = fmaxf(M, xor_lane<16>(M));
    M = fmaxf(M, xor_lane<32>(M));
    mark(3, M);
    // p = exp(s - M) as the P.V A operand (hi + lo f16 parts), l = sum p (the chunk holds
    // position t0 <= pos, so M is finite; exp(-inf) = 0 for the masked positions)
    float L = 0.0f;
    h8 ph[A::PS], pl[A::PS];
#pragma unroll
    for (int tau = 0; tau < A::PT; ++tau)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#if MIO_ATT_FASTEXP
            // exp(x) = 2^(x log2 e) on v_exp_f32 (relative error ~ |x| 2^-24 + 1 ulp)
            const float p = __builtin_amdgcn_exp2f((s[tau][e] - M) * 1.44269504088896341f);
#else
            const float p = expf(s[tau][e] - M);
#endif
            L += p;
            const _Float16 hi = (_Float16)p;
            ph[tau >> 1][(tau & 1) * 4 + e] = hi;
            pl[tau >> 1][(tau & 1) * 4 + e] = (_Float16)(p - (float)hi);
        }
    L += xor_lane<16>(L);
    L += xor_lane<32>(L);
    mark(4, L);
    // P.V for this wave's dims
    f4v o[A::DTW];
#pragma unroll
    for (int n = 0; n < A::DTW; ++n) o[n] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < A::PS; ++s2)
#pragma unroll
        for (int n = 0; n < A::DTW; ++n) {
            const h4v *b2 = vb[s2][n];
            const h8 vf = h8{b2[0][0], b2[0][1], b2[0][2], b2[0][3], b2[1][0], b2[1][1], b2[1][2], b2[1][3]};
            o[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph[s2], vf, o[n], 0, 0, 0);
            o[n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl[s2], vf, o[n], 0, 0, 0);
        }
    mark(5, o[0][0]);
    // o[n][e] = O[head 4 h + e][dim 16 (wave DTW + n) + i]
#pragma unroll
    for (int n = 0; n < A::DTW; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int g = 4 * h + e;
            if (g < G) st1_sc1(dst, ((uint32_t)g * g_stride + 16 * (wave * A::DTW + n) + i) * 4u, o[n][e]);
        }
    if (wave == 0 && h == 0 && i < G) {
        st1_sc1(dst, ((uint32_t)i * g_stride + HD) * 4u, M);
        st1_sc1(dst, ((uint32_t)i * g_stride + HD + 1) * 4u, L);
    }
}

// q heads as f16 (the f16-exact prepared values) for attend_chunk_mfma's B operand: one wave,
// head row src (HD floats) -> dst
template <int HD>
__device__ __forceinline__ void q_to_f16(const float *src, _Float16 *dst) {
    const int lane = MIO_TIDX & 63;
#pragma unroll
    for (int e = lane; e < HD; e += 64) dst[e] = (_Float16)src[e];
}

// After attend_chunk: the chunk workgroups of one (kv head [, token]) take arrival tickets;
// the last of the nch arrivals merges every chunk's records (merge_out4) into the G heads'
// outputs out[G][HD] (plain stores: read by the next launch). Hand-off (MI355X_MICROARCH
// "Valid forms", first row): every record byte was stored sc1 (attend_chunk), each wave
// drains its stores (vmcnt(0)) before the workgroup barrier, then ONE lane adds to the
// unsharded ticket with an agent-scope atomic; the workgroup whose add returned nch - 1 loads
// the records only after that add returned (its other waves after the barrier that follows),
// and every load of them is an sc1 load. The last arriver also resets the ticket to 0 for the
// next launch (kernel boundaries order that store before any later add). part / head0: the
// wave-uniform record base and the element offset of head g = 0's record array (head g at
// head0 + g * g_stride).
// ak >= 0 (multi-token launches): the merger also writes the outputs' activation record for
// the O matvec (ak = akind of W_o: 1 Q8_K, 0 Q8_0) into rec, blocks from blk0 on: wave w of
// the merger holds outputs 256 w .. 256 w + 255 in quant_regs' layout, so the records are
// k_bt_quant's bits and its launch is not needed (host: (G * HD) % 256 == 0 for Q8_K, % 32
// for Q8_0).
// rdy != nullptr (the fused attention + O launch, k_att_o): the outputs are consumed by other
// workgroups of the same launch, so they are stored sc1 (write-through), drained, and then
// lanes 0..7 add 1 to each of the 8 counter shards rdy[64 i] (the O workgroups wait for n_kv
// adds on theirs), the same hand-off form as the records'.
template <int HD, int G>
__device__ void attn_merge_last(const float *part, uint32_t head0, uint32_t g_stride, int nch, int *cnt, float *out,
                                int ak = -1, ActL rec = {}, int blk0 = 0, int *rdy = nullptr,
                                unsigned long long *tl = nullptr) {
    constexpr int NT = AttCfg<HD>::NT, REC = AttCfg<HD>::REC;
    __shared__ int last_;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (MIO_TIDX == 0) {
        auto *c = (__attribute__((address_space(1))) int *)cnt;
        const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_ = old == nch - 1;
        if (old == nch - 1) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last_) return;
    if (tl && MIO_TIDX == 0) tl[5] = __builtin_amdgcn_s_memrealtime();  // step timeline: merger's ticket
    // one float4 of outputs per thread and pass (G * hd > 4 NT: several passes); in pass b,
    // wave w holds outputs 4 NT b + 256 w .. + 255 (one Q8_K superblock / eight Q8_0 blocks)
#pragma unroll
    for (int b = 0; b < (G * HD + 4 * NT - 1) / (4 * NT); ++b) {
        const int e = 4 * NT * b + 4 * (int)MIO_TIDX;
        float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < G * HD) {
            const int g = e / HD, dd = e - g * HD;
            y = merge_out4(part, head0 + (uint32_t)g * g_stride, nch, REC, HD, dd);
            if (rdy)
                st4_sc1(out, (uint32_t)e * 4, y);
            else
                *reinterpret_cast<float4 *>(out + e) = y;
        }
        if (ak >= 0) {
            const int wave = __builtin_amdgcn_readfirstlane(MIO_TIDX >> 6), lane = MIO_TIDX & 63;
            const int sb = (4 * NT * b) / 256 + wave;
            if (sb * 256 < G * HD) {
                const float vv[4] = {y.x, y.y, y.z, y.w};
                if (ak == 1)
                    q8k_store(vv, abs_max4(vv), blk0 + sb, rec);
                else
                    q80_store(vv, blk0 + sb * 8 + (lane >> 3), e < G * HD, rec);
            }
        }
    }
    if (rdy) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tl && MIO_TIDX == 0) tl[6] = __builtin_amdgcn_s_memrealtime();  // outputs written through
        if (MIO_TIDX < 8)
            __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(rdy + 64 * MIO_TIDX), 1,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------------------ host-side dispatch
// Calls f.template operator()<SU>() for the instantiated single-group sizes of NP.
template <int NP, class F>
void dispatch_su(int su, F &&f) {
    if constexpr (NP == 1) {
        if (su == 1) return f.template operator()<1>();
        if (su == 2) return f.template operator()<2>();
        if (su == 3) return f.template operator()<3>();
        if (su == 4) return f.template operator()<4>();
        if (su == 6) return f.template operator()<6>();
    }
    if constexpr (NP == 3) {
        if (su == 3) return f.template operator()<3>();
    }
    f.template operator()<0>();
}
}  // namespace
}  // namespace mio
