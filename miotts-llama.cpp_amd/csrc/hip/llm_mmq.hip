// Multi-token quantized matmul on the gfx950 int8 matrix cores (batched prompt prefill and
// the batched decode of several utterances: the layers of llama_decode for a batch of tokens,
// test-to-speech.cpp:132-148).
//
// y[t][row] = W[row] . a[t] for up to 32 tokens t per tile, W in the split quant layout
// (csrc/host/quant.h: GGUF blocks regrouped per plane), a[t] the token's activation already
// re-quantized to the weight's ggml vec_dot_type by k_bt_quant (Q8_K for K-quants, Q8_0 for
// Q8_0) - the decode prologue's own arithmetic.
//
// One workgroup per (32-row tile, 32-token tile); its 8 waves split K by the decode engine's
// lane slots (below). Every quantization group (Q4_K: 32-value
// sub-block, Q6_K: 16-value sub-block, Q8_0: 32-value block) is one MFMA:
//   v_mfma_i32_32x32x32_i8 (Q4_K, Q8_0) / v_mfma_i32_32x32x16_i8 (Q6_K),
// A = the 32 tokens' int8 activations, B = the 32 rows' codes, C[token][row] = the group's
// exact integer dot. The group scales are applied exactly as ggml's vec_dot does (integer
// sums per superblock, then one float term per superblock / block), and the float terms are
// summed in the decode engine's order (per-lane pass accumulation, then the balanced DPP
// trees of row_total), so every (row, token) equals the single-token decode step's value BIT
// FOR BIT (tests/test_llm_gpu.py::test_batched_prefill_matches_sequential).
//   Q4_K: the min term sum_sb m_sb * sum(a in sb) is a second MFMA against m_sb broadcast
//         (it accumulates over the superblock in the matrix core, no VALU)
//   Q6_K: codes enter as q - 32 (signed 6-bit), so sum_j sc_j * (q - 32) . a needs no bsums
// C/D layout (gfx950, dtype independent): lane l holds column (weight row) l & 31 and rows
// (tokens) (r & 3) + 8 (r >> 2) + 4 (l >> 5), r = 0..15. A/B: lane l holds row/column
// l & 31 and a contiguous half of K (the same half in A and B; exact-integer probe:
// tools/micro/mfma_i8_probe.hip).
#include "llm_device.h"
#include "llm_mmq.h"
#include "llm_quant_producer.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#pragma clang fp contract(off)

namespace mio {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int RT = 32;  // rows per tile (MFMA N)
constexpr int TT = 32;  // tokens per tile (MFMA M)
#ifndef MIO_MMQ_NT
#define MIO_MMQ_NT 512
#endif
constexpr int MMQ_NT = MIO_MMQ_NT;  // 8 waves: one per decode lane slot (64: one wave, all slots)

// token of accumulator register r of lane l
__device__ __forceinline__ int tok_of(int lane, int r) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Balanced pairwise sum over a stream of 2^L values pushed in order (the decode's DPP trees:
// ((s7+s6)+(s5+s4))+((s3+s2)+(s1+s0)) for L = 3), 16 tokens per lane.
template <int L, class V = v16f>
struct Tree {
    V lv[L];
    template <int I>
    __device__ __forceinline__ void push(V x) {
        // carry chain of the binary counter at index I (compile-time)
        if constexpr (L >= 1 && (I & 1)) x = lv[0] + x;
        if constexpr (L >= 2 && (I & 3) == 3) x = lv[1] + x;
        if constexpr (L >= 3 && (I & 7) == 7) x = lv[2] + x;
        if constexpr (L >= 4 && (I & 15) == 15) x = lv[3] + x;
        if constexpr (L >= 5 && (I & 31) == 31) x = lv[4] + x;
        if constexpr (L >= 6 && (I & 63) == 63) x = lv[5] + x;
        constexpr int lvl = (I & 1) == 0 ? 0 : (I & 3) != 3 ? 1 : (I & 7) != 7 ? 2 : (I & 15) != 15 ? 3
                          : (I & 31) != 31 ? 4 : (I & 63) != 63 ? 5 : 6;
        if constexpr (lvl < L) lv[lvl] = x;
        else result = x;
    }
    V result;
};

// 16 int8 activations of token row `t` (record base) at byte offset e.. e+15
__device__ __forceinline__ v4i act16(const int8_t *qs, int e) { return *reinterpret_cast<const v4i *>(qs + e); }

// ---------------------------------------------------------------- per-type slot products
// The 8 waves of a workgroup split a 32x32 tile's K by the decode engine's lane slots: wave k
// computes slot k's pass accumulation (superblocks s = p * 8 + k, p = 0, 1, ...; Q8_0: the
// 8 slots of lane group k, already summed by their 8-leaf tree), and wave 0 then sums the 8
// waves' results with the decode's tree (row_total). Each returns 16 values: this lane's row,
// its 16 tokens.

// Q4_K superblock s of row `row`: v = d * isum - dmin * imin per token (ggml vec_dot_q4_K_q8_K).
__device__ __forceinline__ v16f sb_q4k(const uint8_t *qrow, const uint8_t *hrow, int s, const int8_t *aq,
                                       const float *da_lds) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const uint4 hd = *reinterpret_cast<const uint4 *>(hrow + (size_t)s * 16);
    uint4 nb[4];
    v4i al[4], ah[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        nb[c] = *reinterpret_cast<const uint4 *>(qrow + (size_t)s * 128 + 32 * c + 16 * h);
        al[c] = act16(aq, s * 256 + 64 * c + 16 * h);
        ah[c] = act16(aq, s * 256 + 64 * c + 32 + 16 * h);
    }
    v16i isum = {}, imin = {};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        // scale/min pair word of sub-blocks 2c, 2c+1 (24 bits at bit 24c of hd.yzw)
        const uint32_t wlo = c < 2 ? hd.y : (c == 2 ? hd.z : hd.w);
        const uint32_t whi = c < 2 ? hd.z : hd.w;
        const uint32_t F = __builtin_amdgcn_alignbit(whi, wlo, (24 * c) & 31);
        const int sc0 = F & 63, m0 = (F >> 6) & 63, sc1 = (F >> 12) & 63, m1 = (F >> 18) & 63;
        const uint4 q = nb[c];
        const v4i blo = {(int)(q.x & M4), (int)(q.y & M4), (int)(q.z & M4), (int)(q.w & M4)};
        const v4i bhi = {(int)((q.x >> 4) & M4), (int)((q.y >> 4) & M4), (int)((q.z >> 4) & M4), (int)((q.w >> 4) & M4)};
        const v16i clo = __builtin_amdgcn_mfma_i32_32x32x32_i8(al[c], blo, v16i{}, 0, 0, 0);
        const v16i chi = __builtin_amdgcn_mfma_i32_32x32x32_i8(ah[c], bhi, v16i{}, 0, 0, 0);
        const int mb0 = m0 * 0x01010101, mb1 = m1 * 0x01010101;
        imin = __builtin_amdgcn_mfma_i32_32x32x32_i8(al[c], v4i{mb0, mb0, mb0, mb0}, imin, 0, 0, 0);
        imin = __builtin_amdgcn_mfma_i32_32x32x32_i8(ah[c], v4i{mb1, mb1, mb1, mb1}, imin, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) isum[r] += __mul24(sc0, clo[r]) + __mul24(sc1, chi[r]);
    }
    const float dw = h2f(hd.x & 0xFFFF), dmw = h2f(hd.x >> 16);
    v16f v;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float da = da_lds[s * TT + tok_of(lane, r)];
        const float d = dw * da, dmin = dmw * da;
        float x = d * (float)isum[r];
        x = x - dmin * (float)imin[r];
        v[r] = x;
    }
    return v;
}

// q - 32 for 4 packed 6-bit codes (signed int8): bit 5 set -> q & 31, clear -> q | 0xE0
__device__ __forceinline__ int q6s(uint32_t q) {
    const uint32_t t = q ^ 0x20202020u, m = t & 0x20202020u;
    return (int)(t | (m << 1) | (m << 2));
}

// Q6_K superblock s: 16 sub-blocks of 16 values, one 32x32x16 MFMA each on (q - 32);
// v = d * sum_j sc_j * C_j (ggml vec_dot_q6_K_q8_K).
__device__ __forceinline__ v16f sb_q6k(const QMat &W, int row, int s, const int8_t *aq, const float *da_lds) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int nsb = W.k >> 8;
    const uint8_t *qlrow = W.p0 + (size_t)row * (W.k / 2);
    const uint8_t *qhrow = W.p1 + (size_t)row * (W.k / 4);
    const int8_t *screw = (const int8_t *)W.p2 + (size_t)row * (W.k / 16);
    const uint16_t *drow = (const uint16_t *)W.p3 + (size_t)row * nsb;
    // split-layout scales: pair p2 = 4n + r -> {scales[8n + r], scales[8n + r + 4]}
    const uint4 scr = *reinterpret_cast<const uint4 *>(screw + (size_t)s * 16);
    int8_t sc[16];
    __builtin_memcpy(sc, &scr, 16);
    uint2 qh[2][2], ql[2][2][2];
    long aa[16];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            qh[n][b] = *reinterpret_cast<const uint2 *>(qhrow + (size_t)s * 64 + 32 * n + 16 * b + 8 * h);
#pragma unroll
            for (int a = 0; a < 2; ++a)
                ql[n][a][b] = *reinterpret_cast<const uint2 *>(qlrow + (size_t)s * 128 + 64 * n + 32 * a + 16 * b + 8 * h);
        }
#pragma unroll
    for (int j = 0; j < 16; ++j) aa[j] = *reinterpret_cast<const long *>(aq + s * 256 + 16 * j + 8 * h);
    v16i isum = {};
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int hi = 0; hi < 2; ++hi) {
                    // g = 2 hi + a: q1 (ql low, qh bits 0-1), q2 (ql[+32] low, bits 2-3), q3 (ql
                    // high, bits 4-5), q4 (ql[+32] high, bits 6-7); value 128n + 32g + 16b + 8h + i
                    const int g = 2 * hi + a;
                    const int j = 8 * n + 2 * g + b;  // sub-block (values 16j ..)
                    const uint2 l8 = ql[n][a][b], h8v = qh[n][b];
                    const uint32_t lx = hi ? (l8.x >> 4) & M4 : l8.x & M4;
                    const uint32_t ly = hi ? (l8.y >> 4) & M4 : l8.y & M4;
                    const uint32_t hx = ((h8v.x >> (2 * g)) & M2) << 4, hy = ((h8v.y >> (2 * g)) & M2) << 4;
                    const long bq = (long)(uint32_t)q6s(lx | hx) | ((long)(uint32_t)q6s(ly | hy) << 32);
                    const v16i c = __builtin_amdgcn_mfma_i32_32x32x16_i8(aa[j], bq, v16i{}, 0, 0, 0);
                    const int nn = j >> 3, rr = j & 7;
                    const int scj = rr < 4 ? sc[2 * (4 * nn + rr)] : sc[2 * (4 * nn + rr - 4) + 1];
#pragma unroll
                    for (int r = 0; r < 16; ++r) isum[r] += __mul24(scj, c[r]);
                }
    const float dw = h2f(drow[s]);
    v16f v;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float d = dw * da_lds[s * TT + tok_of(lane, r)];
        v[r] = d * (float)isum[r];
    }
    return v;
}

// slot k's pass accumulation (K-quants)
template <int T>
__device__ v16f slot_kq(const QMat &W, int row, int k, const int8_t *aq, const float *da_lds) {
    const int nsb = W.k >> 8, NP = (nsb + 7) / 8;
    v16f acc = {};
    for (int p = 0; p < NP; ++p) {
        const int s = p * 8 + k;
        v16f v = {};
        if (s < nsb) {
            if constexpr (T == 12)
                v = sb_q4k(W.p0 + (size_t)row * (W.k / 2), W.p1 + (size_t)row * nsb * 16, s, aq, da_lds);
            else
                v = sb_q6k(W, row, s, aq, da_lds);
        }
        acc = acc + v;  // the decode lane's pass accumulation (0 + v0 + v1 ...)
    }
    return acc;
}

// Q8_0: lane group k = slots 8k .. 8k+7 (block b = p * 64 + slot), each slot's pass sum,
// then sum8_f's tree over the group. With one pass (K <= 2048) the 8 slots' weight /
// activation / scale loads are all issued before the first MFMA (one memory round trip, not
// eight); longer K goes four slots at a time (register budget). Same arithmetic and order
// either way.
// One-pass Q8_0 slot (K <= 2048) in registers: the loads are issued by q80_load before the
// tile's activation-scale staging and its barrier (one memory round trip per workgroup, not
// two), q80_sum runs after it.
struct Q80Regs {
    v4i w[8], a[8];
    float dw[8];
};
__device__ __forceinline__ void q80_load(const QMat &W, int row, int k, const int8_t *aq, Q80Regs &q) {
    const int h = (threadIdx.x & 63) >> 5;
    const int nb = W.k >> 5;
    const int8_t *qrow = (const int8_t *)W.p0 + (size_t)row * W.k;
    const uint16_t *drow = (const uint16_t *)W.p1 + (size_t)row * nb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int b = min(8 * k + i, nb - 1);  // clamped: every load in flight at once
        q.w[i] = *reinterpret_cast<const v4i *>(qrow + (size_t)b * 32 + 16 * h);
        q.a[i] = act16(aq, b * 32 + 16 * h);
        q.dw[i] = h2f(drow[b]);
    }
}
__device__ __forceinline__ v16f q80_sum(const Q80Regs &q, int nb, int k, const float *da_lds) {
    const int lane = threadIdx.x & 63;
    Tree<3> inner;
    auto slot1 = [&]<int i>() {
        const int b = 8 * k + i;
        v16f v = {};
        if (b < nb) {  // wave-uniform: the MFMA runs with the full EXEC
            const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(q.a[i], q.w[i], v16i{}, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = (float)c[r] * (q.dw[i] * da_lds[b * TT + tok_of(lane, r)]);
        }
        const v16f acc = v16f{} + v;
        inner.template push<i>(acc);
    };
    slot1.template operator()<0>();
    slot1.template operator()<1>();
    slot1.template operator()<2>();
    slot1.template operator()<3>();
    slot1.template operator()<4>();
    slot1.template operator()<5>();
    slot1.template operator()<6>();
    slot1.template operator()<7>();
    return inner.result;
}

__device__ v16f slot_q80(const QMat &W, int row, int k, const int8_t *aq, const float *da_lds) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int nb = W.k >> 5, NP = (nb + 63) / 64;
    const int8_t *qrow = (const int8_t *)W.p0 + (size_t)row * W.k;
    const uint16_t *drow = (const uint16_t *)W.p1 + (size_t)row * nb;
    Tree<3> inner;
    if (NP == 1) {
        Q80Regs q;
        q80_load(W, row, k, aq, q);
        return q80_sum(q, nb, k, da_lds);
    }
    // several passes (K > 2048): four slots at a time, each pass's loads of the four issued
    // together (two round trips per pass instead of eight); slot i still accumulates its
    // passes in order and enters the tree in slot order
    auto half = [&]<int H>() {
        v16f acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = v16f{};
        for (int p = 0; p < NP; ++p) {
            v4i w[4], a[4];
            float dw[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int b = min(p * 64 + 8 * k + 4 * H + i, nb - 1);
                w[i] = *reinterpret_cast<const v4i *>(qrow + (size_t)b * 32 + 16 * h);
                a[i] = act16(aq, b * 32 + 16 * h);
                dw[i] = h2f(drow[b]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int b = p * 64 + 8 * k + 4 * H + i;
                v16f v = {};
                if (b < nb) {
                    const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], w[i], v16i{}, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 16; ++r) v[r] = (float)c[r] * (dw[i] * da_lds[b * TT + tok_of(lane, r)]);
                }
                acc[i] = acc[i] + v;
            }
        }
        inner.template push<4 * H + 0>(acc[0]);
        inner.template push<4 * H + 1>(acc[1]);
        inner.template push<4 * H + 2>(acc[2]);
        inner.template push<4 * H + 3>(acc[3]);
    };
    half.template operator()<0>();
    half.template operator()<1>();
    return inner.result;
}

template <int T>
__device__ __forceinline__ v16f slot_val(const QMat &W, int row, int k, const int8_t *aq, const float *da_lds) {
    if constexpr (T == 8) return slot_q80(W, row, k, aq, da_lds);
    else return slot_kq<T>(W, row, k, aq, da_lds);
}

// The activation scales of the tile's tokens into LDS as [group][token] (Q8_K: one per 256,
// Q8_0: one per 32; the whole workgroup, then a barrier); returns this lane's token's codes.
template <int T>
__device__ __forceinline__ const int8_t *stage_act(const MmqArgs &a, int t0, int K, float *da_lds) {
    const int ng = T == 8 ? K >> 5 : K >> 8;
    const size_t ab = a.act_stride;
    for (int e = threadIdx.x; e < ng * TT; e += MMQ_NT) {
        const int g = e / TT, t = min(t0 + e % TT, a.nt - 1);
        da_lds[e] = reinterpret_cast<const float *>(a.act + (size_t)t * ab + K)[g];
    }
    __syncthreads();
    const int t = min(t0 + (threadIdx.x & 31), a.nt - 1);
    return reinterpret_cast<const int8_t *>(a.act + (size_t)t * ab);
}
// this lane's token's codes (no loads)
__device__ __forceinline__ const int8_t *act_codes(const MmqArgs &a, int t0) {
    const int t = min(t0 + (threadIdx.x & 31), a.nt - 1);
    return reinterpret_cast<const int8_t *>(a.act + (size_t)t * a.act_stride);
}

// sum of the 8 waves' slot values with the decode's row_total tree (valid in wave 0): each
// wave stores its slot value(s) (NV sets: gate and up of SwiGLU share one barrier), then wave
// 0 reads the 8 slots of every set in slot order
__device__ __forceinline__ void slot_store(const v16f &mine, float *red) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *dst = red + ((size_t)wave * 64 + lane) * 16;
#pragma unroll
    for (int r = 0; r < 16; r += 4) *reinterpret_cast<float4 *>(dst + r) = make_float4(mine[r], mine[r + 1], mine[r + 2], mine[r + 3]);
}
__device__ __forceinline__ v16f slot_sum(const float *red) {
    const int lane = threadIdx.x & 63;
    Tree<3> t;
    auto leaf = [&]<int k>() {
        const float *src = red + ((size_t)k * 64 + lane) * 16;
        v16f x;
#pragma unroll
        for (int r = 0; r < 16; r += 4) {
            const float4 f = *reinterpret_cast<const float4 *>(src + r);
            x[r] = f.x, x[r + 1] = f.y, x[r + 2] = f.z, x[r + 3] = f.w;
        }
        t.template push<k>(x);
    };
    leaf.template operator()<0>();
    leaf.template operator()<1>();
    leaf.template operator()<2>();
    leaf.template operator()<3>();
    leaf.template operator()<4>();
    leaf.template operator()<5>();
    leaf.template operator()<6>();
    leaf.template operator()<7>();
    return t.result;
}

// the tile's 16 row totals per lane of W (and of U when NV = 2), valid in wave 0
template <int T, int NV>
__device__ __forceinline__ void all_slots(const QMat &W, const QMat &U, int row, const int8_t *aq, const float *da,
                                          float *red, v16f &y, v16f &u) {
    // the slot index must be wave-uniform in the compiler's eyes: a VGPR-held slot makes
    // every superblock branch divergent, and the matrix-core ops inside it then ran with
    // a partial EXEC (wrong sums; tests/test_llm_gpu.py::test_mmq_equals_single_token_matvec)
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    slot_store(slot_val<T>(W, row, k, aq, da), red);
    if constexpr (NV == 2) slot_store(slot_val<T>(U, row, k, aq, da), red + MMQ_NT * 16);
    __syncthreads();
    if (k == 0) {
        y = slot_sum(red);
        if constexpr (NV == 2) u = slot_sum(red + MMQ_NT * 16);
    }
}

template <int T0, int T1, int T2, int MODE>
__global__ __launch_bounds__(MMQ_NT) void k_mmq(MmqSeg s0, MmqSeg s1, MmqSeg s2, MmqArgs a, MmqQuant) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    float *red = reinterpret_cast<float *>(lds);                          // [8 waves][64][16] (x2 SWIGLU)
    float *da = red + (MODE == MMQ_SWIGLU ? 2 : 1) * MMQ_NT * 16;         // [groups][32 tokens]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t0 = blockIdx.y * TT;
    int tile_id = blockIdx.x;
    // segment of this tile (uniform branch): q | k | v of the attention input, or one matrix
    auto run = [&]<int T>(const MmqSeg &sg, int ti) {
        const int row0 = ti * RT, row = min(row0 + (lane & 31), sg.w.rows - 1);
        v16f y = {}, u = {};
        if (T == 8 && a.K <= 2048) {
            // one pass: the slot's weight / code / scale loads go out before the activation
            // scales' staging barrier (same values, same order of every float operation)
            const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            const int8_t *aq = act_codes(a, t0);
            Q80Regs qw, qu;
            q80_load(sg.w, row, k, aq, qw);
            if constexpr (MODE == MMQ_SWIGLU) q80_load(a.w_up, row, k, aq, qu);
            stage_act<8>(a, t0, a.K, da);
            slot_store(q80_sum(qw, sg.w.k >> 5, k, da), red);
            if constexpr (MODE == MMQ_SWIGLU) slot_store(q80_sum(qu, a.w_up.k >> 5, k, da), red + MMQ_NT * 16);
            __syncthreads();
            if (k == 0) {
                y = slot_sum(red);
                if constexpr (MODE == MMQ_SWIGLU) u = slot_sum(red + MMQ_NT * 16);
            }
        } else {
            const int8_t *aq = stage_act<T>(a, t0, a.K, da);
            all_slots<T, MODE == MMQ_SWIGLU ? 2 : 1>(sg.w, a.w_up, row, aq, da, red, y, u);
        }
        const int orow = row0 + (lane & 31);
        if (wave != 0 || orow >= sg.w.rows) return;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int t = t0 + tok_of(lane, r);
            if (t >= a.nt) continue;
            float *o = a.out + (size_t)t * a.ld + sg.out_off + orow;
            if constexpr (MODE == MMQ_STORE) *o = y[r];
            else if constexpr (MODE == MMQ_RESID) *o = y[r] + *o;
            else *o = silu_f(y[r]) * u[r];
        }
    };
    if (tile_id < s0.tiles) return run.template operator()<T0>(s0, tile_id);
    tile_id -= s0.tiles;
    if constexpr (T1 >= 0) {
        if (tile_id < s1.tiles) return run.template operator()<T1>(s1, tile_id);
        tile_id -= s1.tiles;
    }
    if constexpr (T2 >= 0) {
        if (tile_id < s2.tiles) return run.template operator()<T2>(s2, tile_id);
    }
}

// ---------------------------------------------------------------- 16-row x 16-token tiles
// The same matmul for launches of at most 16 tokens (the batched decode of up to 16
// utterances) on v_mfma_i32_16x16x32_i8: a 32x32 tile pads 8 tokens to 32 (75 % of every
// MFMA and of its float epilogue wasted) and gives a 2048-row matrix 64 tiles; 16 x 16 tiles
// pad to 16 and give it 128. Operands (8 bytes per lane): lane l holds token / weight row
// l & 15 and the 8 K elements 8 (l >> 4) .. +7 of the 32-element group; the result: lane l,
// weight row l & 15, tokens 4 (l >> 4) + i (tools/micro/mfma_i8_probe, 16x16x32_i8 hyp 1).
// Per group the integer dot is exact and the scales, per-lane pass accumulation and the
// decode's trees are applied exactly as in the 32 x 32 kernel above: every (row, token)
// equals the single-token decode step bit for bit.
constexpr int RT16 = 16, TT16 = 16;
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int tok16(int lane, int i) { return 4 * (lane >> 4) + i; }
__device__ __forceinline__ long act8(const int8_t *qs, int e) { return *reinterpret_cast<const long *>(qs + e); }
__device__ __forceinline__ v4i mfma16(long a, long b, v4i c) {
    return __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ long lo_nib(uint2 q) {
    return (long)(uint32_t)(q.x & M4) | ((long)(uint32_t)(q.y & M4) << 32);
}
__device__ __forceinline__ long hi_nib(uint2 q) {
    return (long)(uint32_t)((q.x >> 4) & M4) | ((long)(uint32_t)((q.y >> 4) & M4) << 32);
}

// Q8_0 with 16-B loads (K % 256 == 0): lane (row / token l & 15, group g = l >> 4) loads 16 B
// at byte 16 g of a 64-B block pair (b, b + 1) - groups 0, 1 hold block b, groups 2, 3 block
// b + 1 - and one v_permlane32_swap per dword swaps the high 8 B of lanes 0-31 with the low
// 8 B of lanes 32-63: the low halves of the 4 groups are then block b's bytes {0-7, 16-23,
// 8-15, 24-31}, the high halves block b + 1's, in the weights and in the activations alike, so
// one 16x16x32 MFMA per block gives the same exact integer dot. A wave's 8 weight scales of a
// pass are one 16-B load. Per wave and pass: 4 weight loads per matrix, 4 activation loads,
// one scale load per matrix, instead of 8 + 8 + 8 (8-B weights / activations, 2-B scales):
// the vector-memory instruction count is what bounds these launches at 8 tokens
// (tools/micro/mmq_probe.hip: 2 x 10752 x 2048 gate|up 28.7 -> 13.7 us, bit-equal).
__device__ __forceinline__ void swap_halves(v4i &x) {
    const auto p = __builtin_amdgcn_permlane32_swap(x.x, x.z, false, false);
    const auto q = __builtin_amdgcn_permlane32_swap(x.y, x.w, false, false);
    x.x = p[0], x.z = p[1], x.y = q[0], x.w = q[1];
}
__device__ __forceinline__ long lo8(const v4i &x) { return (long)(uint32_t)x.x | ((long)(uint32_t)x.y << 32); }
__device__ __forceinline__ long hi8(const v4i &x) { return (long)(uint32_t)x.z | ((long)(uint32_t)x.w << 32); }

// Q4_K superblock s: v = d * isum - dmin * imin per token (ggml vec_dot_q4_K_q8_K). Loads as
// in the Q8_0 pair path (swap_halves): the 32-B nibble runs of sub-block pairs c, c + 1 are
// one 16-B load per lane, the 64 activation bytes of sub-blocks 2c, 2c + 1 another; after the
// swaps the low / high halves hold one run / one sub-block each in the same K order.
struct Q4Pass {
    uint4 hd;
    v4i w[2];
};
__device__ __forceinline__ void q4p_load(const uint8_t *qrow, const uint8_t *hrow, int s, Q4Pass &p) {
    const int g = (threadIdx.x & 63) >> 4;
    p.hd = *reinterpret_cast<const uint4 *>(hrow + (size_t)s * 16);
#pragma unroll
    for (int i = 0; i < 2; ++i) p.w[i] = *reinterpret_cast<const v4i *>(qrow + (size_t)s * 128 + 64 * i + 16 * g);
}
// x: the superblock's activation codes of this lane, already swap_halves'd
__device__ __forceinline__ v4f q4p_val(Q4Pass p, const v4i (&x)[4], int s, const float *da_lds) {
    const int lane = threadIdx.x & 63;
    const uint4 hd = p.hd;
    v4i (&w)[2] = p.w;
#pragma unroll
    for (int i = 0; i < 2; ++i) swap_halves(w[i]);
    v4i isum = {}, imin = {};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t wlo = c < 2 ? hd.y : (c == 2 ? hd.z : hd.w);
        const uint32_t whi = c < 2 ? hd.z : hd.w;
        const uint32_t F = __builtin_amdgcn_alignbit(whi, wlo, (24 * c) & 31);
        const int sc0 = F & 63, m0 = (F >> 6) & 63, sc1 = (F >> 12) & 63, m1 = (F >> 18) & 63;
        const long q = (c & 1) ? hi8(w[c >> 1]) : lo8(w[c >> 1]);
        const long al = lo8(x[c]), ah = hi8(x[c]);
        const v4i clo = mfma16(al, q & 0x0F0F0F0F0F0F0F0Fl, v4i{});
        const v4i chi = mfma16(ah, (q >> 4) & 0x0F0F0F0F0F0F0F0Fl, v4i{});
        const long mb0 = (long)(uint32_t)(m0 * 0x01010101) * 0x100000001l;
        const long mb1 = (long)(uint32_t)(m1 * 0x01010101) * 0x100000001l;
        imin = mfma16(al, mb0, imin);
        imin = mfma16(ah, mb1, imin);
#pragma unroll
        for (int i = 0; i < 4; ++i) isum[i] += __mul24(sc0, clo[i]) + __mul24(sc1, chi[i]);
    }
    const float dw = h2f(hd.x & 0xFFFF), dmw = h2f(hd.x >> 16);
    v4f v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float da = da_lds[s * TT16 + tok16(lane, i)];
        const float d = dw * da, dmin = dmw * da;
        float xx = d * (float)isum[i];
        xx = xx - dmin * (float)imin[i];
        v[i] = xx;
    }
    return v;
}
// A lane's activation record in the launches whose own producer workgroups wrote it (in-launch
// quantization, QNP > 0): the wave-uniform record base plus this lane's token offset, read with
// 16-B / 4-B sc1 buffer loads (L1 bypassed). The producers store every record byte sc1, drain
// them and add to 8 counter replicas behind a workgroup barrier; the consumer polls one replica
// and releases its waves with a barrier: MI355X_MICROARCH's replica-counter hand-off, whose
// loads must ALL be sc1 loads (plain loads after a relaxed poll may return a stale L1 line;
// round 5's repair was an agent-scope acquire per workgroup, an L1 invalidate that also waited
// for the early weight loads: 8 streams 240 -> 140x). Records an earlier launch wrote stay
// plain pointers (the kernel boundary orders them).
struct ActSc1 {
    const char *base;
    uint32_t off;
};
__device__ __forceinline__ v4i ld_act16(const int8_t *p, int o) { return *reinterpret_cast<const v4i *>(p + o); }
__device__ __forceinline__ v4i ld_act16(const ActSc1 &p, int o) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(p.base, 0x7FFFFFF0u), p.off + (uint32_t)o, 0, 16);
    return v4i{(int)v.x, (int)v.y, (int)v.z, (int)v.w};
}
__device__ __forceinline__ float ld_scale(const char *base, size_t off, bool sc1) {
    if (sc1)
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(base, 0x7FFFFFF0u), (uint32_t)off, 0, 16));
    return *reinterpret_cast<const float *>(base + off);
}

// this lane's activation codes of superblock s (kq_act_ld: the loads alone, so a caller can
// issue them ahead of the scales' staging round trip; kq_act: loaded and swap_halves'd)
template <class AP>
__device__ __forceinline__ void kq_act_ld(const AP &aq, int s, v4i (&x)[4]) {
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = ld_act16(aq, s * 256 + 64 * c + 16 * g);
}
template <class AP>
__device__ __forceinline__ void kq_act(const AP &aq, int s, v4i (&x)[4]) {
    kq_act_ld(aq, s, x);
#pragma unroll
    for (int c = 0; c < 4; ++c) swap_halves(x[c]);
}
template <class AP>
__device__ __forceinline__ v4f sb16_q4k(const uint8_t *qrow, const uint8_t *hrow, int s, const AP &aq,
                                        const float *da_lds) {
    Q4Pass p;
    q4p_load(qrow, hrow, s, p);
    v4i x[4];
    kq_act(aq, s, x);
    return q4p_val(p, x, s, da_lds);
}

// Q6_K superblock s: v = d * sum_j sc_j * dot_j over its 16 sub-blocks of 16 (ggml
// vec_dot_q6_K_q8_K). A q-group (n, g4) = values 128 n + 32 g4 + l, l < 32: low (g4 0, 1) or
// high (g4 2, 3) nibbles of ql[64 n + 32 (g4 & 1) + l] with bits 2 g4 of qh[32 n + l], i.e.
// sub-blocks 8 n + 2 g4 and + 1. Loads as in the Q8_0 pair path (swap_halves): ql's 64 B of
// half n, qh's 64 B and the 64 activation bytes of q-groups (n, 2i), (n, 2i + 1) are one 16-B
// load per lane each; after the swaps every lane holds 8 values l in {0-7, 16-23, 8-15, 24-31}
// of its group g, so sub-block 8 n + 2 g4 lies in groups 0, 2 and the next one in groups 1, 3:
// two 16x16x32 MFMAs per q-group, each on one sub-block's lanes (the others zero).
// the weight loads of superblock s of `row` (sb16_q6k's), kept apart so a tile loop can hold
// the next tile's in flight (k_mmq16_loop_kq)
struct Q6Pass {
    uint4 scr;
    v4i ql[2], qh;
    uint16_t d;
};
__device__ __forceinline__ void q6p_load(const QMat &W, int row, int s, Q6Pass &p) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int nsb = W.k >> 8;
    const uint8_t *qlrow = W.p0 + (size_t)row * (W.k / 2);
    const uint8_t *qhrow = W.p1 + (size_t)row * (W.k / 4);
    const int8_t *screw = (const int8_t *)W.p2 + (size_t)row * (W.k / 16);
    const uint16_t *drow = (const uint16_t *)W.p3 + (size_t)row * nsb;
    // split-layout scales: pair p2 = 4n + r -> {scales[8n + r], scales[8n + r + 4]}
    p.scr = *reinterpret_cast<const uint4 *>(screw + (size_t)s * 16);
#pragma unroll
    for (int n = 0; n < 2; ++n) p.ql[n] = *reinterpret_cast<const v4i *>(qlrow + (size_t)s * 128 + 64 * n + 16 * g);
    p.qh = *reinterpret_cast<const v4i *>(qhrow + (size_t)s * 64 + 16 * g);
    p.d = drow[s];
}
// x: the superblock's activation codes of this lane, already swap_halves'd
__device__ __forceinline__ v4f q6p_val(Q6Pass p, const v4i (&x)[4], int s, const float *da_lds) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const bool first = (g & 1) == 0;  // groups 0, 2: the q-group's first sub-block
    int8_t sc[16];
    __builtin_memcpy(sc, &p.scr, 16);
    v4i (&ql)[2] = p.ql;
    v4i &qh = p.qh;
    const float dw = h2f(p.d);
    swap_halves(ql[0]);
    swap_halves(ql[1]);
    swap_halves(qh);
    v4i isum = {};
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const uint32_t hw0 = n ? (uint32_t)qh.z : (uint32_t)qh.x, hw1 = n ? (uint32_t)qh.w : (uint32_t)qh.y;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            // ql bytes 32 (g4 & 1) + l of half n: the low (g4 & 1 == 0) or high halves after the swap
            const uint32_t lw0 = (g4 & 1) ? (uint32_t)ql[n].z : (uint32_t)ql[n].x;
            const uint32_t lw1 = (g4 & 1) ? (uint32_t)ql[n].w : (uint32_t)ql[n].y;
            const int sh = 4 * (g4 >> 1);
            const uint32_t b0 = q6s(((lw0 >> sh) & M4) | (((hw0 >> (2 * g4)) & M2) << 4));
            const uint32_t b1 = q6s(((lw1 >> sh) & M4) | (((hw1 >> (2 * g4)) & M2) << 4));
            const long bq = (long)b0 | ((long)b1 << 32);
            const v4i &xa = x[2 * n + (g4 >> 1)];
            const long a = (g4 & 1) ? hi8(xa) : lo8(xa);
            const v4i c0 = mfma16(first ? a : 0l, bq, v4i{});
            const v4i c1 = mfma16(first ? 0l : a, bq, v4i{});
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j = 8 * n + 2 * g4 + h;  // sub-block
                const int nn = j >> 3, rr = j & 7;
                const int scj = rr < 4 ? sc[2 * (4 * nn + rr)] : sc[2 * (4 * nn + rr - 4) + 1];
                const v4i &c = h ? c1 : c0;
#pragma unroll
                for (int i = 0; i < 4; ++i) isum[i] += __mul24(scj, c[i]);
            }
        }
    }
    v4f v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float d = dw * da_lds[s * TT16 + tok16(lane, i)];
        v[i] = d * (float)isum[i];
    }
    return v;
}

template <class AP>
__device__ __forceinline__ v4f sb16_q6k(const QMat &W, int row, int s, const AP &aq, const float *da_lds) {
    Q6Pass p;
    q6p_load(W, row, s, p);
    v4i x[4];
    kq_act(aq, s, x);
    return q6p_val(p, x, s, da_lds);
}

template <int T, class AP>
__device__ v4f slot16_kq(const QMat &W, int row, int k, const AP &aq, const float *da_lds) {
    const int nsb = W.k >> 8, NP = (nsb + 7) / 8;
    v4f acc = {};
    for (int p = 0; p < NP; ++p) {
        const int s = p * 8 + k;
        v4f v = {};
        if (s < nsb) {
            if constexpr (T == 12)
                v = sb16_q4k(W.p0 + (size_t)row * (W.k / 2), W.p1 + (size_t)row * nsb * 16, s, aq, da_lds);
            else
                v = sb16_q6k(W, row, s, aq, da_lds);
        }
        acc = acc + v;  // the decode lane's pass accumulation (0 + v0 + v1 ...)
    }
    return acc;
}

// Q8_0: slots 8k .. 8k+7 of lane group k (block b = p * 64 + slot), each slot's pass sum in
// order, then sum8_f's tree over the 8 slots; per pass the 8 blocks' loads go out together
__device__ v4f slot16_q80(const QMat &W, int row, int k, const int8_t *aq, const float *da_lds) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int nb = W.k >> 5, NP = (nb + 63) / 64;
    const int8_t *qrow = (const int8_t *)W.p0 + (size_t)row * W.k;
    const uint16_t *drow = (const uint16_t *)W.p1 + (size_t)row * nb;
    v4f acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = v4f{};
    for (int p = 0; p < NP; ++p) {
        long w[8], a[8];
        float dw[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int b = min(p * 64 + 8 * k + i, nb - 1);  // clamped: every load in flight at once
            w[i] = *reinterpret_cast<const long *>(qrow + (size_t)b * 32 + 8 * g);
            a[i] = act8(aq, b * 32 + 8 * g);
            dw[i] = h2f(drow[b]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int b = p * 64 + 8 * k + i;
            v4f v = {};
            if (b < nb) {  // wave-uniform
                const v4i c = mfma16(a[i], w[i], v4i{});
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (float)c[j] * (dw[i] * da_lds[b * TT16 + tok16(lane, j)]);
            }
            acc[i] = acc[i] + v;
        }
    }
    Tree<3, v4f> inner;
    inner.template push<0>(acc[0]);
    inner.template push<1>(acc[1]);
    inner.template push<2>(acc[2]);
    inner.template push<3>(acc[3]);
    inner.template push<4>(acc[4]);
    inner.template push<5>(acc[5]);
    inner.template push<6>(acc[6]);
    inner.template push<7>(acc[7]);
    return inner.result;
}

struct Q80Pass {
    v4i w[4];
    v4i ds;  // the 8 blocks' f16 scales
};
// pass p of slot group k (blocks p * 64 + 8 k .. + 7; the group is wave-uniform, and with
// K % 256 == 0 either all of its blocks exist or none: clamped loads, values skipped)
__device__ __forceinline__ void q80p_load(const QMat &W, int row, int p, int k, Q80Pass &q) {
    const int g = (threadIdx.x & 63) >> 4, nb = W.k >> 5;
    const int b0 = min(p * 64 + 8 * k, nb - 8);
    const int8_t *qrow = (const int8_t *)W.p0 + (size_t)row * W.k;
#pragma unroll
    for (int i = 0; i < 4; ++i) q.w[i] = *reinterpret_cast<const v4i *>(qrow + (size_t)(b0 + 2 * i) * 32 + 16 * g);
    q.ds = *reinterpret_cast<const v4i *>((const uint16_t *)W.p1 + (size_t)row * nb + b0);
}
template <class AP>
__device__ __forceinline__ void act_load(const AP &aq, int K, int p, int k, v4i (&a)[4]) {
    const int g = (threadIdx.x & 63) >> 4;
    const int b0 = min(p * 64 + 8 * k, (K >> 5) - 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ld_act16(aq, (b0 + 2 * i) * 32 + 16 * g);
}
// the 8 slots' values of one pass added to acc (a: the pass's activations, already swapped)
__device__ __forceinline__ void q80p_acc(Q80Pass &q, const v4i (&a)[4], int p, int k, int nb, const float *da_lds,
                                         v4f (&acc)[8]) {
    const int lane = threadIdx.x & 63;
    const int b0 = p * 64 + 8 * k;
#pragma unroll
    for (int i = 0; i < 4; ++i) swap_halves(q.w[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v4f v = {};
        if (b0 < nb) {  // wave-uniform
            const v4i &w = q.w[i >> 1], &x = a[i >> 1];
            const v4i c = (i & 1) ? mfma16(hi8(x), hi8(w), v4i{}) : mfma16(lo8(x), lo8(w), v4i{});
            const uint32_t dd = (uint32_t)q.ds[i >> 1];
            const float dw = h2f((i & 1) ? dd >> 16 : dd & 0xFFFF);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (float)c[j] * (dw * da_lds[(b0 + i) * TT16 + tok16(lane, j)]);
        }
        acc[i] = acc[i] + v;
    }
}
__device__ __forceinline__ v4f tree8(const v4f (&acc)[8]) {
    Tree<3, v4f> t;
    t.template push<0>(acc[0]);
    t.template push<1>(acc[1]);
    t.template push<2>(acc[2]);
    t.template push<3>(acc[3]);
    t.template push<4>(acc[4]);
    t.template push<5>(acc[5]);
    t.template push<6>(acc[6]);
    t.template push<7>(acc[7]);
    return t.result;
}
// NV matrices (W, then U) over the same activations, one pass at a time
template <int NV, class AP>
__device__ __forceinline__ void slot16_q80p(const QMat &W, const QMat &U, int row, int k, const AP &aq,
                                            const float *da_lds, v4f &y, v4f &u) {
    const int nb = W.k >> 5, NP = (nb + 63) / 64;
    v4f aw[8], au[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) aw[i] = v4f{}, au[i] = v4f{};
    for (int p = 0; p < NP; ++p) {
        Q80Pass qw, qu;
        v4i x[4];
        q80p_load(W, row, p, k, qw);
        if constexpr (NV == 2) q80p_load(U, row, p, k, qu);
        act_load(aq, W.k, p, k, x);
#pragma unroll
        for (int i = 0; i < 4; ++i) swap_halves(x[i]);
        q80p_acc(qw, x, p, k, nb, da_lds, aw);
        if constexpr (NV == 2) q80p_acc(qu, x, p, k, nb, da_lds, au);
    }
    y = tree8(aw);
    if constexpr (NV == 2) u = tree8(au);
}

template <int T, class AP>
__device__ __forceinline__ v4f slot16_val(const QMat &W, int row, int k, const AP &aq, const float *da_lds) {
    if constexpr (T == 8) {
        // the 8-B Q8_0 path (K % 256 != 0) never runs in an in-launch-quantization launch
        // (launch_mmq_q takes K % 256 == 0 only)
        if constexpr (std::is_same_v<AP, ActSc1>) return v4f{};
        else return slot16_q80(W, row, k, aq, da_lds);
    } else {
        return slot16_kq<T>(W, row, k, aq, da_lds);
    }
}

// this lane's token's codes (A operand: token lane & 15; no loads); SC: the producers of this
// launch wrote them (ActSc1, sc1 loads)
template <bool SC>
__device__ __forceinline__ auto act16_codes(const MmqArgs &a, int t0) {
    const int t = min(t0 + (threadIdx.x & 15), a.nt - 1);
    if constexpr (SC)
        return ActSc1{a.act, (uint32_t)((size_t)t * a.act_stride)};
    else
        return reinterpret_cast<const int8_t *>(a.act + (size_t)t * a.act_stride);
}

// activation scales of the tile's 16 tokens -> LDS [group][token]; returns this lane's
// token's codes (A operand: token lane & 15)
template <int T, bool SC = false>
__device__ __forceinline__ auto stage_act16(const MmqArgs &a, int t0, int K, float *da_lds) {
    const int ng = T == 8 ? K >> 5 : K >> 8;
    const size_t ab = a.act_stride;
    // token-major walk: consecutive threads read consecutive scales of one record
    for (int e = threadIdx.x; e < ng * TT16; e += MMQ_NT) {
        const int tt = e / ng, g = e - tt * ng, t = min(t0 + tt, a.nt - 1);
        da_lds[g * TT16 + tt] = ld_scale(a.act, (size_t)t * ab + K + 4 * (size_t)g, SC);
    }
    __syncthreads();
    return act16_codes<SC>(a, t0);
}

__device__ __forceinline__ void slot16_store(const v4f &mine, float *red) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    *reinterpret_cast<float4 *>(red + ((size_t)wave * 64 + lane) * 4) = make_float4(mine[0], mine[1], mine[2], mine[3]);
}
__device__ __forceinline__ v4f slot16_sum(const float *red) {
    const int lane = threadIdx.x & 63;
    Tree<3, v4f> t;
    auto leaf = [&]<int k>() {
        const float4 f = *reinterpret_cast<const float4 *>(red + ((size_t)k * 64 + lane) * 4);
        t.template push<k>(v4f{f.x, f.y, f.z, f.w});
    };
    leaf.template operator()<0>();
    leaf.template operator()<1>();
    leaf.template operator()<2>();
    leaf.template operator()<3>();
    leaf.template operator()<4>();
    leaf.template operator()<5>();
    leaf.template operator()<6>();
    leaf.template operator()<7>();
    return t.result;
}

// KP: the launch is Q8_0 with K % 256 == 0 and (1) K <= 2048 or (2) K > 2048 (host-checked),
// so only that pair path is compiled into it: the generic kernel (KP 0) carries three Q8_0
// paths, and its size alone cost the 2.6B gate|up launch 19.2 vs 14.4 us
// In-launch quantization producer (launch_mmq_q): workgroup t quantizes token t's input with
// k_bt_quant's arithmetic into an LDS record laid out as the global one, copies it out with
// 16-B write-through stores, drains them and adds 1 to each of the 8 counter shards. Workgroup
// 0 also zeroes the other counter set (the next fused launch's).
template <int AK, int QNP, int QM>
__device__ __forceinline__ void mmq_quant_producer(const MmqArgs &a, const MmqQuant &q, char *lds) {
    const int t = blockIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 8)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(q.other + 64 * threadIdx.x), 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    Smem st = carve(lds + act_bytes(a.K), a.K);
    st.a = carve_t(lds, a.K, 0).a;
    XRegs<QNP> xr;
    load_x(q.src + (size_t)t * a.K, QM == 0 ? q.norm_w : nullptr, a.K, xr);
    if constexpr (QM == 0)
        rmsnorm_quant(xr, a.K, q.eps, AK, st);
    else
        plain_quant(xr, a.K, AK, st);
    const int n16 = (int)(act_bytes(a.K) / 16);
    const auto dst = rsrc(a.act + (size_t)t * a.act_stride, (uint32_t)act_bytes(a.K));
    for (int i = threadIdx.x; i < n16; i += MMQ_NT) {
        const uint4 v = reinterpret_cast<const uint4 *>(lds)[i];
        u32x4 u;
        u.x = v.x, u.y = v.y, u.z = v.z, u.w = v.w;
        __builtin_amdgcn_raw_buffer_store_b128(u, dst, i * 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 8)
        __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(q.cnt + 64 * threadIdx.x), 1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int T>
using KqPass = std::conditional_t<T == 12, Q4Pass, Q6Pass>;
template <int T>
__device__ __forceinline__ void kqp_load(const QMat &W, int row, int s, KqPass<T> &p) {
    if constexpr (T == 12)
        q4p_load(W.p0 + (size_t)row * (W.k / 2), W.p1 + (size_t)row * (W.k >> 8) * 16, s, p);
    else
        q6p_load(W, row, s, p);
}
template <int T>
__device__ __forceinline__ v4f kqp_val(const KqPass<T> &p, const v4i (&x)[4], int s, const float *da) {
    if constexpr (T == 12)
        return q4p_val(p, x, s, da);
    else
        return q6p_val(p, x, s, da);
}

// MIO_MMQ_XPRE (A/B builds; default 1): k_mmq16's residual epilogue adds values loaded at the
// tile's start instead of loading them behind the reduction
#ifndef MIO_MMQ_XPRE
#define MIO_MMQ_XPRE 1
#endif
// MIO_LOOP_D (A/B builds; default 4): tiles whose weights a tile-walking workgroup
// (k_mmq16_loop, k_mmq16_loop_kq) holds: D - 1 in flight while one is reduced (2 = the
// ping-pong of rounds 4-5; 4 holds every tile of the 1.7B / 2.6B gate|up walks, <= 4 per
// workgroup, before the producers' wait)
#ifndef MIO_LOOP_D
#define MIO_LOOP_D 4
#endif
// MIO_LOOP_DQ8: the same for the Q8_0 walk (k_mmq16_loop), 3 (the 2.6B gate|up's <= 3 tiles per
// workgroup; 4 Q8_0 W | U sets exceed 256 VGPRs)
#ifndef MIO_LOOP_DQ8
#define MIO_LOOP_DQ8 3
#endif
// MIO_MMQ_ACT1 (A/B builds; default 1): the K-quant tiles issue their weights, then their
// activation codes, then the scales' staging (one activation round trip instead of two)
#ifndef MIO_MMQ_ACT1
#define MIO_MMQ_ACT1 1
#endif
// QNP > 0 (k_mmq16q): the first a.nt workgroups are quantization producers (MmqQuant, XRegs
// of QNP passes, QM = its mode), the tiles follow and wait before their activation reads.
template <int T0, int T1, int T2, int MODE, int KP = 0, int QNP = 0, int QM = 0>
__global__ __launch_bounds__(MMQ_NT) void k_mmq16(MmqSeg s0, MmqSeg s1, MmqSeg s2, MmqArgs a, MmqQuant q) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int NV = MODE == MMQ_SWIGLU ? 2 : 1;
    constexpr bool QF = QNP > 0;
    // plain rows (QM 1, the down's h) are quantized by one producer per (token, 2048-element
    // chunk) (chunk_quant_producer); RMSNorm rows by one per token
    // (q.mode 2 = plain rows one producer per token: MIO_BT_QCHUNK=0, A/B)
    static_assert(QM != 1 || MMQ_NT == 512, "chunk_quant_producer covers 2048 elements with 512 threads");
    const bool chunked = QM == 1 && q.mode == 1;
    const int nq = !QF ? 0 : (chunked ? a.nt * ((a.K + 2047) / 2048) : a.nt);
    if constexpr (QF) {
        if ((int)blockIdx.x < nq) {
            if (chunked)
                chunk_quant_producer(q.src, a.K, T0 != 8, (a.K + 2047) / 2048, const_cast<char *>(a.act), q.cnt,
                                     q.other, lds);
            else
                mmq_quant_producer<T0 == 8 ? 0 : 1, QNP, QM>(a, q, lds);
            return;
        }
    }
    float *red = reinterpret_cast<float *>(lds);  // [NV][8 waves][64][4]
    float *da = red + NV * MMQ_NT * 4;           // [groups][16 tokens]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t0 = blockIdx.y * TT16;
    int tile_id = (int)blockIdx.x - nq;
    // the producers' records are complete: one lane waits, the barrier releases the others; every
    // record load after it is an sc1 load (ActSc1, stage_act16<T, QF>)
    auto wait_act = [&]() {
        if constexpr (QF) {
            if (threadIdx.x == 0) wait_count(q.cnt + 64 * (blockIdx.x & 7), nq, q.flag);
            asm volatile("s_barrier" ::: "memory");
        }
    };
    auto run = [&]<int T>(const MmqSeg &sg, int ti) {
        const int row0 = ti * RT16, row = min(row0 + (lane & 15), sg.w.rows - 1);
        // MMQ_RESID: the residual values wave 0's epilogue adds, loaded before anything else
        // (the launch before this one wrote them; read at the end they were a dependent
        // round trip behind the reduction)
        float xres[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE == MMQ_RESID && MIO_MMQ_XPRE) {
            if (wave == 0 && row0 + (lane & 15) < sg.w.rows) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int t = t0 + tok16(lane, i);
                    if (t < a.nt) xres[i] = a.out[(size_t)t * a.ld + sg.out_off + row0 + (lane & 15)];
                }
            }
        }
        // the slot index must be wave-uniform (divergent branches around the MFMAs would run
        // them with a partial EXEC)
        const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        if (T == 8 && (KP != 0 || a.K % 256 == 0)) {
            const auto aq = act16_codes<QF>(a, t0);
            v4f y = {}, u = {};
            if (KP == 1 || (KP == 0 && a.K <= 2048)) {
                // one pass: every weight / activation / scale load goes out before the
                // activation scales' staging barrier
                const int nb = a.K >> 5;
                Q80Pass qw, qu;
                v4i x[4];
                q80p_load(sg.w, row, 0, k, qw);
                if constexpr (NV == 2) q80p_load(a.w_up, row, 0, k, qu);
                wait_act();
                act_load(aq, a.K, 0, k, x);
                stage_act16<8, QF>(a, t0, a.K, da);
#pragma unroll
                for (int i = 0; i < 4; ++i) swap_halves(x[i]);
                v4f aw[8], au[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) aw[i] = v4f{}, au[i] = v4f{};
                q80p_acc(qw, x, 0, k, nb, da, aw);
                y = tree8(aw);
                if constexpr (NV == 2) {
                    q80p_acc(qu, x, 0, k, nb, da, au);
                    u = tree8(au);
                }
            } else {
                wait_act();
                stage_act16<8, QF>(a, t0, a.K, da);
                slot16_q80p<NV>(sg.w, a.w_up, row, k, aq, da, y, u);
            }
            slot16_store(y, red);
            if constexpr (NV == 2) slot16_store(u, red + MMQ_NT * 4);
        } else {
            if constexpr (NV == 1 && (T == 12 || T == 14) && (QF || MIO_MMQ_ACT1)) {
                // up to three passes' weights (K <= 6144, the 1.7B down) are in flight before
                // the activations are read (with in-launch quantization: while the producers
                // quantize); then slot16_kq's arithmetic. MIO_MMQ_ACT1: the activation codes of
                // every pass are issued before the scales' staging, so codes and scales arrive
                // in one round trip (and the launches without producers, the O, take this path
                // too)
                // register sets for NPX passes: 3 for the plain-row down (K <= 6144), one
                // elsewhere (K <= 2048: the q|k|v launch must stay at <= 128 VGPRs, two
                // workgroups per CU, for its 256 tiles + producers); longer K: the generic path
                constexpr int NPX = QF && QM == 1 ? 3 : 1;
                const int nsb = sg.w.k >> 8, np = (nsb + 7) / 8;
                if ((!QF || q.early) && np <= NPX) {
                    KqPass<T> ps[NPX];
#pragma unroll
                    for (int p = 0; p < NPX; ++p)
                        if (p < np) kqp_load<T>(sg.w, row, min(p * 8 + k, nsb - 1), ps[p]);
                    wait_act();
#if MIO_MMQ_ACT1
                    const auto aq = act16_codes<QF>(a, t0);
                    v4i xs[NPX][4];
#pragma unroll
                    for (int p = 0; p < NPX; ++p)
                        if (p < np) kq_act_ld(aq, min(p * 8 + k, nsb - 1), xs[p]);
                    stage_act16<T, QF>(a, t0, a.K, da);
#else
                    const auto aq = stage_act16<T, QF>(a, t0, a.K, da);
#endif
                    v4f acc = {};
#pragma unroll
                    for (int p = 0; p < NPX; ++p) {
                        if (p < np) {
                            const int s = p * 8 + k;
#if MIO_MMQ_ACT1
                            v4i(&x)[4] = xs[p];
#pragma unroll
                            for (int c = 0; c < 4; ++c) swap_halves(x[c]);
#else
                            v4i x[4];
                            kq_act(aq, min(s, nsb - 1), x);
#endif
                            v4f v = {};
                            if (s < nsb) v = kqp_val<T>(ps[p], x, s, da);
                            acc = acc + v;  // the decode lane's pass accumulation (0 + v0 + v1 ...)
                        }
                    }
                    slot16_store(acc, red);
                    goto reduce;
                }
            }
            wait_act();
            const auto aq = stage_act16<T, QF>(a, t0, a.K, da);
            slot16_store(slot16_val<T>(sg.w, row, k, aq, da), red);
            if constexpr (NV == 2) slot16_store(slot16_val<T>(a.w_up, row, k, aq, da), red + MMQ_NT * 4);
        }
    reduce:
        __syncthreads();
        if (wave != 0) return;
        const v4f y = slot16_sum(red);
        v4f u = {};
        if constexpr (NV == 2) u = slot16_sum(red + MMQ_NT * 4);
        const int orow = row0 + (lane & 15);
        if (orow >= sg.w.rows) return;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = t0 + tok16(lane, i);
            if (t >= a.nt) continue;
            float *o = a.out + (size_t)t * a.ld + sg.out_off + orow;
            if constexpr (MODE == MMQ_STORE) *o = y[i];
            else if constexpr (MODE == MMQ_RESID) *o = y[i] + (MIO_MMQ_XPRE ? xres[i] : *o);
            else *o = silu_f(y[i]) * u[i];
        }
    };
    const int n0 = (s0.w.rows + RT16 - 1) / RT16;
    if (tile_id < n0) return run.template operator()<T0>(s0, tile_id);
    tile_id -= n0;
    if constexpr (T1 >= 0) {
        const int n1 = (s1.w.rows + RT16 - 1) / RT16;
        if (tile_id < n1) return run.template operator()<T1>(s1, tile_id);
        tile_id -= n1;
    }
    if constexpr (T2 >= 0) {
        if (tile_id < (s2.w.rows + RT16 - 1) / RT16) return run.template operator()<T2>(s2, tile_id);
    }
}


// Q8_0 one-pass pairs (K % 256 == 0, K <= 2048), one matrix (W, or W | U for SwiGLU): each
// workgroup walks tiles blockIdx, + G, + 2G ... with the next tile's weights in flight while it
// reduces the current one (ping-pong register sets, no copies), and loads the activations and
// their scales ONCE. With 672 tiles (the 2.6B gate|up) the plain grid runs 1.3 rounds of two
// workgroups per CU; here one workgroup per CU streams its 2-3 tiles back to back. Per tile the
// arithmetic is k_mmq16's (q80p_acc, tree8, slot16_sum, the same epilogue): bit-identical.
// QNP > 0: the first a.nt workgroups are the in-launch quantization producers.
template <int MODE, int QNP, int QM>
__global__ __launch_bounds__(MMQ_NT) void k_mmq16_loop(MmqSeg s0, MmqArgs a, MmqQuant q, int n_tiles) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int NV = MODE == MMQ_SWIGLU ? 2 : 1;
    constexpr bool QF = QNP > 0;
    const int nq = QF ? a.nt : 0;
    if constexpr (QF) {
        if ((int)blockIdx.x < nq) {
            mmq_quant_producer<0, QNP, QM>(a, q, lds);
            return;
        }
    }
    float *red = reinterpret_cast<float *>(lds);  // [NV][8 waves][64][4]
    float *da = red + NV * MMQ_NT * 4;           // [groups][16 tokens]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = (int)gridDim.x - nq;
    int tile = (int)blockIdx.x - nq;
    if (tile >= n_tiles) return;
    const int nb = a.K >> 5;
    auto row_of = [&](int ti) { return min(ti * RT16 + (lane & 15), s0.w.rows - 1); };
    // ring of D tiles' weights: D - 1 tiles in flight while one is reduced
    constexpr int D = MIO_LOOP_DQ8;
    Q80Pass w[D], u[D];
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        const int ti = tile + d * G;
        if (ti < n_tiles) {
            q80p_load(s0.w, row_of(ti), 0, k, w[d]);
            if constexpr (NV == 2) q80p_load(a.w_up, row_of(ti), 0, k, u[d]);
        }
    }
    if constexpr (QF) {  // the records' loads below are sc1 (ActSc1)
        if (threadIdx.x == 0) wait_count(q.cnt + 64 * (blockIdx.x & 7), a.nt, q.flag);
        asm volatile("s_barrier" ::: "memory");
    }
    const auto aq = act16_codes<QF>(a, 0);
    v4i x[4];
    act_load(aq, a.K, 0, k, x);
    stage_act16<8, QF>(a, 0, a.K, da);
#pragma unroll
    for (int i = 0; i < 4; ++i) swap_halves(x[i]);
    // one tile: the loads of the tile D - 1 ahead go out first, into the set the previous
    // tile freed
    auto step = [&](Q80Pass &cw, Q80Pass &cu, Q80Pass &nw, Q80Pass &nu) -> bool {
        const int ahead = tile + (D - 1) * G;
        if (ahead < n_tiles) {
            q80p_load(s0.w, row_of(ahead), 0, k, nw);
            if constexpr (NV == 2) q80p_load(a.w_up, row_of(ahead), 0, k, nu);
        }
        v4f acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = v4f{};
        q80p_acc(cw, x, 0, k, nb, da, acc);
        slot16_store(tree8(acc), red);
        if constexpr (NV == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = v4f{};
            q80p_acc(cu, x, 0, k, nb, da, acc);
            slot16_store(tree8(acc), red + MMQ_NT * 4);
        }
        __syncthreads();
        if (wave == 0) {
            const v4f y = slot16_sum(red);
            v4f u = {};
            if constexpr (NV == 2) u = slot16_sum(red + MMQ_NT * 4);
            const int orow = tile * RT16 + (lane & 15);
            if (orow < s0.w.rows) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int t = tok16(lane, i);
                    if (t >= a.nt) continue;
                    float *o = a.out + (size_t)t * a.ld + s0.out_off + orow;
                    if constexpr (MODE == MMQ_STORE) *o = y[i];
                    else if constexpr (MODE == MMQ_RESID) *o = y[i] + *o;
                    else *o = silu_f(y[i]) * u[i];
                }
            }
        }
        __syncthreads();  // red is rewritten by the next tile
        if (tile + G >= n_tiles) return false;
        tile += G;
        return true;
    };
    for (;;) {
#pragma unroll
        for (int d = 0; d < D; ++d)
            if (!step(w[d], u[d], w[(d + D - 1) % D], u[(d + D - 1) % D])) return;
    }
}

// K-quants (T 12 = Q4_K, 14 = Q6_K), K <= 2048 (one superblock per wave): k_mmq16_loop's walk
// (the batched lm_head: 10296 16-row Q6_K tiles; the 1.7B gate|up: 384 Q4_K tile pairs). The
// activation codes (this wave's superblock k of every tile) and their scales are loaded once
// per workgroup, the next tile's weights (q4p_load / q6p_load) are in flight while the current
// one is reduced. Per tile the arithmetic is k_mmq16's slot16_kq (the 0 + v pass sum,
// slot16_sum, the same epilogue): bit-identical. QNP > 0: the first a.nt workgroups are the
// in-launch quantization producers (as k_mmq16_loop).
// IQ (QNP 0, RMSNorm rows, nt <= 8, K <= 2048): no producer workgroups; every walking
// workgroup RMSNorm-quantizes the nt token rows itself, one wave per token (xpre_issue before
// its weight loads, xpre_quant into LDS records: k_bt_quant's bits), and reads the records from
// LDS; workgroup 0 zeroes the other counter set as a producer would.
template <int T, int MODE, int QNP, int QM, bool IQ = false>
__global__ __launch_bounds__(MMQ_NT) void k_mmq16_loop_kq(MmqSeg s0, MmqArgs a, MmqQuant q, int n_tiles) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int NV = MODE == MMQ_SWIGLU ? 2 : 1;
    constexpr bool QF = QNP > 0;
    const int nq = QF ? a.nt : 0;
    if constexpr (QF) {
        if ((int)blockIdx.x < nq) {
            mmq_quant_producer<1, QNP, QM>(a, q, lds);
            return;
        }
    }
    float *red = reinterpret_cast<float *>(lds);  // [NV][8 waves][64][4]
    float *da = red + NV * MMQ_NT * 4;           // [superblocks][16 tokens]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int G = (int)gridDim.x - nq;
    int tile = (int)blockIdx.x - nq;
    if (tile >= n_tiles) return;
    const bool live = k < (a.K >> 8);  // wave-uniform: this wave's superblock exists
    const int sb = live ? k : 0;
    auto row_of = [&](int ti) { return min(ti * RT16 + (lane & 15), s0.w.rows - 1); };
    static_assert(!IQ || (QNP == 0 && NV == 2), "in-prologue quantization: the gate|up walk");
    char *rec = reinterpret_cast<char *>(da + (a.K >> 8) * TT16);  // IQ: the nt records
    XPre xp;
    if constexpr (IQ) {
        if (blockIdx.x == 0 && threadIdx.x < 8)
            __hip_atomic_store((__attribute__((address_space(1))) int *)(q.other + 64 * threadIdx.x), 0,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        xpre_issue(q.src, q.norm_w, a.K, a.nt, xp);
    }
    // ring of D tiles' weights: D - 1 tiles in flight while one is reduced
    constexpr int D = MIO_LOOP_D;
    KqPass<T> w[D], u[D];
#pragma unroll
    for (int d = 0; d < D - 1; ++d) {
        const int ti = tile + d * G;
        if (ti < n_tiles) {
            kqp_load<T>(s0.w, row_of(ti), sb, w[d]);
            if constexpr (NV == 2) kqp_load<T>(a.w_up, row_of(ti), sb, u[d]);
        }
    }
    if constexpr (QF) {  // the records' loads below are sc1 (ActSc1)
        if (threadIdx.x == 0) wait_count(q.cnt + 64 * (blockIdx.x & 7), a.nt, q.flag);
        asm volatile("s_barrier" ::: "memory");
    }
    MmqArgs al = a;
    if constexpr (IQ) {
        xpre_quant(xp, a.K, q.eps, true, rec, a.nt);
        al.act = rec, al.act_stride = act_bytes(a.K);
    }
    v4i x[4];
#if MIO_MMQ_ACT1
    // codes issued ahead of the scales' staging: one round trip for both
    kq_act_ld(act16_codes<QF>(al, 0), sb, x);
    stage_act16<T, QF>(al, 0, a.K, da);
#pragma unroll
    for (int c = 0; c < 4; ++c) swap_halves(x[c]);
#else
    const auto aq = stage_act16<T, QF>(al, 0, a.K, da);
    kq_act(aq, sb, x);
#endif
    auto step = [&](KqPass<T> &cw, KqPass<T> &cu, KqPass<T> &nw, KqPass<T> &nu) -> bool {
        const int ahead = tile + (D - 1) * G;
        if (ahead < n_tiles) {
            kqp_load<T>(s0.w, row_of(ahead), sb, nw);
            if constexpr (NV == 2) kqp_load<T>(a.w_up, row_of(ahead), sb, nu);
        }
        {
            v4f acc = {}, v = {};
            if (live) v = kqp_val<T>(cw, x, sb, da);
            acc = acc + v;
            slot16_store(acc, red);
        }
        if constexpr (NV == 2) {
            v4f acc = {}, v = {};
            if (live) v = kqp_val<T>(cu, x, sb, da);
            acc = acc + v;
            slot16_store(acc, red + MMQ_NT * 4);
        }
        __syncthreads();
        if (wave == 0) {
            const v4f y = slot16_sum(red);
            v4f u = {};
            if constexpr (NV == 2) u = slot16_sum(red + MMQ_NT * 4);
            const int orow = tile * RT16 + (lane & 15);
            if (orow < s0.w.rows) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int t = tok16(lane, i);
                    if (t >= a.nt) continue;
                    float *o = a.out + (size_t)t * a.ld + s0.out_off + orow;
                    if constexpr (MODE == MMQ_STORE) *o = y[i];
                    else if constexpr (MODE == MMQ_RESID) *o = y[i] + *o;
                    else *o = silu_f(y[i]) * u[i];
                }
            }
        }
        __syncthreads();  // red is rewritten by the next tile
        if (tile + G >= n_tiles) return false;
        tile += G;
        return true;
    };
    for (;;) {
#pragma unroll
        for (int d = 0; d < D; ++d)
            if (!step(w[d], u[d], w[(d + D - 1) % D], u[(d + D - 1) % D])) return;
    }
}
}  // namespace

size_t mmq_lds(int type, int K, int mode) {
    return (size_t)(mode == MMQ_SWIGLU ? 2 : 1) * MMQ_NT * 16 * sizeof(float) +
           (size_t)(type == 8 ? K / 32 : K / 256) * TT * sizeof(float);
}

// dynamic LDS above 64 KB (Q8_0 activation scales of a long K) needs the per-kernel opt-in,
// once per (device, kernel)
static void allow_lds_mmq(const void *kern) {
    static std::mutex mu;
    static std::vector<std::pair<int, const void *>> done;
    int dev = 0;
    hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    for (const auto &q : done)
        if (q.first == dev && q.second == kern) return;
    hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
    done.push_back({dev, kern});
}

int mmq_tiles(int rows) { return (rows + RT - 1) / RT; }

// types: {T0, T1, T2} (-1 = segment unused); mode MMQ_*.
// 16 x 16 tiles (k_mmq16) for launches of at most 16 tokens; MIO_MMQ16=0: 32 x 32 tiles always
// CUs of the current device (the tile-loop grids: one workgroup per CU), cached
static int n_cu() {
    static const int n = [] {
        int dev = 0, v = 0;
        hipGetDevice(&dev);
        return hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
    }();
    return n;
}
// MIO_MMQ_LOOP (default 1): Q8_0 one-pass launches with more 16-row tiles than CUs walk their
// tiles in k_mmq16_loop (one workgroup per CU) instead of one workgroup per tile
static bool mmq_loop_on() {
    static const bool on = !(getenv("MIO_MMQ_LOOP") && getenv("MIO_MMQ_LOOP")[0] == '0');
    return on;
}

// MIO_MMQ_LOOP_KQ (bits, default 3): K-quant (Q4_K / Q6_K, K <= 2048) matmuls of more 16-row
// tiles than CUs walk their tiles in k_mmq16_loop_kq: bit 0 without in-launch quantization
// (the batched lm_head), bit 1 with it (the batched gate|up)
static int kq_loop_mask() {
    static const int m = getenv("MIO_MMQ_LOOP_KQ") ? atoi(getenv("MIO_MMQ_LOOP_KQ")) : 3;
    return m;
}

bool mmq16_on(int nt) {
    static const bool on = !(getenv("MIO_MMQ16") && getenv("MIO_MMQ16")[0] == '0');
    return on && nt <= TT16;
}

void launch_mmq(const MmqSeg *seg, const int *types, int nseg, int mode, const MmqArgs &a, hipStream_t s) {
    MmqSeg sg[3] = {seg[0], nseg > 1 ? seg[1] : MmqSeg{}, nseg > 2 ? seg[2] : MmqSeg{}};
    const bool t16 = mmq16_on(a.nt);
    int tiles = 0;
    for (int i = 0; i < nseg; ++i) tiles += t16 ? (sg[i].w.rows + RT16 - 1) / RT16 : sg[i].tiles;
    const dim3 grid(tiles, t16 ? 1 : (a.nt + TT - 1) / TT);
    size_t lds = 0;
    for (int i = 0; i < nseg; ++i)
        lds = std::max(lds, t16 ? (size_t)(mode == MMQ_SWIGLU ? 2 : 1) * MMQ_NT * 4 * sizeof(float) +
                                      (size_t)(types[i] == 8 ? a.K / 32 : a.K / 256) * TT16 * sizeof(float)
                                : mmq_lds(types[i], a.K, mode));
    auto go = [&]<int A, int B, int C>() {
        auto launch = [&](auto kern) {
            if (lds > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
            hipLaunchKernelGGL(kern, grid, dim3(MMQ_NT), lds, s, sg[0], sg[1], sg[2], a, MmqQuant{});
        };
        if (t16) {
            const bool q8 = A == 8 && (B < 0 || B == 8) && (C < 0 || C == 8) && a.K % 256 == 0;
            const int kp = q8 ? (a.K <= 2048 ? 1 : 2) : 0;
            if constexpr ((A == 12 || A == 14) && B < 0) {
                if (a.K % 256 == 0 && a.K <= 2048 && tiles > n_cu() && mmq_loop_on() && (kq_loop_mask() & 1)) {
                    auto kl = [&](auto kern) {
                        if (lds > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
                        hipLaunchKernelGGL(kern, dim3(n_cu()), dim3(MMQ_NT), lds, s, sg[0], a, MmqQuant{}, tiles);
                    };
                    if (mode == MMQ_STORE) kl(k_mmq16_loop_kq<A, MMQ_STORE, 0, 0>);
                    else if (mode == MMQ_RESID) kl(k_mmq16_loop_kq<A, MMQ_RESID, 0, 0>);
                    else kl(k_mmq16_loop_kq<A, MMQ_SWIGLU, 0, 0>);
                    return;
                }
            }
            if constexpr (A == 8 && B < 0) {
                if (kp == 1 && tiles > n_cu() && mmq_loop_on()) {
                    auto kl = [&](auto kern) {
                        if (lds > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
                        hipLaunchKernelGGL(kern, dim3(n_cu()), dim3(MMQ_NT), lds, s, sg[0], a, MmqQuant{}, tiles);
                    };
                    if (mode == MMQ_STORE) kl(k_mmq16_loop<MMQ_STORE, 0, 0>);
                    else if (mode == MMQ_RESID) kl(k_mmq16_loop<MMQ_RESID, 0, 0>);
                    else kl(k_mmq16_loop<MMQ_SWIGLU, 0, 0>);
                    return;
                }
            }
            auto kpl = [&]<int M>() {
                if (kp == 1) launch(k_mmq16<A, B, C, M, 1>);
                else if (kp == 2) launch(k_mmq16<A, B, C, M, 2>);
                else launch(k_mmq16<A, B, C, M, 0>);
            };
            if (mode == MMQ_STORE)
                kpl.template operator()<MMQ_STORE>();
            else if (mode == MMQ_RESID)
                kpl.template operator()<MMQ_RESID>();
            else
                kpl.template operator()<MMQ_SWIGLU>();
            return;
        }
        if (mode == MMQ_STORE)
            launch(k_mmq<A, B, C, MMQ_STORE>);
        else if (mode == MMQ_RESID)
            launch(k_mmq<A, B, C, MMQ_RESID>);
        else
            launch(k_mmq<A, B, C, MMQ_SWIGLU>);
    };
    auto one = [&]<int A>() {
        if (nseg == 1) return go.template operator()<A, -1, -1>();
        // attention input: q, k share a type; v is Q4_K / Q6_K (Q4_K_M) or Q8_0
        if (types[2] == 14) return go.template operator()<A, A, 14>();
        if (types[2] == 12) return go.template operator()<A, A, 12>();
        return go.template operator()<A, A, 8>();
    };
    if (types[0] == 12) one.template operator()<12>();
    else if (types[0] == 14) one.template operator()<14>();
    else one.template operator()<8>();
}


// The fused shapes of the batched decode (launch_layers): q|k|v of the K-quant models (three
// segments, RMSNorm input), gate|up (Q4_K, or Q8_0 one-pass pairs; RMSNorm input) and the
// K-quant down matmul (plain h rows of 3 passes). Anything else: false.
bool launch_mmq_q(const MmqSeg *seg, const int *types, int nseg, int mode, const MmqArgs &a, const MmqQuant &q,
                  hipStream_t s) {
    if (!mmq16_on(a.nt)) return false;
    MmqSeg sg[3] = {seg[0], nseg > 1 ? seg[1] : MmqSeg{}, nseg > 2 ? seg[2] : MmqSeg{}};
    int tiles = 0;
    size_t lds = 0;
    for (int i = 0; i < nseg; ++i) {
        tiles += (sg[i].w.rows + RT16 - 1) / RT16;
        lds = std::max(lds, (size_t)(mode == MMQ_SWIGLU ? 2 : 1) * MMQ_NT * 4 * sizeof(float) +
                                (size_t)(types[i] == 8 ? a.K / 32 : a.K / 256) * TT16 * sizeof(float));
    }
    lds = std::max(lds, act_bytes(a.K) + smem_bytes(a.K));  // the producers' record + scratch
    // k_mmq16's producer count: per (token, 2048-element chunk) for plain rows (q.mode 1)
    static const bool qchunk = !(getenv("MIO_BT_QCHUNK") && getenv("MIO_BT_QCHUNK")[0] == '0');
    MmqQuant qq = q;
    if (q.mode == 1 && !qchunk) qq.mode = 2;
    // MIO_KQ_EARLY=0: K-quant tiles issue their weight loads after the producers' wait (A/B)
    static const bool early = !(getenv("MIO_KQ_EARLY") && getenv("MIO_KQ_EARLY")[0] == '0');
    qq.early = early ? 1 : 0;
    const int nq = qq.mode == 1 ? a.nt * ((a.K + 2047) / 2048) : a.nt;
    const dim3 grid(nq + tiles);
    auto go = [&](auto kern) {
        if (lds > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
        hipLaunchKernelGGL(kern, grid, dim3(MMQ_NT), lds, s, sg[0], sg[1], sg[2], a, qq);
        return true;
    };
    const int np = pick_np(a.K);
    if (mode == MMQ_STORE && nseg == 3 && q.mode == 0 && np == 1 && types[0] == 12 && types[1] == 12) {
        if (types[2] == 12) return go(k_mmq16<12, 12, 12, MMQ_STORE, 0, 1, 0>);
        if (types[2] == 14) return go(k_mmq16<12, 12, 14, MMQ_STORE, 0, 1, 0>);
    }
    // Q8_0 q|k|v (one pass, K <= 2048) when MIO_BT_FQ=0 takes it off the dot4 in-launch path
    if (mode == MMQ_STORE && nseg == 3 && q.mode == 0 && np == 1 && types[0] == 8 && types[1] == 8 && types[2] == 8 &&
        a.K % 256 == 0 && a.K <= 2048)
        return go(k_mmq16<8, 8, 8, MMQ_STORE, 1, 1, 0>);
    if (mode == MMQ_SWIGLU && nseg == 1 && q.mode == 0 && np == 1) {
        if (types[0] == 12) {
            // MIO_BT_IQ=1 (opt-in): the walk quantizes its <= 8 tokens in its own prologue instead
            // of behind producer workgroups. Bit-exact, but 8 streams 1.7B 1.366 vs 1.252 ms per
            // step (profiles/r06/bt_iq_ab.txt): one wave per token quantizing 8 superblocks in a
            // row is a longer chain than the producers' hop
            static const bool iq = getenv("MIO_BT_IQ") && getenv("MIO_BT_IQ")[0] == '1';
            if (iq && a.nt <= 8 && a.K % 256 == 0 && a.K <= 2048 && tiles > n_cu() && mmq_loop_on() &&
                (kq_loop_mask() & 2)) {
                auto kern = k_mmq16_loop_kq<12, MMQ_SWIGLU, 0, 0, true>;
                const size_t l = (size_t)2 * MMQ_NT * 4 * sizeof(float) + (size_t)(a.K / 256) * TT16 * sizeof(float) +
                                 (size_t)a.nt * act_bytes(a.K);
                if (l > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
                hipLaunchKernelGGL(kern, dim3(n_cu()), dim3(MMQ_NT), l, s, sg[0], a, q, tiles);
                return true;
            }
            const int nl = n_cu() - a.nt;  // the producers keep CUs of their own
            if (a.K % 256 == 0 && a.K <= 2048 && tiles > nl && nl > 0 && mmq_loop_on() && (kq_loop_mask() & 2)) {
                auto kern = k_mmq16_loop_kq<12, MMQ_SWIGLU, 1, 0>;
                if (lds > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
                hipLaunchKernelGGL(kern, dim3(a.nt + nl), dim3(MMQ_NT), lds, s, sg[0], a, q, tiles);
                return true;
            }
            return go(k_mmq16<12, -1, -1, MMQ_SWIGLU, 0, 1, 0>);
        }
        if (types[0] == 8 && a.K % 256 == 0 && a.K <= 2048) {
            const int nl = n_cu() - a.nt;  // the producers keep CUs of their own
            if (tiles > nl && nl > 0 && mmq_loop_on()) {
                auto kern = k_mmq16_loop<MMQ_SWIGLU, 1, 0>;
                if (lds > 64 * 1024) allow_lds_mmq(reinterpret_cast<const void *>(kern));
                hipLaunchKernelGGL(kern, dim3(a.nt + nl), dim3(MMQ_NT), lds, s, sg[0], a, q, tiles);
                return true;
            }
            return go(k_mmq16<8, -1, -1, MMQ_SWIGLU, 1, 1, 0>);
        }
    }
    if (mode == MMQ_RESID && nseg == 1 && q.mode == 1 && np == 3) {
        if (types[0] == 12) return go(k_mmq16<12, -1, -1, MMQ_RESID, 0, 3, 1>);
        if (types[0] == 14) return go(k_mmq16<14, -1, -1, MMQ_RESID, 0, 3, 1>);
    }
    // Q8_0 down (multi-pass pair path) when MIO_MMQ_MASK puts it on the matrix cores
    if (mode == MMQ_RESID && nseg == 1 && q.mode == 1 && types[0] == 8 && a.K % 256 == 0 && a.K > 2048) {
        if (np == 3) return go(k_mmq16<8, -1, -1, MMQ_RESID, 2, 3, 1>);
        if (np == 6) return go(k_mmq16<8, -1, -1, MMQ_RESID, 2, 6, 1>);
    }
    return false;
}

}  // namespace mio
