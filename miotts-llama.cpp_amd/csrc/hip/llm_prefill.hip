// Batched prompt prefill for gfx950 (replaces the prefill llama_decode of
// test-to-speech.cpp:132-148: every prompt token through every layer, K/V cache rows
// written, logits needed only for the last token, which the decode step then produces).
//
// The decode step streams all weights once per token; the prompt (tens of tokens) would pay
// that once per prompt token. Here a chunk of up to kPrefillB tokens shares ONE weight pass
// per launch: the streaming-rows engine (llm_device.h) loads each weight fragment once and
// dots it with every token's re-quantized activation slice, which lives in LDS. Per layer:
//   k_pf_attn_in   RMSNorm + quantize nt tokens -> q|k|v for all of them
//   k_pf_rope      q/k RMSNorm (qwen3) + RoPE + f16 rounding; k/v rows -> F16 KV cache
//   k_pf_attention per (128-position chunk, kv head, token): causal online softmax over
//                  positions <= the token's own, chunk partial records
//   k_pf_attn_out  per-token chunk merge + quantize -> O matvec -> x += .
//   k_pf_ffn_in    RMSNorm + quantize -> gate|up -> silu(g)*u
//   k_pf_ffn_down  quantize -> down -> x += .
// lfm2 short-conv layers: in_proj on the matrix cores, k_bt_conv (gated conv per token, the
// window from earlier tokens of the chunk or the sequence's ring), k_bt_conv_state (ring),
// out_proj.
// Arithmetic is the decode step's, token by token, in the same order (same quantizers,
// same per-superblock integer sums, the same pass order per row, the same online-softmax
// order): the K/V cache and the last token's logits equal a token-by-token decode bit for
// bit (tests/test_llm_gpu.py::test_batched_prefill_matches_sequential).
#include "llm_device.h"
#include "llm_mmq.h"
#include "llm_quant_producer.h"

#include <mutex>
#include <utility>
#include <vector>

#pragma clang fp contract(off)

namespace mio {
namespace {

constexpr int LDS_MAX = 160 * 1024;

// ------------------------------------------------------------------ LDS layout
// act[t] = {qs i8[K] | d f32[K/32+8] | bs i16[K/16+8]} x nt | resid f32[MW][nt * rpw] (the
// wave's residual rows per token). The prologues quantize straight from registers (one wave
// per token), so no f32 staging row is needed. (act_bytes / carve_t: llm_device.h)
// K of the act record layout for a weight type: BF16 weights take the activation as K bf16
// values (ggml's vec_dot_bf16 operand, 2 bytes each), stored in the qs area of a record laid out
// for 2K (the d / bs areas then go unused)
__host__ __device__ constexpr int rec_k(int K, int type) { return type == 30 ? 2 * K : K; }
__host__ __device__ inline size_t pf_lds_bytes(int K, int nt, int rpw) {
    return act_base(K) + act_bytes(K) * nt + (size_t)MW * nt * rpw * 4;
}

__device__ inline float *resid_lds(char *base, int K, int nt, int rpw) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return (float *)(base + act_base(K) + act_bytes(K) * nt) + (size_t)w * nt * rpw;
}

// ------------------------------------------------------------------ batched streaming rows
// A register group holds RU whole rows (all NM matrices, all NP passes): every fragment is
// loaded once and dotted with each token's activation; row totals per token as in the
// decode engine (acc over passes in order, then row_total).
// MIO_BT_UNITS / MIO_BT_UNITS_Q8 (compile-time, A/B builds): weight units per row group for
// K-quant / Q8_0 matrices. Smaller groups turn over faster (the next group's loads go out
// sooner); 8-stream steps (graph, profiles/r04_bt_units_ab.txt): 2.6B Q8_0 2.36 / 2.23 / 2.20
// ms at 4 / 2 / 1 units, 1.7B Q4_K_M 1.84 / 1.77 / 1.81 ms
#ifndef MIO_BT_UNITS
#define MIO_BT_UNITS 2
#endif
#ifndef MIO_BT_UNITS_Q8
#define MIO_BT_UNITS_Q8 1
#endif
// NG register groups in flight per wave: two (one loading while the other is dotted), or one
// for NP = 6 (a 6-pass row is 13 KB per wave; 8 waves x one row already keep 100 KB per CU in
// flight, and the registers go to the activation records, act_issue)
// BF16 units are 64 B per lane (4 registers of 8 weights): one unit per group, or the
// batched kernels spill
template <int T, int NP, int NM>
struct CfgB {
    static constexpr int UN = T == 8 ? MIO_BT_UNITS_Q8 : (T == 30 ? 1 : MIO_BT_UNITS);
    static constexpr int RU = NP * NM >= UN ? 1 : UN / (NP * NM);
    static constexpr int U = RU * NP * NM;
    static constexpr int NG = (NP >= 6 || T == 30) ? 1 : 2;
};

template <int T, int NP, int NM>
__device__ __forceinline__ void load_rows(const QMat W0, const QMat W1, int r, int hi, Frag (&F)[CfgB<T, NP, NM>::U],
                                          int split) {
#pragma unroll
    for (int ri = 0; ri < CfgB<T, NP, NM>::RU; ++ri) {
        const int row = __builtin_amdgcn_readfirstlane(min(r + ri, hi - 1));  // wave-uniform
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                Frag &f = F[(ri * NM + m) * NP + p];
                if constexpr (NM == 1)
                    f = load_frag<T>(row >= split ? W1 : W0, row >= split ? row - split : row, p);
                else
                    f = load_frag<T>(m ? W1 : W0, row, p);
            }
    }
}

template <int T, int NP, int NM>
__device__ __forceinline__ void load_first_b(const QMat W0, const QMat W1, int lo, int hi,
                                             Frag (&A)[CfgB<T, NP, NM>::U], Frag (&B)[CfgB<T, NP, NM>::U],
                                             int split = INT_MAX) {
    if (hi <= lo) return;
    load_rows<T, NP, NM>(W0, W1, lo, hi, A, split);
    if constexpr (CfgB<T, NP, NM>::NG == 2) load_rows<T, NP, NM>(W0, W1, lo + CfgB<T, NP, NM>::RU, hi, B, split);
}

// ------------------------------------------------------------------ transposed row totals
// The decode's row_total is a balanced tree over the wave's lanes by lane bit 0, 1, ..., 5
// (sum8_f's row_shr 1/2/4 prefix, then row_shr 8 and row_bcast 15/31; K-quants: bits 3..5 over
// the superblock lanes 8k+7, their integer sums being exact). A multi-token group has N such
// totals (token x row x matrix) per lane; reducing each on its own costs N full trees plus N
// wave-uniform epilogues. Here the N trees run together as a reduce-scatter: at lane bit b the
// lanes with the bit clear keep the lower half of their values and add the partner's copy of
// it, the others the upper half, so every level halves the values per lane. Every value still
// sums the same two subtrees at every level (float addition is commutative), so each total is
// bitwise the decode's; at the end each lane holds its own totals and the epilogue runs once
// per (row, token) on the lane that owns it instead of once per value on the whole wave.
constexpr int ROW_SHL4 = 0x104, ROW_SHL8 = 0x108;
// v(l) + v(l ^ 2^B) (every lane)
template <int B>
__device__ __forceinline__ float xpair_sum(float v) {
    const int lane = threadIdx.x & 63;
    if constexpr (B == 0) return v + dpp_f<0xB1>(v);
    else if constexpr (B == 1) return v + dpp_f<0x4E>(v);
    else if constexpr (B == 2 || B == 3) {
        const float up = dpp_f<B == 2 ? ROW_SHL4 : ROW_SHL8>(v);  // lane l + 2^B
        const float dn = dpp_f<B == 2 ? ROW_SHR4 : ROW_SHR8>(v);  // lane l - 2^B
        return v + (((lane >> B) & 1) ? dn : up);
    } else {
        return v + xor_lane<(1 << B)>(v);
    }
}
// one scatter level at lane bit B: lanes with the bit clear return a(l) + a(l ^ 2^B), the
// others b(l) + b(l ^ 2^B)
template <int B>
__device__ __forceinline__ float xpair_scatter(float a, float b) {
    const int lane = threadIdx.x & 63;
    if constexpr (B == 4 || B == 5) {
        // the permlane swap exchanges a's upper lanes with b's lower ones: afterwards each lane
        // holds its own kept value in one register and the partner's copy in the other
        const auto r = B == 4 ? __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false)
                              : __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else if constexpr (B == 0 || B == 1) {
        const float sa = a + dpp_f<B == 0 ? 0xB1 : 0x4E>(a), sb = b + dpp_f<B == 0 ? 0xB1 : 0x4E>(b);
        return ((lane >> B) & 1) ? sb : sa;
    } else {
        const float sa = a + dpp_f<B == 2 ? ROW_SHL4 : ROW_SHL8>(a);
        const float sb = b + dpp_f<B == 2 ? ROW_SHR4 : ROW_SHR8>(b);
        return ((lane >> B) & 1) ? sb : sa;
    }
}
// Levels B..5 over the first N entries of v: scatter while more than R values remain, then
// all-reduce; returns nothing, v[0 .. max(R, N >> (6 - B))) hold the lane's totals.
template <int B, int N, int R, int NV>
__device__ __forceinline__ void xreduce(float (&v)[NV]) {
    if constexpr (B < 6) {
        if constexpr (N > R) {
            constexpr int H = N / 2;
#pragma unroll
            for (int i = 0; i < H; ++i) v[i] = xpair_scatter<B>(v[i], v[i + H]);
            xreduce<B + 1, H, R>(v);
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) v[i] = xpair_sum<B>(v[i]);
            xreduce<B + 1, N, R>(v);
        }
    }
}
// tokens per reduce-scatter group (the dot loop still goes TT tokens at a time)
template <int NP>
struct XRedCfg {
    static constexpr int TT = NP == 1 ? 4 : (NP == 3 ? 2 : 1);
    static constexpr int TB = NP == 1 ? 8 : (NP == 3 ? 4 : 8);
};
// MIO_BT_MINB (compile-time A/B): workgroups per CU the one-pass batched matvecs (attn_out,
// ffn_in) are register-budgeted for; with MIO_BT_WGM=2 at run time their grids double
#ifndef MIO_BT_MINB
#define MIO_BT_MINB 1
#endif
#ifndef MIO_BT_XRED
#define MIO_BT_XRED 1
#endif

// epi(row, t, dot0, dot1): once per (row, token); with MIO_BT_XRED on the lane that holds
// the totals (lane-varying values), else wave-uniform values on every lane
template <int T, int NP, int NM, class Epi>
__device__ __forceinline__ void stream_rows_bx(const QMat W0, const QMat W1, int lo, int hi,
                                               Frag (&A)[CfgB<T, NP, NM>::U], Frag (&B)[CfgB<T, NP, NM>::U], char *smem,
                                               int nt, Epi &&epi, int split = INT_MAX) {
    constexpr int RU = CfgB<T, NP, NM>::RU, U = CfgB<T, NP, NM>::U;
    constexpr int TT = XRedCfg<NP>::TT, TB = XRedCfg<NP>::TB;
    constexpr int N = TB * RU * NM;             // totals per group: index ((t * RU + ri) * NM + m)
    constexpr int LB = (T == 8 || T == 30) ? 0 : 3;  // first tree level (K-quants: lanes 8k+7)
    constexpr int NF = N >> (6 - LB) > NM ? N >> (6 - LB) : NM;  // totals per lane at the end
    constexpr int SL = __builtin_ctz(N / NF);   // scatter levels
    const int K = W0.k, KR = rec_k(K, T);
    const int lane = threadIdx.x & 63;
    if (hi <= lo) return;
    // the lane's first total after the scatter (level k at lane bit LB + k halves the index
    // range), and whether it is the replica that runs the epilogue
    int jb = 0;
#pragma unroll
    for (int k = 0; k < SL; ++k) jb += ((lane >> (LB + k)) & 1) * (N >> (k + 1));
    const bool owner = (LB == 0 || (lane & 7) == 7) && (lane >> (LB + SL)) == 0;
    auto consume = [&](const Frag (&F)[U], int r) {
        const int nr = min(RU, hi - r);
        for (int tb = 0; tb < nt; tb += TB) {
            float acc[N];
#pragma unroll
            for (int i = 0; i < N; ++i) acc[i] = 0.0f;
#pragma unroll
            for (int t0 = 0; t0 < TB; t0 += TT) {
                if (tb + t0 < nt) {
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        ALane al[TT];
#pragma unroll
                        for (int j = 0; j < TT; ++j)
                            al[j] = load_alane<T>(carve_t(smem, KR, min(tb + t0 + j, nt - 1)).a, K, p);
#pragma unroll
                        for (int ri = 0; ri < RU; ++ri) {
                            if (ri < nr) {
#pragma unroll
                                for (int m = 0; m < NM; ++m)
#pragma unroll
                                    for (int j = 0; j < TT; ++j)
                                        acc[((t0 + j) * RU + ri) * NM + m] += dot_frag<T>(F[(ri * NM + m) * NP + p], al[j], K, p);
                            }
                        }
                    }
                }
            }
            xreduce<LB, N, NF>(acc);
            if (owner) {
#pragma unroll
                for (int i = 0; i < NF / NM; ++i) {
                    const int q = jb / NM + i, t = tb + q / RU, ri = q % RU;
                    if (t < nt && ri < nr) epi(r + ri, t, acc[i * NM], acc[i * NM + NM - 1]);
                }
            }
        }
    };
    if constexpr (CfgB<T, NP, NM>::NG == 1) {
        for (int r = lo;;) {
            consume(A, r);
            r += RU;
            if (r >= hi) break;
            load_rows<T, NP, NM>(W0, W1, r, hi, A, split);
        }
        return;
    }
    for (int r = lo;;) {
        consume(A, r);
        r += RU;
        if (r >= hi) break;
        load_rows<T, NP, NM>(W0, W1, r + RU, hi, A, split);
        consume(B, r);
        r += RU;
        if (r >= hi) break;
        load_rows<T, NP, NM>(W0, W1, r + RU, hi, B, split);
    }
}

// epi(row, t, dot0, dot1): wave-uniform values, once per (row, token)
template <int T, int NP, int NM, class Epi>
__device__ __forceinline__ void stream_rows_bu(const QMat W0, const QMat W1, int lo, int hi,
                                               Frag (&A)[CfgB<T, NP, NM>::U], Frag (&B)[CfgB<T, NP, NM>::U], char *smem,
                                               int nt, Epi &&epi, int split = INT_MAX) {
    constexpr int RU = CfgB<T, NP, NM>::RU, U = CfgB<T, NP, NM>::U;
    const int K = W0.k, KR = rec_k(K, T);
    if (hi <= lo) return;
    // TT tokens per iteration: their activation loads are in flight together and their dot
    // / reduction chains interleave (the weight decode is shared); rows of the group past hi
    // (a wave owning fewer rows than RU) are not dotted
    // (BF16: one token at a time, its activation slice alone is 16 registers)
    constexpr int TT = T == 30 ? 1 : (NP == 1 ? 4 : (NP == 3 ? 2 : 1));
    auto consume = [&](const Frag (&F)[U], int r) {
        const int nr = min(RU, hi - r);
        for (int t0 = 0; t0 < nt; t0 += TT) {
            float acc[TT][RU * NM];
#pragma unroll
            for (int j = 0; j < TT; ++j)
#pragma unroll
                for (int i = 0; i < RU * NM; ++i) acc[j][i] = 0.0f;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                ALane al[TT];
#pragma unroll
                for (int j = 0; j < TT; ++j) al[j] = load_alane<T>(carve_t(smem, KR, min(t0 + j, nt - 1)).a, K, p);
#pragma unroll
                for (int ri = 0; ri < RU; ++ri) {
                    if (ri < nr) {
#pragma unroll
                        for (int m = 0; m < NM; ++m)
#pragma unroll
                            for (int j = 0; j < TT; ++j)
                                acc[j][ri * NM + m] += dot_frag<T>(F[(ri * NM + m) * NP + p], al[j], K, p);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < TT; ++j) {
                if (t0 + j < nt) {
#pragma unroll
                    for (int ri = 0; ri < RU; ++ri) {
                        if (ri < nr) {
                            const float v0 = row_total<T>(acc[j][ri * NM]);
                            const float v1 = NM == 2 ? row_total<T>(acc[j][ri * NM + NM - 1]) : 0.0f;
                            if ((threadIdx.x & 63) == 0) epi(r + ri, t0 + j, v0, v1);
                        }
                    }
                }
            }
        }
    };
    if constexpr (CfgB<T, NP, NM>::NG == 1) {
        for (int r = lo;;) {
            consume(A, r);
            r += RU;
            if (r >= hi) break;
            load_rows<T, NP, NM>(W0, W1, r, hi, A, split);
        }
        return;
    }
    for (int r = lo;;) {
        consume(A, r);
        r += RU;
        if (r >= hi) break;
        load_rows<T, NP, NM>(W0, W1, r + RU, hi, A, split);
        consume(B, r);
        r += RU;
        if (r >= hi) break;
        load_rows<T, NP, NM>(W0, W1, r + RU, hi, B, split);
    }
}

// The multi-token streaming rows: transposed totals (MIO_BT_XRED, default) or one wave-wide
// tree per total (A/B build). Either way epi runs once per (row, token) on one lane.
template <int T, int NP, int NM, class Epi>
__device__ __forceinline__ void stream_rows_b(const QMat W0, const QMat W1, int lo, int hi,
                                              Frag (&A)[CfgB<T, NP, NM>::U], Frag (&B)[CfgB<T, NP, NM>::U], char *smem,
                                              int nt, Epi &&epi, int split = INT_MAX) {
    // BF16: the per-total trees (its 64-B units and 16-register activation slices leave no
    // room for the transposed reduction's token groups)
    if constexpr (MIO_BT_XRED && T != 30)
        stream_rows_bx<T, NP, NM>(W0, W1, lo, hi, A, B, smem, nt, epi, split);
    else
        stream_rows_bu<T, NP, NM>(W0, W1, lo, hi, A, B, smem, nt, epi, split);
}

// ------------------------------------------------------------------ multi-token prologues
// Every matvec workgroup needs every token's quantized activation. It is produced ONCE per
// launch by k_bt_quant (one workgroup per token, running the single-token decode prologue
// itself: rmsnorm_quant / plain_quant, so the values are the decode's bit
// for bit) into pb.act, and each matvec workgroup copies the records into LDS with all its
// loads in flight (one memory latency for all tokens).
__device__ __forceinline__ void prologue_copy(const char *act, int K, char *smem, int nt) {
    constexpr int UN = 8;
    const int n16 = (int)(act_bytes(K) * nt / 16);
    const uint4 *src = reinterpret_cast<const uint4 *>(act);
    uint4 *dst = reinterpret_cast<uint4 *>(smem + act_base(K));
    for (int i0 = threadIdx.x; i0 < n16; i0 += UN * MT) {
        uint4 v[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) v[u] = src[min(i0 + u * MT, n16 - 1)];  // clamped: all in flight
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            const int i = i0 + u * MT;
            if (i < n16) dst[i] = v[u];
        }
    }
    lds_barrier();
}

// The records' loads issued AHEAD of the launch's weight loads: vmcnt retires in order, so a
// copy issued after the first weight groups (prologue_copy) waits for all of them before its
// LDS stores and barrier - the launch then streams weights, THEN copies, THEN dots. Issued
// first, the copy (L2 / Infinity Cache resident) lands while the weights are still in flight.
// CP uint4 per thread cover nt tokens when act_bytes(K) * nt <= CP * MT * 16; a larger batch
// copies the rest after (act_store_rest).
template <int NP>
struct ActPre {
    static constexpr int CP = NP == 1 ? 6 : (NP == 3 ? 10 : 14);
    uint4 v[CP];
};
// 16-B granule i of the records; SC: written by producer workgroups of this launch, so read
// with an sc1 load (llm_mmq.hip ActSc1 explains the hand-off)
template <bool SC>
__device__ __forceinline__ uint4 act_granule(const char *act, int i) {
    if constexpr (SC) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(act, 0x7FFFFFF0u), (uint32_t)i * 16u, 0, 16);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return reinterpret_cast<const uint4 *>(act)[i];
    }
}
template <int NP, bool SC = false>
__device__ __forceinline__ void act_issue(const char *act, int K, int nt, ActPre<NP> &ap) {
    const int n16 = (int)(act_bytes(K) * nt / 16);
#pragma unroll
    for (int u = 0; u < ActPre<NP>::CP; ++u) ap.v[u] = act_granule<SC>(act, min((int)threadIdx.x + u * MT, n16 - 1));
}
template <int NP, bool SC = false>
__device__ __forceinline__ void act_store(const ActPre<NP> &ap, const char *act, int K, char *smem, int nt) {
    const int n16 = (int)(act_bytes(K) * nt / 16);
    uint4 *dst = reinterpret_cast<uint4 *>(smem + act_base(K));
#pragma unroll
    for (int u = 0; u < ActPre<NP>::CP; ++u) {
        const int i = (int)threadIdx.x + u * MT;
        if (i < n16) dst[i] = ap.v[u];
    }
    for (int i = (int)threadIdx.x + ActPre<NP>::CP * MT; i < n16; i += MT) dst[i] = act_granule<SC>(act, i);
    lds_barrier();
}

// XPre / xpre_issue / xpre_quant (the in-launch RMSNorm + quantization of up to 8 tokens by
// one wave each): llm_quant_producer.h

// One workgroup per token t: MODE 0 RMSNorm(src[t]) * norm_w, 1 src[t] as is (the attention
// output pb.att, h); quantized (Q8_K / Q8_0) into the token's act record.
// ak = akind of the consuming weights (0 Q8_0, 1 Q8_K, 2 BF16: the record then holds K bf16
// values and is laid out for rec_k = 2K)
template <int NP, int MODE>
__global__ __launch_bounds__(MT) void k_bt_quant(LlmDims d, const float *src, int K, const float *norm_w, int ak,
                                                 PrefillBuffers pb) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = blockIdx.x;
    // the quantizers store straight into the token's global record (its layout is the LDS
    // record's: qs | d | bs), no LDS staging + barrier + copy; LDS keeps the reduction scratch
    Smem s = carve(smem, K);
    s.a = carve_t(pb.act, ak == 2 ? 2 * K : K, t).a;
    XRegs<NP> xr;
    load_x(src + (size_t)t * K, MODE == 0 ? norm_w : nullptr, K, xr);
    if constexpr (MODE == 0)
        rmsnorm_quant(xr, K, d.eps, ak, s);
    else
        plain_quant(xr, K, ak, s);
}

// MODE 1 (plain rows, K % 256 == 0) split over 2048-element chunks: grid (nt, chunks). Q8_K
// superblocks / Q8_0 blocks are quantized independently of each other, so each chunk
// workgroup's records are k_bt_quant's bits (quant_regs: thread tid of chunk c holds elements
// c * 2048 + 4 tid .. + 3, i.e. wave w holds superblock 8 c + w / blocks 64 c + 8 w ..).
__global__ __launch_bounds__(MT) void k_bt_quant_split(const float *src, int K, int kq, PrefillBuffers pb) {
    const int t = blockIdx.x, c = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (c * 2048 + wave * 256 >= K) return;  // wave-uniform
    const ActL a = carve_t(pb.act, K, t).a;
    const float4 x = *reinterpret_cast<const float4 *>(src + (size_t)t * K + c * 2048 + 4 * (int)threadIdx.x);
    const float v[4] = {x.x, x.y, x.z, x.w};
    if (kq)
        q8k_store(v, abs_max4(v), c * 8 + wave, a);
    else
        q80_store(v, c * 64 + wave * 8 + (lane >> 3), true, a);
}

// lfm2 short-conv layer, one workgroup per token t: the gated conv of t (conv_load /
// conv_quant, the decode step's prologue) quantized into t's act record. Window inputs of
// positions pos - 1, pos - 2: the bcx rows of the tokens before t in this launch when they are
// that sequence's previous positions, else the sequence's ring (written by an earlier chunk or
// decode step), zeros before the sequence start. ring = layer il's ring of sequence 0.
template <int NP>
__global__ __launch_bounds__(MT) void k_bt_conv(LlmDims d, const float *conv_w, const float *ring, int kq,
                                                PrefillBuffers pb) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = blockIdx.x, K = d.n_embd;
    const size_t CW = (size_t)3 * K;
    // quantized straight into the token's global record (k_bt_quant's way); LDS keeps the
    // reduction scratch
    Smem s = carve(smem, K);
    s.a = carve_t(pb.act, K, t).a;
    const int pos = pb.pos[t * pb.pos_stride], sq = pb.seq[t * pb.seq_stride];
    const float *rs = ring + (size_t)sq * pb.seq_ring;
    ConvPrev pv[2];
#pragma unroll
    for (int k = 1; k <= 2; ++k) {
        const int p = pos - k;
        if (p < 0)
            pv[k - 1] = ConvPrev{nullptr, 0};
        else if (t >= k && pb.seq[(t - k) * pb.seq_stride] == sq && pb.pos[(t - k) * pb.pos_stride] == p)
            pv[k - 1] = ConvPrev{pb.qkv + (t - k) * CW, 1};
        else
            pv[k - 1] = ConvPrev{rs + (size_t)(p & (kConvSlots - 1)) * K, 0};
    }
    ConvRegs<NP> cr;
    conv_load(pb.qkv + t * CW, pv[0], pv[1], conv_w, K, cr);
    conv_quant(cr, K, kq != 0, s, nullptr);
}

// After k_bt_conv: the bx rows of each sequence's last two positions in this launch go to
// its ring (a later chunk or decode step reads them). Sequences occupy consecutive tokens
// with consecutive positions, so token t is among them unless t + 2 continues its run.
__global__ __launch_bounds__(ST) void k_bt_conv_state(LlmDims d, float *ring, PrefillBuffers pb, int nt) {
    const int t = blockIdx.x, K = d.n_embd;
    const int pos = pb.pos[t * pb.pos_stride], sq = pb.seq[t * pb.seq_stride];
    if (t + 2 < nt && pb.seq[(t + 2) * pb.seq_stride] == sq && pb.pos[(t + 2) * pb.pos_stride] == pos + 2) return;
    const float *row = pb.qkv + (size_t)t * 3 * K;
    float *dst = ring + (size_t)sq * pb.seq_ring + (size_t)(pos & (kConvSlots - 1)) * K;
    for (int e = threadIdx.x; e < K; e += ST) dst[e] = row[e] * row[2 * K + e];
}

// Residual rows [lo, hi) of every token (row stride E) in two registers per lane: entry
// i = t * rpw + r at lane i % 64, register i / 64 (nt * rpw <= 128, host-checked).
struct Resid {
    float v0, v1;
};
__device__ inline Resid load_resid_b(const float *x, int E, int lo, int hi, int nt, int rpw) {
    const int lane = threadIdx.x & 63;
    Resid r;
    float *o[2] = {&r.v0, &r.v1};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = lane + 64 * k, t = i / rpw, rr = i - t * rpw;
        *o[k] = (t < nt && lo + rr < hi) ? x[(size_t)t * E + lo + rr] : 0.0f;
    }
    return r;
}
__device__ inline void store_resid_b(const Resid &r, float *lds, int nt, int rpw) {
    const int lane = threadIdx.x & 63;
    if (lane < nt * rpw) lds[lane] = r.v0;
    if (lane + 64 < nt * rpw) lds[lane + 64] = r.v1;
}

// ------------------------------------------------------------------ kernels
template <int NP, int TQ, int TV, int FQ = 0>
__global__ __launch_bounds__(MT) void k_pf_attn_in(LlmDims d, const float *norm_w, QMat wq, QMat wk, QMat wv,
                                                   int g_qk, PrefillBuffers pb, int nt) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd, QD = (d.n_head + 2 * d.n_kv) * d.hd, KR = rec_k(K, TQ);
    const int lane = threadIdx.x & 63;
    const int o1 = wq.rows, o2 = wq.rows + wk.rows;
    Frag ga[CfgB<TQ, NP, 1>::U], gb[CfgB<TQ, NP, 1>::U];
    XPre xp;
    if constexpr (FQ == 2) xpre_issue(pb.x, norm_w, K, nt, xp);
    auto prologue = [&]() {
        if constexpr (FQ == 2)
            xpre_quant(xp, K, d.eps, TQ != 8, smem, nt);
        else
            prologue_copy(pb.act, KR, smem, nt);
    };
    int lo, hi;
    if ((int)blockIdx.x < g_qk) {
        wave_range(o2, lo, hi, blockIdx.x, g_qk);
        load_first_b<TQ, NP, 1>(wq, wk, lo, hi, ga, gb, o1);
        prologue();
        stream_rows_b<TQ, NP, 1>(wq, wk, lo, hi, ga, gb, smem, nt, [&](int row, int t, float v, float) {
            pb.qkv[(size_t)t * QD + row] = v;
        }, o1);
    } else {
        wave_range(wv.rows, lo, hi, blockIdx.x - g_qk, gridDim.x - g_qk);
        load_first_b<TV, NP, 1>(wv, wv, lo, hi, ga, gb);
        prologue();
        stream_rows_b<TV, NP, 1>(wv, wv, lo, hi, ga, gb, smem, nt, [&](int row, int t, float v, float) {
            pb.qkv[(size_t)t * QD + o2 + row] = v;
        });
    }
}

// One wave per (head, token): q heads are normalized / rotated / f16-rounded in place, k
// heads likewise and written with the v row to the F16 cache at the token's position
// (prep_head: the decode step's head preparation).
template <int HD>
__global__ __launch_bounds__(64) void k_pf_rope(LlmDims d, const float *q_norm, const float *k_norm,
                                                const float *bqkv, _Float16 *kc, _Float16 *vc, PrefillBuffers pb) {
    constexpr int PER = HD / 64;
    __shared__ float row[HD];
    const int hh = blockIdx.x, t = blockIdx.y, lane = threadIdx.x;
    const int pos = pb.pos[t * pb.pos_stride];
    const size_t kvo = (size_t)pb.seq[t * pb.seq_stride] * pb.seq_kv;
    const int QD = (d.n_head + 2 * d.n_kv) * HD;
    const bool isk = hh >= d.n_head;
    const int kvh = hh - d.n_head;
    float *src = pb.qkv + (size_t)t * QD + (size_t)hh * HD;
    float vv[PER];
    if (isk) {
        const size_t vo = (size_t)(d.n_head + d.n_kv + kvh) * HD;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            vv[i] = pb.qkv[(size_t)t * QD + vo + lane + 64 * i];
            if (bqkv) vv[i] = vv[i] + bqkv[vo + lane + 64 * i];
        }
    }
    prep_head<HD>(src, bqkv ? bqkv + (size_t)hh * HD : nullptr, isk ? k_norm : q_norm,
                  pb.rope + (size_t)pos * (HD / 2), d, row);
    if (!isk) {
#pragma unroll
        for (int i = 0; i < PER; ++i) src[lane + 64 * i] = row[lane + 64 * i];
    } else {
        _Float16 *kd = kc + kvo + ((size_t)kvh * d.n_ctx + pos) * HD;
        _Float16 *vd = vc + kvo + ((size_t)kvh * d.n_ctx + pos) * HD;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int p = lane + 64 * i;
            kd[p] = (_Float16)row[p];
            vd[p] = (_Float16)f16r(vv[i]);
        }
    }
}

// attend_chunk(_mfma) + attn_merge_last of token t's (kv head, chunk): records in pb.part
// [t][H][max_splits][REC], tickets pb.att_cnt[t][Hkv], outputs pb.att[t][H * hd].
// att_q >= 0: the merger also writes token t's O-matvec activation record (attn_merge_last).
template <int HD, int G>
__device__ __forceinline__ void merge_token(const LlmDims &d, int pos, int t, int kvh, const PrefillBuffers &pb,
                                            int att_q, float *part, uint32_t head0, uint32_t gs) {
    const int KO = d.n_head * HD;
    attn_merge_last<HD, G>(part, head0, gs, pos / ATT_CHUNK + 1, pb.att_cnt + (size_t)t * d.n_kv + kvh,
                           pb.att + (size_t)t * KO + (size_t)kvh * G * HD, att_q, carve_t(pb.act, KO, t).a,
                           att_q == 1 ? kvh * G * HD / 256 : kvh * G * HD / 32);
}
#if MIO_ATT_MFMA
template <int HD, int G>
__device__ __forceinline__ void attend_and_merge(const LlmDims &d, const _Float16 (*qh)[HD], const char *img, int t0,
                                                 int pos, int ch, int t, int kvh, const PrefillBuffers &pb, int att_q) {
    using C = AttCfg<HD>;
    const uint32_t gs = (uint32_t)(d.max_splits * C::REC);
    float *part = pb.part + (size_t)t * d.n_head * gs;  // token t's records (wave-uniform)
    const uint32_t head0 = (uint32_t)(kvh * G) * gs;
    attend_chunk_mfma<HD, G>(qh, img, img + AttM<HD>::IMG, t0, pos, d.scale, part + head0 + (uint32_t)ch * C::REC, gs);
    merge_token<HD, G>(d, pos, t, kvh, pb, att_q, part, head0, gs);
}
#else
template <int HD, int G>
__device__ __forceinline__ void attend_and_merge(const LlmDims &d, const float (*qs)[HD],
                                                 const h8 (&kr)[AttCfg<HD>::IT], const h8 (&vr)[AttCfg<HD>::IT],
                                                 int t0, int pos, int ch, int t, int kvh,
                                                 float (*wres)[G][HD + 2], const PrefillBuffers &pb, int att_q) {
    using C = AttCfg<HD>;
    const uint32_t gs = (uint32_t)(d.max_splits * C::REC);
    float *part = pb.part + (size_t)t * d.n_head * gs;  // token t's records (wave-uniform)
    const uint32_t head0 = (uint32_t)(kvh * G) * gs;
    attend_chunk<HD, G>(qs, kr, vr, t0, pos, d.scale, wres, part + head0 + (uint32_t)ch * C::REC, gs);
    merge_token<HD, G>(d, pos, t, kvh, pb, att_q, part, head0, gs);
}
#endif

// One workgroup per (ATT_CHUNK-position chunk, kv head, token): causal softmax over the
// chunk's positions <= the token's position in the token's own sequence, all rows read from
// the cache (this launch's own rows were written by k_pf_rope); the attention and
// attn_merge_last are the decode step's, so pb.att holds the decode's outputs bit for bit.
// Chunks past the token's position exit at once. Grid (n_kv * nt, chunks): consecutive
// workgroup ids are different (kv head, token) pairs of one chunk, so the workgroups with
// work (the low chunks) spread over all XCDs instead of one.
template <int HD, int G>
__global__ __launch_bounds__(AttCfg<HD>::NT) void k_pf_attention(LlmDims d, const _Float16 *kc, const _Float16 *vc,
                                                                 PrefillBuffers pb, int att_q) {
    using C = AttCfg<HD>;
    __shared__ float qs[G][HD];
    const int kvh = blockIdx.x % d.n_kv, t = blockIdx.x / d.n_kv, ch = blockIdx.y;
    const int pos = pb.pos[t * pb.pos_stride];
    const int t0 = ch * ATT_CHUNK;
    if (t0 > pos) return;
    const size_t kvo = (size_t)pb.seq[t * pb.seq_stride] * pb.seq_kv + (size_t)kvh * d.n_ctx * HD;
    const int QD = (d.n_head + 2 * d.n_kv) * HD;
    const float *qsrc = pb.qkv + (size_t)t * QD + (size_t)kvh * G * HD;
#if MIO_ATT_MFMA
    using A = AttM<HD>;
    __shared__ __attribute__((aligned(16))) char img[2 * A::IMG];
    __shared__ __attribute__((aligned(16))) _Float16 qh[G][HD];
    h8 kr[A::VI], vr[A::VI];
    kv_issue<HD>(kc + kvo, vc + kvo, t0, pos, kr, vr);
    for (int e = threadIdx.x; e < G * HD; e += C::NT) qh[e / HD][e % HD] = (_Float16)qsrc[e];
    kv_stage<HD>(kr, vr, -1, img, img + A::IMG);
    lds_barrier();
    attend_and_merge<HD, G>(d, qh, img, t0, pos, ch, t, kvh, pb, att_q);
#else
    __shared__ float wres[C::NW][G][HD + 2];
    h8 kr[C::IT], vr[C::IT];
    load_kv_rows<HD>(kc + kvo, vc + kvo, t0, pos, kr, vr);
    for (int e = threadIdx.x; e < G * HD; e += C::NT) qs[e / HD][e % HD] = qsrc[e];
    lds_barrier();
    attend_and_merge<HD, G>(d, qs, kr, vr, t0, pos, ch, t, kvh, wres, pb, att_q);
#endif
}

// Batched decode attention (one token per sequence, so no token of the launch reads a row
// another one writes): per (kv head, token, chunk) the decode step's k_attention — the
// token's q heads (and, in the chunk owning its position, its k / v row) get q/k RMSNorm +
// bias + RoPE + f16 rounding in LDS, the owner appends the row to the sequence's cache and
// stages it from LDS, then the chunk's softmax partials. Replaces k_pf_rope + k_pf_attention
// (one launch less per layer; the same prep_head / attention / attn_merge_last arithmetic,
// so the outputs equal theirs bit for bit).
template <int HD, int G>
__global__ __launch_bounds__(AttCfg<HD>::NT) void k_bt_attention(LlmDims d, const float *q_norm, const float *k_norm,
                                                         const float *bqkv, _Float16 *kcache, _Float16 *vcache,
                                                         PrefillBuffers pb, int att_q) {
    using C = AttCfg<HD>;
    constexpr int PER = HD / 64;
    __shared__ float qs[G][HD];
    __shared__ float knew[HD], vnew[HD];
#if MIO_ATT_MFMA
    using A = AttM<HD>;
    __shared__ __attribute__((aligned(16))) char img[2 * A::IMG];
    __shared__ __attribute__((aligned(16))) _Float16 qh[G][HD];
#else
    __shared__ float wres[C::NW][G][HD + 2];
#endif
    const int kvh = blockIdx.x % d.n_kv, t = blockIdx.x / d.n_kv, ch = blockIdx.y;
    const int pos = pb.pos[t * pb.pos_stride];
    const int t0 = ch * ATT_CHUNK;
    // a stream that sampled its end token is frozen (k_bt_sample): its attention is skipped
    // (in the batched decode pb.pos points at StepState.pos of each stream)
    static_assert(offsetof(StepState, done) - offsetof(StepState, pos) == 3 * sizeof(int), "StepState layout");
    if (t0 > pos || pb.pos[t * pb.pos_stride + 3]) return;
    const size_t kvo = (size_t)pb.seq[t * pb.seq_stride] * pb.seq_kv + (size_t)kvh * d.n_ctx * HD;
    _Float16 *kc = kcache + kvo, *vc = vcache + kvo;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float2 *rope = pb.rope + (size_t)pos * (HD / 2);
    const float *qkv = pb.qkv + (size_t)t * (d.n_head + 2 * d.n_kv) * HD;
    const bool owner = pos < t0 + ATT_CHUNK;
    // the loads of each wave's first head go out before its K/V rows (as k_attention)
    auto head_src = [&](int hh, HeadIn<HD> &in) {
        const bool isk = hh == G;
        const size_t so = isk ? (size_t)(d.n_head + kvh) * HD : (size_t)(kvh * G + hh) * HD;
        const size_t vo = (size_t)(d.n_head + d.n_kv + kvh) * HD;
        head_load<HD>(qkv + so, bqkv ? bqkv + so : nullptr, isk ? k_norm : q_norm, rope, d, in,
                      isk ? qkv + vo : nullptr, isk && bqkv ? bqkv + vo : nullptr);
    };
    HeadIn<HD> hin;
    if (wave < G + (owner ? 1 : 0)) head_src(wave, hin);
#if MIO_ATT_MFMA
    h8 kr[A::VI], vr[A::VI];
    kv_issue<HD>(kc, vc, t0, pos, kr, vr);  // row pos is staged from LDS below
#else
    h8 kr[C::IT], vr[C::IT];
    load_kv_rows<HD>(kc, vc, t0, pos, kr, vr);  // row pos comes from LDS below
#endif
    for (int hh = wave; hh < G + (owner ? 1 : 0); hh += C::NW) {
        const bool isk = hh == G;
        if (hh != wave) head_src(hh, hin);
        head_prep<HD>(hin, d, isk ? knew : qs[hh]);
        if (isk) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int p = lane + 64 * i;
                const float vr16 = f16r(hin.vv[i]);
                vnew[p] = vr16;
                kc[(size_t)pos * HD + p] = (_Float16)knew[p];
                vc[(size_t)pos * HD + p] = (_Float16)vr16;
            }
#if MIO_ATT_MFMA
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            kv_stage_row<HD>(knew, vnew, pos - t0, img, img + A::IMG);
#endif
        }
#if MIO_ATT_MFMA
        else {
            q_to_f16<HD>(qs[hh], qh[hh]);
        }
#endif
    }
#if MIO_ATT_MFMA
    kv_stage<HD>(kr, vr, owner ? pos - t0 : -1, img, img + A::IMG);
    lds_barrier();
    attend_and_merge<HD, G>(d, qh, img, t0, pos, ch, t, kvh, pb, att_q);
#else
    lds_barrier();
    if (owner) {
        const int sl = threadIdx.x / C::LP, lp = lane % C::LP, r = pos - t0;
        if (sl == r % C::NS) {
            h8 kn, vn;
#pragma unroll
            for (int i = 0; i < 8; ++i) kn[i] = (_Float16)knew[lp * 8 + i], vn[i] = (_Float16)vnew[lp * 8 + i];
#pragma unroll
            for (int it = 0; it < C::IT; ++it)
                if (it == r / C::NS) kr[it] = kn, vr[it] = vn;
        }
    }
    attend_and_merge<HD, G>(d, qs, kr, vr, t0, pos, ch, t, kvh, wres, pb, att_q);
#endif
}

template <int NP, int T>
__global__ __launch_bounds__(MT, MIO_BT_MINB) void k_pf_attn_out(LlmDims d, QMat wo, PrefillBuffers pb, int nt, int rpw) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = wo.k, E = d.n_embd, KR = rec_k(K, T);
    int lo, hi;
    wave_range(d, wo.rows, lo, hi);
    const Resid xr = load_resid_b(pb.x, E, lo, hi, nt, rpw);
    ActPre<NP> ap;
    act_issue<NP>(pb.act, KR, nt, ap);
    Frag ga[CfgB<T, NP, 1>::U], gb[CfgB<T, NP, 1>::U];
    load_first_b<T, NP, 1>(wo, wo, lo, hi, ga, gb);
    float *res = resid_lds(smem, KR, nt, rpw);
    store_resid_b(xr, res, nt, rpw);
    act_store<NP>(ap, pb.act, KR, smem, nt);
    stream_rows_b<T, NP, 1>(wo, wo, lo, hi, ga, gb, smem, nt, [&](int row, int t, float v, float) {
        const float r = res[t * rpw + row - lo];
        pb.x[(size_t)t * E + row] = v + r;
    });
}

// FQ = 2: RMSNorm + quantization in the launch from inputs loaded ahead of the weights (xpre)
template <int NP, int T, int FQ = 0>
__global__ __launch_bounds__(MT, MIO_BT_MINB) void k_pf_ffn_in(LlmDims d, const float *norm_w, QMat gate, QMat up,
                                                  PrefillBuffers pb, int nt) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd, KR = rec_k(K, T);
    int lo, hi;
    wave_range(d, gate.rows, lo, hi);
    ActPre<NP> ap;
    XPre xp;
    if constexpr (FQ == 2)
        xpre_issue(pb.x, norm_w, K, nt, xp);
    else
        act_issue<NP>(pb.act, KR, nt, ap);
    Frag ga[CfgB<T, NP, 2>::U], gb[CfgB<T, NP, 2>::U];
    load_first_b<T, NP, 2>(gate, up, lo, hi, ga, gb);
    if constexpr (FQ == 2)
        xpre_quant(xp, K, d.eps, T != 8, smem, nt);
    else
        act_store<NP>(ap, pb.act, KR, smem, nt);
    stream_rows_b<T, NP, 2>(gate, up, lo, hi, ga, gb, smem, nt, [&](int row, int t, float g, float u) {
        pb.h[(size_t)t * d.n_ff + row] = silu_f(g) * u;
    });
}

template <int NP, int T>
__global__ __launch_bounds__(MT) void k_pf_ffn_down(LlmDims d, QMat down, PrefillBuffers pb, int nt, int rpw) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = down.k, E = d.n_embd, KR = rec_k(K, T);
    int lo, hi;
    wave_range(d, down.rows, lo, hi);
    const Resid rr = load_resid_b(pb.x, E, lo, hi, nt, rpw);
    ActPre<NP> ap;
    act_issue<NP>(pb.act, KR, nt, ap);
    Frag ga[CfgB<T, NP, 1>::U], gb[CfgB<T, NP, 1>::U];
    load_first_b<T, NP, 1>(down, down, lo, hi, ga, gb);
    float *res = resid_lds(smem, KR, nt, rpw);
    store_resid_b(rr, res, nt, rpw);
    act_store<NP>(ap, pb.act, KR, smem, nt);
    stream_rows_b<T, NP, 1>(down, down, lo, hi, ga, gb, smem, nt, [&](int row, int t, float v, float) {
        const float r = res[t * rpw + row - lo];
        pb.x[(size_t)t * E + row] = v + r;
    });
}

// The batched decode's down on the dot4 engine with the h quantization in the launch (no
// k_bt_quant_split launch in front; MIO_BT_QF). Workgroups [0, npr) are producers, one per
// (token t, 2048-element chunk c) as k_bt_quant_split's grid: the chunk is quantized into an
// LDS image of t's record with k_bt_quant_split's arithmetic (the same bits), its code, scale
// and (Q8_K) bsum ranges are copied out with 16-B write-through stores, drained, and each
// producer adds 1 to the 8 counter shards (workgroup 0 first zeroes the other set, the next
// fused launch's). The matvec workgroups follow: residual and first weight group issued, one
// lane waits for npr on its shard, then the records are copied to LDS with sc1 loads (the
// replica-counter hand-off of llm_mmq.hip ActSc1: no plain load of a record this launch wrote).
// Deadlock-free by dispatch order (producers first, they never wait).
template <int NP, int T>
__global__ __launch_bounds__(MT) void k_pf_ffn_down_q(LlmDims d, QMat down, PrefillBuffers pb, int nt, int rpw,
                                                      MmqQuant q, int nch) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = down.k, E = d.n_embd, KR = rec_k(K, T), npr = nt * nch;
    if ((int)blockIdx.x < npr) {
        chunk_quant_producer(q.src, K, T != 8, nch, pb.act, q.cnt, q.other, smem);
        return;
    }
    int lo, hi;
    wave_range(down.rows, lo, hi, (int)blockIdx.x - npr, matvec_grid_n(d.n_wg, down.rows));
    const Resid rr = load_resid_b(pb.x, E, lo, hi, nt, rpw);
    Frag ga[CfgB<T, NP, 1>::U], gb[CfgB<T, NP, 1>::U];
    load_first_b<T, NP, 1>(down, down, lo, hi, ga, gb);
    if (threadIdx.x == 0) wait_count(q.cnt + 64 * (blockIdx.x & 7), npr, q.flag);
    asm volatile("s_barrier" ::: "memory");
    ActPre<NP> ap;
    act_issue<NP, true>(pb.act, KR, nt, ap);
    float *res = resid_lds(smem, KR, nt, rpw);
    store_resid_b(rr, res, nt, rpw);
    act_store<NP, true>(ap, pb.act, KR, smem, nt);
    stream_rows_b<T, NP, 1>(down, down, lo, hi, ga, gb, smem, nt, [&](int row, int t, float v, float) {
        const float r = res[t * rpw + row - lo];
        pb.x[(size_t)t * E + row] = v + r;
    });
}

__global__ __launch_bounds__(ST) void k_pf_embed(LlmDims d, QMat emb, PrefillBuffers pb, int p0) {
    const int t = blockIdx.x;
    embed_row(emb, pb.tokens[p0 + t], d.n_embd, pb.x + (size_t)t * d.n_embd);
}

// ------------------------------------------------------------------ batched decode (B utterances)
// lm_head of the B residual streams with ONE pass over the output matrix (final RMSNorm +
// quantization per stream in the prologue, as k_lm_head does for one): logits[b][row] and,
// per stream, this workgroup's Gumbel-max partial over its rows (the decode sampler's noise
// gumbel(seed_b, step_b, row), so every stream draws exactly what a single-stream decode with
// its seed draws). A wave's row values park in LDS (<= 128 rows per wave, host-checked).
template <int NP, int T>
__global__ __launch_bounds__(MT) void k_bt_lm_head(LlmDims d, const float *norm_w, QMat lm, PrefillBuffers pb,
                                                   BatchBuffers bb, int nt) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float bs_[MW];
    __shared__ int bi_[MW];
    const int K = d.n_embd, KR = rec_k(K, T);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int lo, hi;
    wave_range(d, lm.rows, lo, hi);
    ActPre<NP> ap;
    act_issue<NP>(pb.act, KR, nt, ap);
    Frag ga[CfgB<T, NP, 1>::U], gb[CfgB<T, NP, 1>::U];
    load_first_b<T, NP, 1>(lm, lm, lo, hi, ga, gb);
    act_store<NP>(ap, pb.act, KR, smem, nt);
    float *vals = reinterpret_cast<float *>(smem + pf_lds_bytes(KR, nt, 0)) + (size_t)wave * nt * 128;
    stream_rows_b<T, NP, 1>(lm, lm, lo, hi, ga, gb, smem, nt, [&](int row, int t, float v, float) {
        vals[t * 128 + row - lo] = v;
    });
    lds_barrier();
    for (int t = 0; t < nt; ++t) {
        const SampleCfg sc = bb.cfg[t];
        const int step = bb.st[t].step;
        const uint64_t seed = ((uint64_t)sc.seed_hi << 32) | sc.seed_lo;
        float best = -INFINITY;
        int bi = INT_MAX;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = lo + lane + 64 * h;
            if (row < hi) {
                const float v = vals[t * 128 + row - lo];
                bb.logits[(size_t)t * lm.rows + row] = v;
                if (row >= sc.lo && row < sc.hi) {
                    const float g = sc.temp > 0.0f ? v / sc.temp + gumbel(seed, step, row) : v;
                    if (g > best || (g == best && row < bi)) best = g, bi = row;
                }
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float ov = __shfl_xor(best, o);
            const int oi = __shfl_xor(bi, o);
            if (ov > best || (ov == best && oi < bi)) best = ov, bi = oi;
        }
        if (lane == 0) bs_[wave] = best, bi_[wave] = bi;
        lds_barrier();
        if (threadIdx.x == 0) {
            for (int w = 1; w < MW; ++w)
                if (bs_[w] > best || (bs_[w] == best && bi_[w] < bi)) best = bs_[w], bi = bi_[w];
            float *o = bb.smp + ((size_t)t * gridDim.x + blockIdx.x) * 2;
            o[0] = best;
            o[1] = __int_as_float(bi);
        }
        lds_barrier();
    }
}

// The batched lm_head's sampling partials from logits already in bb.logits ([t][rows], the
// int8 matrix-core lm_head, MIO_BT_LM_MMQ): workgroup b of nblk takes rows [R b / nblk,
// R (b + 1) / nblk) and writes, per stream, the Gumbel-max over its allowed rows as
// k_bt_lm_head does (largest value, lowest row on ties: a total order, so k_bt_sample's
// reduction picks the same token whatever the partition).
__global__ __launch_bounds__(MT) void k_bt_gumbel(int R, BatchBuffers bb, int nt) {
    // one wave per stream (t = wave, wave + 8, ..): its row loads go out 12 per lane at a time
    // and it reduces with shuffles alone (no workgroup barrier between streams)
    constexpr int U = 12;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r0 = (int)((long)R * blockIdx.x / gridDim.x), r1 = (int)((long)R * (blockIdx.x + 1) / gridDim.x);
    for (int t = wave; t < nt; t += MW) {
        const SampleCfg sc = bb.cfg[t];
        const int step = bb.st[t].step;
        const uint64_t seed = ((uint64_t)sc.seed_hi << 32) | sc.seed_lo;
        const int lo = max(r0, sc.lo), hi = min(r1, sc.hi);
        const float *lg = bb.logits + (size_t)t * R;
        float best = -INFINITY;
        int bi = INT_MAX;
        for (int base = lo; base < hi; base += 64 * U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = lg[min(base + lane + 64 * u, hi - 1)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int row = base + lane + 64 * u;
                if (row < hi) {
                    const float g = sc.temp > 0.0f ? v[u] / sc.temp + gumbel(seed, step, row) : v[u];
                    if (g > best || (g == best && row < bi)) best = g, bi = row;
                }
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float ov = __shfl_xor(best, o);
            const int oi = __shfl_xor(bi, o);
            if (ov > best || (ov == best && oi < bi)) best = ov, bi = oi;
        }
        if (lane == 0) {
            float *o = bb.smp + ((size_t)t * gridDim.x + blockIdx.x) * 2;
            o[0] = best;
            o[1] = __int_as_float(bi);
        }
    }
}

// One workgroup per stream b: the lm_head partials -> the sampled token (k_sample's
// selection rule), the token ring, end-token flag, the next embedding into pb.x[b], and the
// state advance. A stream whose step budget (cfg.max_steps) is spent, or that sampled an end
// token, is frozen: nothing is recorded and its position no longer advances.
__global__ __launch_bounds__(ST) void k_bt_sample(LlmDims d, QMat emb, int nblk, PrefillBuffers pb,
                                                  BatchBuffers bb) {
    __shared__ float bs_[ST / 64];
    __shared__ int bi_[ST / 64];
    __shared__ int tok_s;
    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the step's last launch: both sets of the in-launch quantization counters start the next
    // step at zero (launch_layers alternates them within a step)
    if (t == 0 && tid < 16 && pb.qcnt)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(pb.qcnt + 64 * tid), 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const SampleCfg sc = bb.cfg[t];
    StepState *st = bb.st + t;
    const int step = st->step;
    const float *smp = bb.smp + (size_t)t * nblk * 2;
    float best = -INFINITY;
    int bi = INT_MAX;
    for (int i = tid; i < nblk; i += ST) {
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
    if (lane == 0) bs_[wave] = best, bi_[wave] = bi;
    lds_barrier();
    if (tid == 0) {
        for (int w = 1; w < ST / 64; ++w)
            if (bs_[w] > best || (bs_[w] == best && bi_[w] < bi)) best = bs_[w], bi = bi_[w];
        int tok = bi;
        if (tok == INT_MAX) tok = sc.lo;
        if (sc.force && step < sc.n_force && sc.force[step] >= 0) tok = sc.force[step];
        tok_s = tok;
    }
    lds_barrier();
    const int tok = tok_s;
    // a stream whose step budget is spent or that sampled its end token stays frozen
    // (test-to-speech.cpp:168-170: the reference decodes nothing after the end token)
    const bool live = step < sc.max_steps && !st->done;
    if (live) embed_row(emb, tok, d.n_embd, pb.x + (size_t)t * d.n_embd);
    if (tid == 0 && live) {
        sc.out_tokens[step] = tok;
        if (tok == sc.eos0 || tok == sc.eos1) st->done = 1, signal_host_done(sc);
        st->token = tok;
        // a stream ending at a full context stays frozen on its last cache row
        st->pos = min(st->pos + 1, d.n_ctx - 1);
        st->step = step + 1;
    }
}

__global__ __launch_bounds__(ST) void k_bt_embed(LlmDims d, QMat emb, PrefillBuffers pb, BatchBuffers bb) {
    const int t = blockIdx.x;
    embed_row(emb, bb.st[t].token, d.n_embd, pb.x + (size_t)t * d.n_embd);
}

template <int HD>
void launch_bt_attention(int G, dim3 grid, hipStream_t s, const LlmDims &d, const LayerW &L, _Float16 *kc,
                         _Float16 *vc, const PrefillBuffers &pb, int att_q) {
    const float *qn = L.q_norm, *kn = L.k_norm, *bi = L.bqkv;
    switch (G) {
        case 1: hipLaunchKernelGGL((k_bt_attention<HD, 1>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, pb, att_q); break;
        case 2: hipLaunchKernelGGL((k_bt_attention<HD, 2>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, pb, att_q); break;
        case 3: hipLaunchKernelGGL((k_bt_attention<HD, 3>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, pb, att_q); break;
        case 4: hipLaunchKernelGGL((k_bt_attention<HD, 4>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, pb, att_q); break;
        case 8: hipLaunchKernelGGL((k_bt_attention<HD, 8>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, pb, att_q); break;
        default: break;
    }
}

template <int HD>
void launch_pf_attention(int G, dim3 grid, hipStream_t s, const LlmDims &d, const _Float16 *kc, const _Float16 *vc,
                         const PrefillBuffers &pb, int att_q) {
    switch (G) {
        case 1: hipLaunchKernelGGL((k_pf_attention<HD, 1>), grid, dim3(AttCfg<HD>::NT), 0, s, d, kc, vc, pb, att_q); break;
        case 2: hipLaunchKernelGGL((k_pf_attention<HD, 2>), grid, dim3(AttCfg<HD>::NT), 0, s, d, kc, vc, pb, att_q); break;
        case 3: hipLaunchKernelGGL((k_pf_attention<HD, 3>), grid, dim3(AttCfg<HD>::NT), 0, s, d, kc, vc, pb, att_q); break;
        case 4: hipLaunchKernelGGL((k_pf_attention<HD, 4>), grid, dim3(AttCfg<HD>::NT), 0, s, d, kc, vc, pb, att_q); break;
        case 8: hipLaunchKernelGGL((k_pf_attention<HD, 8>), grid, dim3(AttCfg<HD>::NT), 0, s, d, kc, vc, pb, att_q); break;
        default: break;
    }
}

// Dynamic LDS beyond the default 64 KB needs the per-kernel opt-in (once per kernel and
// device: the attribute applies to the current device; the limit leaves room for the
// kernel's static LDS). Keyed by (device, kernel address): kernels of one signature share a
// function type.
constexpr int LDS_DYN_MAX = LDS_MAX - 1024;
template <class Kern>
void allow_lds(Kern k) {
    static std::mutex mu;
    static std::vector<std::pair<int, const void *>> done;
    const void *p = reinterpret_cast<const void *>(k);
    int dev = 0;
    hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    for (const auto &q : done)
        if (q.first == dev && q.second == p) return;
    hipFuncSetAttribute(p, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_DYN_MAX);
    done.push_back({dev, p});
}

// residual rows per wave of a matvec over `rows` rows on `grid` workgroups (wave_range)
int rows_per_wave(int rows, int grid) {
    const int rg = (rows + grid - 1) / grid;
    return (rg + MW - 1) / MW;
}

// Largest token count per launch that fits LDS (and the two residual registers).
int tokens_per_launch(int K, int nt, int rpw) {
    int n = nt;
    while (n > 1 && (pf_lds_bytes(K, n, rpw) > (size_t)LDS_DYN_MAX || n * rpw > 128)) --n;
    return n;
}

PrefillBuffers shifted(const LlmDims &d, const PrefillBuffers &pb, int t, int K) {
    PrefillBuffers q = pb;
    q.act += (size_t)t * act_bytes(K);
    q.x += (size_t)t * d.n_embd;
    q.qkv += (size_t)t * (d.n_head + 2 * d.n_kv) * d.hd;
    q.h += (size_t)t * d.n_ff;
    q.part += (size_t)t * d.n_head * d.max_splits * part_rec(d.hd);
    q.att += (size_t)t * d.n_head * d.hd;
    q.att_cnt += (size_t)t * d.n_kv;
    q.pos += (size_t)t * pb.pos_stride;
    q.seq += (size_t)t * pb.seq_stride;
    return q;
}

// act records of nt tokens (k_bt_quant): mode 0 RMSNorm(src) * w, 1 src; ak = akind of the
// consuming weights (0 Q8_0, 1 Q8_K, 2 BF16)
void launch_quant(const LlmDims &d, int mode, const float *src, int K, const float *w, int ak,
                  const PrefillBuffers &pb, int nt, hipStream_t s) {
    // plain rows: one workgroup per (token, 2048 elements) instead of per token (MIO_QSPLIT=0:
    // per token, for A/B)
    static const bool qsplit = !(getenv("MIO_QSPLIT") && getenv("MIO_QSPLIT")[0] == '0');
    if (mode == 1 && qsplit && K % 256 == 0 && ak != 2) {
        hipLaunchKernelGGL(k_bt_quant_split, dim3(nt, (K + 2047) / 2048), dim3(MT), 0, s, src, K, ak, pb);
        return;
    }
    const int np = pick_np(K);
    auto go = [&]<int NP>() {
        const size_t lds = smem_bytes(K);
        if (mode == 0)
            hipLaunchKernelGGL((k_bt_quant<NP, 0>), dim3(nt), dim3(MT), lds, s, d, src, K, w, ak, pb);
        else
            hipLaunchKernelGGL((k_bt_quant<NP, 1>), dim3(nt), dim3(MT), lds, s, d, src, K, w, ak, pb);
    };
    if (np == 1)
        go.template operator()<1>();
    else if (np == 3)
        go.template operator()<3>();
    else
        go.template operator()<6>();
}

// Every layer for nt tokens of pb (residual streams pb.x in, out): one weight pass per
// matvec launch (sub-launches only where a token range does not fit LDS), each preceded by
// the launch that quantizes its activations once (k_bt_quant).
// decode: every token is its own sequence (the batched decode step): attention per token
// with the RoPE / KV append inside (k_bt_attention).
// MIO_BT_WGM (A/B, default 1): grid multiplier of the one-pass batched matvecs (two workgroups
// per CU need a MIO_BT_MINB=2 build: <= 128 VGPRs, and <= 80 KB of LDS)
static LlmDims bt_wgm(const LlmDims &d, int K) {
    static const int m = getenv("MIO_BT_WGM") ? atoi(getenv("MIO_BT_WGM")) : 1;
    LlmDims r = d;
    if (m > 1 && pick_np(K) == 1) r.n_wg = d.n_wg * m;
    return r;
}

void launch_layers(const LlmDims &d, const LayerW *layers, int n_layer, _Float16 *kcache, _Float16 *vcache,
                   const PrefillBuffers &pb, int nt, int n_chunks, bool decode, hipStream_t s) {
    const size_t layer_kv = (size_t)d.n_kv * d.n_ctx * d.hd;
    const int G = d.n_head / d.n_kv;
    // sub-launches over token ranges that fit LDS: f(t_off, n, shifted buffers)
    // (K = the act record's K, rec_k: twice the row length for BF16 weights)
    auto over_tokens = [&](int K, int rpw, auto &&f) {
        const int per = tokens_per_launch(K, nt, rpw);
        for (int t = 0; t < nt; t += per) f(t, nt - t < per ? nt - t : per, shifted(d, pb, t, K));
    };
    // matvecs on the int8 matrix cores (llm_mmq.hip) above 8 tokens per launch, the dot4
    // streaming engine below up to 8 (both bit-exact with the decode step). Same-box A/B,
    // aggregate x realtime: 8 streams 1.7B Q4_K_M dot4 139 / MMQ 133, 2.6B Q8_0 101 / 80;
    // 16 streams 2.6B Q8_0 134 / 144; a 64-token prefill chunk 10.4 / 2.7 ms.
    // MIO_MMQ=0 / 1 forces one engine.
    static const int mmq_env = getenv("MIO_MMQ") ? atoi(getenv("MIO_MMQ")) : -1;
    const bool mmq_all = mmq_env >= 0 ? mmq_env != 0 : nt > 8;
    // At <= 8 tokens the engine is chosen per launch kind (bit 0 attn_in, 1 attn_out, 2 ffn_in,
    // 3 ffn_down set = int8 MFMA). r04: the 16x16 MFMA tiles load 16 B per lane (llm_mmq.hip,
    // swap_halves) and every K-quant matvec runs on the matrix cores (8-stream 1.7B Q4_K_M step
    // 1.516 ms vs 1.640 with q|k|v + gate|up only and 1.676 before the 16-B loads,
    // profiles/r04_batch8_mmq16_ab.txt); Q8_0 (one-pass kernels compiled with the pair path
    // alone, k_mmq16 P1): O and gate|up on MFMA too, q|k|v on the dot4 engine quantizing in the
    // launch, down on dot4 (2.6B 8-stream step 2.026 ms vs 2.059 with q|k|v only, 2.061 adding
    // down).
    // MIO_MMQ_MASK overrides the set for every type (A/B).
    static const int mmq_mask = getenv("MIO_MMQ_MASK") ? atoi(getenv("MIO_MMQ_MASK")) : -1;
    auto use_mmq = [&](int kind, int type) {
        // Q8_0 O and gate|up only where their 16-B pair kernels apply (K % 256 == 0, one pass)
        const bool q8_pair = d.n_embd % 256 == 0 && d.n_embd <= 2048 && (d.n_head * d.hd) % 256 == 0 &&
                             d.n_head * d.hd <= 2048;
        const int mask = mmq_mask >= 0 ? mmq_mask : (type == 8 ? (q8_pair ? 7 : 1) : 15);
        // BF16 weights: the streaming dot engine (v_dot2 in the decode's lane order) at any token
        // count; the matrix-core matmuls are int8
        return type != 30 && (mmq_all || (nt <= 8 && mmq_env < 0 && ((mask >> kind) & 1)));
    };
    const bool mmq = mmq_all;
    // MIO_BT_FQ (bits: 1 attn_in, 2 ffn_in; default below): launches of <= 8 tokens over K <= 2048
    // RMSNorm + quantize in the launch from inputs loaded ahead of the weights (xpre), on the
    // dot4 engine, instead of behind a k_bt_quant launch (and, for q|k|v, on the matrix cores).
    // 8-stream steps (graph; profiles/r04_fq_ab.txt): 2.6B Q8_0 2.354 ms with attn_in only,
    // 2.362 both, 2.488 neither or ffn_in only; 1.7B Q4_K_M 1.837 / 1.881 / 1.843 / 1.891
    // MIO_BT_ATT=0: the batched decode step uses k_pf_rope + k_pf_attention (A/B)
    static const bool bt_att = !(getenv("MIO_BT_ATT") && getenv("MIO_BT_ATT")[0] == '0');
    decode = decode && bt_att;
    // MIO_BT_QF (default 1): in the batched decode, the 16x16 matmuls quantize their input in
    // the launch (launch_mmq_q: producer workgroups + counters) instead of behind a k_bt_quant
    // launch; the counter sets alternate per fused launch (k_bt_sample zeroes both at the end of
    // each step)
    static const bool qf_env = !(getenv("MIO_BT_QF") && getenv("MIO_BT_QF")[0] == '0');
    // MIO_BT_DQ=0: the dot4 down keeps its k_bt_quant_split launch (A/B)
    static const bool dq_env = !(getenv("MIO_BT_DQ") && getenv("MIO_BT_DQ")[0] == '0');
    // default: the Q8_0 q|k|v in-launch on dot4 only where the matrix cores cannot quantize in
    // the launch themselves (r05: C4 169.0-169.3x with q|k|v on k_mmq16 + producers vs
    // 161.8-162.2x on dot4, profiles/r05_c4_qkv_mfma_ab.txt); none for the K-quants (every
    // matvec on the matrix cores)
    static const int fq2_env = getenv("MIO_BT_FQ") ? atoi(getenv("MIO_BT_FQ")) : -1;
    const bool qkv_qf = decode && qf_env && pb.qcnt && d.n_embd % 256 == 0 && d.n_embd <= 2048;
    auto fq2 = [&](int kind, int type) {
        const bool q8_pair = d.n_embd % 256 == 0 && d.n_embd <= 2048;
        const bool on = fq2_env >= 0 ? ((fq2_env >> kind) & 1) != 0 : (type == 8 && (kind == 0 ? !qkv_qf : !q8_pair));
        return !mmq && nt <= MW && pick_np(d.n_embd) == 1 && on && type != 30;
    };
    static const bool att_q_env = !(getenv("MIO_ATT_Q") && getenv("MIO_ATT_Q")[0] == '0');
    int qi = 0;
    auto fused_q = [&](const MmqSeg *sg, const int *ty, int nseg, int mode, const MmqArgs &a, const float *src,
                       const float *nw, int qmode) {
        if (!decode || !qf_env || !pb.qcnt) return false;
        const int set = qi & 1;
        const MmqQuant q{src, nw, qmode, d.eps, pb.qcnt + 512 * set, pb.qcnt + 512 * (1 - set), pb.qcnt + kQcntFlag};
        if (!launch_mmq_q(sg, ty, nseg, mode, a, q, s)) return false;
        ++qi;
        return true;
    };
    const int QD = (d.n_head + 2 * d.n_kv) * d.hd;
    for (int il = 0; il < n_layer; ++il) {
        const LayerW &L = layers[il];
        if (L.conv) {
            // lfm2 short-conv layer: RMSNorm + in_proj -> B | C | X rows, the gated conv (k_bt_conv)
            // -> out_proj -> x += ., ring update. Always on the matrix cores (bit-exact with the
            // decode step's matvec at any token count).
            const int n = d.n_embd;
            float *ring = pb.ring + (size_t)il * kConvSlots * n;
            launch_quant(d, 0, pb.x, n, L.attn_norm, akind(L.in_proj.type), pb, nt, s);
            const MmqSeg sg{L.in_proj, mmq_tiles(L.in_proj.rows), 0};
            launch_mmq(&sg, &L.in_proj.type, 1, MMQ_STORE, MmqArgs{pb.act, act_bytes(n), n, nt, pb.qkv, 3 * n, {}}, s);
            const int np = pick_np(n);
            const int kq = L.out_proj.type != 8;
            if (np == 1)
                hipLaunchKernelGGL((k_bt_conv<1>), dim3(nt), dim3(MT), smem_bytes(n), s, d, L.conv_w, ring, kq, pb);
            else if (np == 3)
                hipLaunchKernelGGL((k_bt_conv<3>), dim3(nt), dim3(MT), smem_bytes(n), s, d, L.conv_w, ring, kq, pb);
            else
                hipLaunchKernelGGL((k_bt_conv<6>), dim3(nt), dim3(MT), smem_bytes(n), s, d, L.conv_w, ring, kq, pb);
            hipLaunchKernelGGL(k_bt_conv_state, dim3(nt), dim3(ST), 0, s, d, ring, pb, nt);
            const MmqSeg so{L.out_proj, mmq_tiles(L.out_proj.rows), 0};
            launch_mmq(&so, &L.out_proj.type, 1, MMQ_RESID, MmqArgs{pb.act, act_bytes(n), n, nt, pb.x, n, {}}, s);
        } else {
            _Float16 *kc = kcache + il * layer_kv, *vc = vcache + il * layer_kv;
            // the attention merger writes the O matvec's activation records when every kv head's
            // G * hd outputs are whole quantization blocks (MIO_ATT_Q=0: a k_bt_quant launch)
            const int gh = G * d.hd;
            const int att_q = !att_q_env || L.wo.type == 30
                                  ? -1
                                  : (L.wo.type == 8 ? (gh % 32 == 0 ? 0 : -1) : (gh % 256 == 0 ? 1 : -1));
            const bool fa = fq2(0, L.wq.type);
            const bool mq0 = !fa && use_mmq(0, L.wq.type);
            const MmqSeg sg0[3] = {{L.wq, mmq_tiles(L.wq.rows), 0}, {L.wk, mmq_tiles(L.wk.rows), L.wq.rows},
                                   {L.wv, mmq_tiles(L.wv.rows), L.wq.rows + L.wk.rows}};
            const int ty0[3] = {L.wq.type, L.wk.type, L.wv.type};
            const MmqArgs a0{pb.act, act_bytes(d.n_embd), d.n_embd, nt, pb.qkv, QD, {}};
            const bool q0 = mq0 && fused_q(sg0, ty0, 3, MMQ_STORE, a0, pb.x, L.attn_norm, 0);
            if (!fa && !q0)
                launch_quant(d, 0, pb.x, d.n_embd, L.attn_norm, akind(L.wq.type), pb, nt, s);
            if (q0) {
            } else if (mq0) {
                launch_mmq(sg0, ty0, 3, MMQ_STORE, a0, s);
            } else {
                int GW, g_qk;
                attn_in_grid(d, L, GW, g_qk);
                const int KR = rec_k(d.n_embd, L.wq.type);
                over_tokens(KR, 0, [&](int, int n, const PrefillBuffers &q) {
                    const size_t lds = pf_lds_bytes(KR, n, 0);
                    dispatch_nt<true>(d.n_embd, L.wq.type, [&]<int NP, int TQ>() {
                        auto go = [&]<int TV>() {
                            if constexpr (NP == 1 && TQ != 30) {
                                if (fa) {
                                    allow_lds(k_pf_attn_in<NP, TQ, TV, 2>);
                                    hipLaunchKernelGGL((k_pf_attn_in<NP, TQ, TV, 2>), dim3(GW), dim3(MT), lds, s, d,
                                                       L.attn_norm, L.wq, L.wk, L.wv, g_qk, q, n);
                                    return;
                                }
                            }
                            allow_lds(k_pf_attn_in<NP, TQ, TV>);
                            hipLaunchKernelGGL((k_pf_attn_in<NP, TQ, TV>), dim3(GW), dim3(MT), lds, s, d, L.attn_norm,
                                               L.wq, L.wk, L.wv, g_qk, q, n);
                        };
                        if constexpr (TQ == 8 || TQ == 30) {
                            go.template operator()<TQ>();
                        } else {
                            if (L.wv.type == 14)
                                go.template operator()<14>();
                            else
                                go.template operator()<12>();
                        }
                    });
                });
            }
            if (decode) {
                const dim3 grid(d.n_kv * nt, n_chunks);
                if (d.hd == 128)
                    launch_bt_attention<128>(G, grid, s, d, L, kc, vc, pb, att_q);
                else
                    launch_bt_attention<64>(G, grid, s, d, L, kc, vc, pb, att_q);
            } else {
                {
                    const dim3 grid(d.n_head + d.n_kv, nt);
                    if (d.hd == 128)
                        hipLaunchKernelGGL((k_pf_rope<128>), grid, dim3(64), 0, s, d, L.q_norm, L.k_norm, L.bqkv, kc,
                                           vc, pb);
                    else
                        hipLaunchKernelGGL((k_pf_rope<64>), grid, dim3(64), 0, s, d, L.q_norm, L.k_norm, L.bqkv, kc,
                                           vc, pb);
                }
                const dim3 grid(d.n_kv * nt, n_chunks);
                if (d.hd == 128)
                    launch_pf_attention<128>(G, grid, s, d, kc, vc, pb, att_q);
                else
                    launch_pf_attention<64>(G, grid, s, d, kc, vc, pb, att_q);
            }
            if (att_q < 0) launch_quant(d, 1, pb.att, L.wo.k, nullptr, akind(L.wo.type), pb, nt, s);
            if (use_mmq(1, L.wo.type)) {
                const MmqSeg sg{L.wo, mmq_tiles(L.wo.rows), 0};
                launch_mmq(&sg, &L.wo.type, 1, MMQ_RESID, MmqArgs{pb.act, act_bytes(L.wo.k), L.wo.k, nt, pb.x, d.n_embd, {}},
                           s);
            } else {
                const LlmDims dw = bt_wgm(d, L.wo.k);
                const int grid = matvec_grid(dw, L.wo.rows), rpw = rows_per_wave(L.wo.rows, grid);
                const int KR = rec_k(L.wo.k, L.wo.type);
                over_tokens(KR, rpw, [&](int, int n, const PrefillBuffers &q) {
                    dispatch_nt<true>(L.wo.k, L.wo.type, [&]<int NP, int T>() {
                        allow_lds(k_pf_attn_out<NP, T>);
                        hipLaunchKernelGGL((k_pf_attn_out<NP, T>), dim3(grid), dim3(MT), pf_lds_bytes(KR, n, rpw), s,
                                           dw, L.wo, q, n, rpw);
                    });
                });
            }
        }
        const bool ff = fq2(1, L.gate.type);
        const bool mq2 = !ff && use_mmq(2, L.gate.type);
        const MmqSeg sg2{L.gate, mmq_tiles(L.gate.rows), 0};
        const MmqArgs a2{pb.act, act_bytes(d.n_embd), d.n_embd, nt, pb.h, d.n_ff, L.up};
        const bool q2 = mq2 && fused_q(&sg2, &L.gate.type, 1, MMQ_SWIGLU, a2, pb.x, L.ffn_norm, 0);
        if (!ff && !q2)
            launch_quant(d, 0, pb.x, d.n_embd, L.ffn_norm, akind(L.gate.type), pb, nt, s);
        if (q2) {
        } else if (mq2) {
            launch_mmq(&sg2, &L.gate.type, 1, MMQ_SWIGLU, a2, s);
        } else {
            const LlmDims dw = bt_wgm(d, d.n_embd);
            const int grid = matvec_grid(dw, L.gate.rows);
            const int KR = rec_k(d.n_embd, L.gate.type);
            over_tokens(KR, 0, [&](int, int n, const PrefillBuffers &q) {
                dispatch_nt<true>(d.n_embd, L.gate.type, [&]<int NP, int T>() {
                    if constexpr (NP == 1 && T != 30) {
                        if (ff) {
                            allow_lds(k_pf_ffn_in<NP, T, 2>);
                            hipLaunchKernelGGL((k_pf_ffn_in<NP, T, 2>), dim3(grid), dim3(MT), pf_lds_bytes(d.n_embd, n, 0),
                                               s, dw, L.ffn_norm, L.gate, L.up, q, n);
                            return;
                        }
                    }
                    allow_lds(k_pf_ffn_in<NP, T>);
                    hipLaunchKernelGGL((k_pf_ffn_in<NP, T>), dim3(grid), dim3(MT), pf_lds_bytes(KR, n, 0), s, dw,
                                       L.ffn_norm, L.gate, L.up, q, n);
                });
            });
        }
        const bool mq3 = use_mmq(3, L.down.type);
        const MmqSeg sg3{L.down, mmq_tiles(L.down.rows), 0};
        const MmqArgs a3{pb.act, act_bytes(L.down.k), L.down.k, nt, pb.x, d.n_embd, {}};
        const bool q3 = mq3 && fused_q(&sg3, &L.down.type, 1, MMQ_RESID, a3, pb.h, nullptr, 1);
        // the dot4 down quantizing h in the launch (Q8_0 / Q8_K, every token in one launch)
        const int KD = L.down.k, akd = akind(L.down.type);
        const bool q3d = !mq3 && decode && qf_env && pb.qcnt && dq_env && KD % 256 == 0 && akd != 2 &&
                         tokens_per_launch(rec_k(KD, L.down.type), nt,
                                           rows_per_wave(L.down.rows, matvec_grid(d, L.down.rows))) >= nt;
        if (!q3 && !q3d) launch_quant(d, 1, pb.h, L.down.k, nullptr, akind(L.down.type), pb, nt, s);
        if (q3) {
        } else if (mq3) {
            launch_mmq(&sg3, &L.down.type, 1, MMQ_RESID, a3, s);
        } else if (q3d) {
            const int grid = matvec_grid(d, L.down.rows), rpw = rows_per_wave(L.down.rows, grid);
            const int KR = rec_k(KD, L.down.type), nch = (KD + 2047) / 2048;
            const int set = qi & 1;
            ++qi;
            const MmqQuant q{pb.h, nullptr, 1, d.eps, pb.qcnt + 512 * set, pb.qcnt + 512 * (1 - set), pb.qcnt + kQcntFlag};
            const size_t lds = std::max(pf_lds_bytes(KR, nt, rpw), act_bytes(KD));
            dispatch_nt<true>(KD, L.down.type, [&]<int NP, int T>() {
                allow_lds(k_pf_ffn_down_q<NP, T>);
                hipLaunchKernelGGL((k_pf_ffn_down_q<NP, T>), dim3(nt * nch + grid), dim3(MT), lds, s, d, L.down, pb, nt,
                                   rpw, q, nch);
            });
        } else {
            const int grid = matvec_grid(d, L.down.rows), rpw = rows_per_wave(L.down.rows, grid);
            const int KR = rec_k(L.down.k, L.down.type);
            over_tokens(KR, rpw, [&](int, int n, const PrefillBuffers &q) {
                dispatch_nt<true>(L.down.k, L.down.type, [&]<int NP, int T>() {
                    allow_lds(k_pf_ffn_down<NP, T>);
                    hipLaunchKernelGGL((k_pf_ffn_down<NP, T>), dim3(grid), dim3(MT), pf_lds_bytes(KR, n, rpw),
                                       s, d, L.down, q, n, rpw);
                });
            });
        }
    }
}

}  // namespace

void launch_prefill_chunk(const LlmDims &d, const LayerW *layers, int n_layer, _Float16 *kcache,
                          _Float16 *vcache, const QMat &tok_embd, const PrefillBuffers &pb, int p0, int nt,
                          int n_chunks, hipStream_t s) {
    if (nt <= 0) return;
    hipLaunchKernelGGL(k_pf_embed, dim3(nt), dim3(ST), 0, s, d, tok_embd, pb, p0);
    launch_layers(d, layers, n_layer, kcache, vcache, pb, nt, n_chunks, false, s);
}

size_t prefill_act_bytes(int k_max) { return act_bytes(k_max) * kPrefillB; }
int prefill_rec_k(int K, int type) { return rec_k(K, type); }

// parity entry (mio_hip_debug_mmq): nt activation rows x[t][K] quantized as the decode does
// (plain_quant), then y[t][rows] = W x[t] on the int8-MFMA matmul
size_t debug_act_bytes(int K) { return act_bytes(K); }
void launch_debug_mmq(const QMat &W, const QMat &up, int mode, const float *x, int nt, char *act, float *y,
                      hipStream_t s) {
    LlmDims d{};
    PrefillBuffers pb{};
    pb.act = act;
    launch_quant(d, 1, x, W.k, nullptr, akind(W.type), pb, nt, s);
    const MmqSeg sg{W, mmq_tiles(W.rows), 0};
    launch_mmq(&sg, &W.type, 1, mode, MmqArgs{act, act_bytes(W.k), W.k, nt, y, W.rows, up}, s);
}

size_t batch_lm_head_lds(const LlmDims &d, int B, int type) {
    return pf_lds_bytes(rec_k(d.n_embd, type), B, 0) + (size_t)MW * B * 128 * 4;
}

bool batch_supported(const LlmDims &d, int B, int lm_type) {
    return B >= 1 && B <= kBatchMax && batch_lm_head_lds(d, B, lm_type) <= (size_t)LDS_DYN_MAX;
}

void launch_batch_step(const LlmDims &d, const LayerW *layers, int n_layer, _Float16 *kcache, _Float16 *vcache,
                       const float *out_norm, const QMat &lm, const QMat &tok_embd, const PrefillBuffers &pb,
                       const BatchBuffers &bb, int B, hipStream_t s) {
    launch_layers(d, layers, n_layer, kcache, vcache, pb, B, d.max_splits, true, s);
    launch_quant(d, 0, pb.x, d.n_embd, out_norm, akind(lm.type), pb, B, s);
    const int nblk = matvec_grid(d, d.n_vocab);  // the batched lm_head keeps one workgroup per CU
    // the logits on the int8 matrix cores (launch_mmq, the dot engine's values bit for bit),
    // then the sampling partials from them (k_bt_gumbel): 8 streams 1.7B 217.0-217.5x vs
    // 214.5-215.0x with k_bt_lm_head (dot4, partials fused), C4 179.5-179.6 vs 177.3-177.5x
    // (profiles/r05_bt_lm_mmq_ab.txt). MIO_BT_LM_MMQ=0: k_bt_lm_head
    static const bool lm_mmq = !(getenv("MIO_BT_LM_MMQ") && getenv("MIO_BT_LM_MMQ")[0] == '0');
    if (lm_mmq && lm.type != 30) {
        const MmqSeg sg{lm, mmq_tiles(lm.rows), 0};
        launch_mmq(&sg, &lm.type, 1, MMQ_STORE,
                   MmqArgs{pb.act, act_bytes(d.n_embd), d.n_embd, B, bb.logits, lm.rows, {}}, s);
        hipLaunchKernelGGL(k_bt_gumbel, dim3(nblk), dim3(MT), 0, s, lm.rows, bb, B);
        hipLaunchKernelGGL(k_bt_sample, dim3(B), dim3(ST), 0, s, d, tok_embd, nblk, pb, bb);
        return;
    }
    dispatch_nt<true>(d.n_embd, lm.type, [&]<int NP, int T>() {
        allow_lds(k_bt_lm_head<NP, T>);
        hipLaunchKernelGGL((k_bt_lm_head<NP, T>), dim3(nblk), dim3(MT), batch_lm_head_lds(d, B, T), s, d, out_norm, lm,
                           pb, bb, B);
    });
    hipLaunchKernelGGL(k_bt_sample, dim3(B), dim3(ST), 0, s, d, tok_embd, nblk, pb, bb);
}

void launch_batch_embed(const LlmDims &d, const QMat &tok_embd, const PrefillBuffers &pb, const BatchBuffers &bb,
                        int B, hipStream_t s) {
    hipLaunchKernelGGL(k_bt_embed, dim3(B), dim3(ST), 0, s, d, tok_embd, pb, bb);
}

}  // namespace mio
