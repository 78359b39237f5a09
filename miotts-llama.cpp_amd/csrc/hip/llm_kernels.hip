// Single-token LLM decode step for gfx950 (replaces llama_decode for one token,
// test-to-speech.cpp:178-185 / :589-596, and the sampler chain :127-130, :165-166).
//
// Per layer, four weight-streaming launches plus attention:
//   k_attn_in   RMSNorm(x) -> act re-quantized in LDS (Q8_K / Q8_0, ggml vec_dot_type)
//               -> q|k|v dequant-matvec
//   k_attention per (128-position chunk, kv head): q/k RMSNorm (qwen3) + RoPE, F16 KV-cache
//               append by the chunk that owns `pos`, online-softmax partial records
//   k_attn_out  chunk merge + re-quantization in the prologue -> O matvec -> x += .
//   k_ffn_in    RMSNorm(x) -> re-quantize -> gate & up matvec -> silu(g)*u
//   k_ffn_down  re-quantize h -> down matvec -> x += .
// An lfm2 short-conv layer replaces the first three with k_attn_in over in_proj (B | C | X)
// and k_conv_out (gated depthwise conv over a 4-slot ring of earlier positions -> out_proj).
// then k_lm_head (final RMSNorm + logits + per-workgroup Gumbel-max). The token is drawn from
// those partials by the next step's layer-0 attn_in (its prologue, beside its first weight
// loads) or, after the last step of a run, by k_sample (token, next embedding, position++).
// All state is device-resident (StepState), so one hipGraph of a step replays every token
// with no host round trip.
//
// Matvec engine ("streaming rows"): one 512-thread workgroup per CU, each wave streams a
// contiguous run of rows. A row is NP "passes" of 2048 weights; one pass of one row is a
// unit = one 16-B-per-lane load (+ block headers). Units are loaded U at a time into
// registers, one group ahead of the group being reduced, and the first group is issued
// before the activation prologue so HBM latency overlaps the RMSNorm/quantization, which
// runs once per CU. The other global loads a workgroup needs up front (x, norm weights,
// residual values) are issued before the first weight load, so in-order vmcnt waits
// never stall on the prefetched group.
//
// Matvec arithmetic = ggml's integer block dots: per superblock the integer sums
// (v_dot4c_i32_i8 on the raw 4/6/8-bit codes x int8 activations) are bit-exact with
// ggml vec_dot_{q4_K,q6_K}_q8_K / vec_dot_q8_0_q8_0; only the float sum over blocks is
// reordered. Weight streams are 16 B per lane, one contiguous run per row (split layout,
// csrc/host/quant.h).
#include "llm_attention.h"

#include <algorithm>
#include <cstdlib>

#pragma clang fp contract(off)

namespace mio {
namespace {


// k_attn_in (RMSNorm + q|k|v matvec, + layer 0: the previous step's sampler) lives in
// llm_attn_in.hip.

template <int NP, int T, int SU, bool DG>
__global__ __launch_bounds__(MT) void k_attn_out(LlmDims d, QMat wo, LlmBuffers b) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    const int K = wo.k;
    const Smem s = carve(smem, K);
    int lo, hi;
    wave_range(d, wo.rows, lo, hi);
    const uint32_t dn = done_issue(b);
    XRegs<NP> xr;
    load_x(b.att, nullptr, K, xr);
    const float xres = load_resid(b.x, lo, hi);
    x_gate();
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 1, SU, MIO_SMALL_AUX>(wo, wo, lo, hi, ga, gb);
    x_after_weights(xr);
    if (done_now(dn)) return;
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    plain_quant(xr, K, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 1, SU, MIO_SMALL_AUX>(wo, wo, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        const float r = lane_value(xres, row - lo);
        if ((threadIdx.x & 63) == 0) b.x[row] = v + r;
    });
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// lfm2 short-conv layer, second launch (the first is k_attn_in over in_proj: bcx in b.qkv):
// the gated conv of this position (conv_load / conv_quant: bx = B * X, the window over the
// layer's ring, y = C * conv) re-quantized in the prologue -> out_proj matvec -> x += .
// Workgroup 0 stores this position's bx into ring slot pos & 3; the window reads slots of
// pos - 1 and pos - 2, so no workgroup reads what another writes in this launch.
template <int NP, int T, int SU, bool DG>
__global__ __launch_bounds__(MT) void k_conv_out(LlmDims d, QMat wo, const float *conv_w, float *ring, LlmBuffers b) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    const int K = wo.k;
    const Smem s = carve(smem, K);
    const uint32_t dn = done_issue(b);
    const int pos = cur_pos(b.st, d);
    const ConvPrev p1{pos >= 1 ? ring + (size_t)((pos - 1) & (kConvSlots - 1)) * K : nullptr, 0};
    const ConvPrev p2{pos >= 2 ? ring + (size_t)((pos - 2) & (kConvSlots - 1)) * K : nullptr, 0};
    ConvRegs<NP> cr;
    conv_load(b.qkv, p1, p2, conv_w, K, cr);
    int lo, hi;
    wave_range(d, wo.rows, lo, hi);
    const float xres = load_resid(b.x, lo, hi);
    x_gate();
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 1, SU>(wo, wo, lo, hi, ga, gb);
    conv_after_weights(cr);
    if (done_now(dn)) return;
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    conv_quant(cr, K, akind(T), s, blockIdx.x == 0 ? ring + (size_t)(pos & (kConvSlots - 1)) * K : nullptr,
               MIO_TL_DIAGSLOT(b));
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 1, SU>(wo, wo, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        const float r = lane_value(xres, row - lo);
        if ((threadIdx.x & 63) == 0) b.x[row] = v + r;
    });
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// adv (layer 0): folds a sampled-in-attn_in token into pos / step (StepState.pending).
__device__ __forceinline__ void advance_state(StepState *st, const LlmDims &d) {
    const int p = st->pending;
    st->pos = min(st->pos + p, d.n_ctx - 1);
    st->step = st->step + p;
    st->pending = 0;
}

// Both k_layer counter sets (every counter but the timeout flag; the chunk tickets reset
// themselves): lm_head, after the step's last k_layer (kernel boundary ordered).
__device__ __forceinline__ void zero_layer_sets(int *cnt) {
    constexpr int n = kRdyShards + kQkvMax + 4 * kFfnShards;
    for (int i = MIO_TIDX; i < 2 * n; i += MT) {
        const int j = i % n;
        const int o = j < kRdyShards ? kRdyOff + kRdyStride * j
                    : j < kRdyShards + kQkvMax ? kQkvOff + kQkvStride * (j - kRdyShards)
                                               : kFfnOff + kFfnStride * (j - kRdyShards - kQkvMax);
        __hip_atomic_store((__attribute__((address_space(1))) int *)(cnt + kLayOff + (i / n) * kLaySet + o), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int NP, int T, int SU, bool DG>
__global__ __launch_bounds__(MT) void k_ffn_in(LlmDims d, const float *norm_w, QMat gate, QMat up,
                                               LlmBuffers b, int adv) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    const uint32_t dn = done_issue(b);
    XRegs<NP> xr;
    load_x(b.x, norm_w, K, xr);
    x_gate();
    // k_att_o / k_layer_att's merge and q|k|v counters: zero again for the next layer's
    // launch (kernel boundary)
    if (blockIdx.x == 0 && MIO_TIDX < kRdyShards)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kRdyOff + kRdyStride * MIO_TIDX), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 1 && MIO_TIDX < d.n_kv)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kQkvOff + kQkvStride * MIO_TIDX), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int lo, hi;
    wave_range(d, gate.rows, lo, hi);
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 2, SU>(gate, up, lo, hi, ga, gb);
    x_after_weights(xr);
    if (done_now(dn)) {  // layer 0 still folds the end token's step (the host counts it)
        if (adv && blockIdx.x == 0 && MIO_TIDX == 0) advance_state(b.st, d);
        return;
    }
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    rmsnorm_quant(xr, K, d.eps, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 2, SU>(gate, up, lo, hi, ga, gb, s.a, [&](int row, float g, float u) {
        if ((threadIdx.x & 63) == 0) b.h[row] = silu_f(g) * u;
    }, INT_MAX, DG ? b.trace : nullptr);
    if (adv && blockIdx.x == 0 && MIO_TIDX == 0) advance_state(b.st, d);
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

template <int NP, int T, int SU, bool DG>
__global__ __launch_bounds__(MT) void k_ffn_down(LlmDims d, QMat down, LlmBuffers b) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    const int K = down.k;
    const Smem s = carve(smem, K);
    const uint32_t dn = done_issue(b);
    XRegs<NP> xr;
    load_x(b.h, nullptr, K, xr);
    int lo, hi;
    wave_range(d, down.rows, lo, hi);
    const float xres = load_resid(b.x, lo, hi);
    x_gate();
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 1, SU>(down, down, lo, hi, ga, gb);
    x_after_weights(xr);
    if (done_now(dn)) return;
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    plain_quant(xr, K, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 1, SU>(down, down, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        const float r = lane_value(xres, row - lo);
        if ((threadIdx.x & 63) == 0) b.x[row] = v + r;
    }, INT_MAX, DG ? b.trace : nullptr);
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// The FFN pair of a layer as ONE launch (which = 12, MIO_FFN_FUSE): two workgroup roles of
// one grid.
//   [0, GI)        k_ffn_in's body (RMSNorm + quant -> gate|up matvec + SwiGLU), the h rows
//                  stored write-through (sc1); every storing wave drains its stores
//                  (vmcnt(0)), a workgroup barrier, then ONE lane adds 1 to shard blockIdx % 8
//                  of the h counter (b.att_cnt + kFfnOff); the shard's last arriver adds 1 to
//                  each of the 8 ready replicas (kFfnRdy)
//   [GI, GI + GD)  k_ffn_down's body: residual rows and the first weight group issued, one lane
//                  waits until its ready replica (blockIdx % 8) counts every shard, a barrier
//                  releases the waves, h is loaded with sc1 loads, quantized, streamed, x += .
// MI355X_MICROARCH hand-off rows 1-2 (sharded arrivals, replicated ready word, every load of the
// handed-off bytes sc1; a first version polled all 8 arrival shards from every down workgroup:
// 256 pollers per word, the step 12 % slower);
// the boundary it removes costs ~1.5-2.1 us plus the down's first-load latency, which now
// overlaps the gate|up stream. Producers never wait and precede every consumer, so in-order
// dispatch makes progress whatever the residency. The consumers write x only after every
// producer has signalled, i.e. after every producer's read of x. Arithmetic = the two
// launches' (bit-identical). The counter is zeroed by the next launch (attn_in / layer_att /
// lm_head), the timeout flag is k_att_o's (kRdyFlag).
template <int NP, int T, int SU, int NPD, int TD, int SUD, bool DG>
__global__ __launch_bounds__(MT) void k_ffn(LlmDims d, const float *norm_w, QMat gate, QMat up, QMat down,
                                            LlmBuffers b, int adv, int GI) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    const uint32_t dn = done_issue(b);
    if ((int)blockIdx.x < GI) {
        const int K = d.n_embd;
        const Smem s = carve(smem, K);
        XRegs<NP> xr;
        load_x(b.x, norm_w, K, xr);
        x_gate();
        if (blockIdx.x == 0 && MIO_TIDX < kRdyShards)
            __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kRdyOff + kRdyStride * MIO_TIDX),
                               0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (blockIdx.x == 1 && MIO_TIDX < d.n_kv)
            __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kQkvOff + kQkvStride * MIO_TIDX),
                               0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int lo, hi;
        wave_range(gate.rows, lo, hi, blockIdx.x, GI);
        Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
        load_first<T, NP, 2, SU>(gate, up, lo, hi, ga, gb);
        x_after_weights(xr);
        if (done_now(dn)) {  // layer 0 still folds the end token's step (the host counts it)
            if (adv && blockIdx.x == 0 && MIO_TIDX == 0) advance_state(b.st, d);
            return;
        }
        MIO_TL_MARK1(b);
        rmsnorm_quant(xr, K, d.eps, akind(T), s, MIO_TL_DIAGSLOT(b));
        MIO_TL_MARK(b, 2);
        stream_rows<T, NP, 2, SU>(gate, up, lo, hi, ga, gb, s.a, [&](int row, float g, float u) {
            if ((threadIdx.x & 63) == 0) st1_sc1(b.h, (uint32_t)row * 4u, silu_f(g) * u);
        });
        if (adv && blockIdx.x == 0 && MIO_TIDX == 0) advance_state(b.st, d);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (MIO_TIDX < 64) {
            int last = 0;
            if (MIO_TIDX == 0) {
                const int sh = blockIdx.x & (kFfnShards - 1), n_sh = (GI - sh + kFfnShards - 1) / kFfnShards;
                last = __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(b.att_cnt + kFfnOff + kFfnStride * sh),
                                              1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_sh - 1;
            }
            // the shard's last arriver: its add returned after every other add of the shard, each
            // made after that workgroup's h stores had drained; one instruction, 8 lanes
            if (__builtin_amdgcn_readfirstlane(last) && MIO_TIDX < kFfnShards)
                __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(b.att_cnt + kFfnRdy + kFfnStride * MIO_TIDX),
                                       1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        const int K = down.k;
        const Smem s = carve(smem, K);
        const int GD = (int)gridDim.x - GI, ob = (int)blockIdx.x - GI;
        int lo, hi;
        wave_range(down.rows, lo, hi, ob, GD);
        const float xres = load_resid(b.x, lo, hi);
        Frag ga[Cfg<NPD, SUD>::U], gb[Cfg<NPD, SUD>::U];
        load_first<TD, NPD, 1, SUD>(down, down, lo, hi, ga, gb);
        if (done_now(dn)) return;  // the producers return too: nobody signals, nobody waits
        if (MIO_TIDX == 0)
            wait_count(b.att_cnt + kFfnRdy + kFfnStride * (blockIdx.x & (kFfnShards - 1)), min(GI, kFfnShards),
                       b.att_cnt + kRdyFlag);
        asm volatile("s_barrier" ::: "memory");
        MIO_TL_MARK(b, 3);
        XRegs<NPD> xr;
        load_x<NPD, 16>(b.h, nullptr, K, xr);
        x_after_weights(xr);
        MIO_TL_MARK1(b);
        plain_quant(xr, K, akind(TD), s, MIO_TL_DIAGSLOT(b));
        MIO_TL_MARK(b, 2);
        stream_rows<TD, NPD, 1, SUD>(down, down, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
            const float r = lane_value(xres, row - lo);
            if ((threadIdx.x & 63) == 0) b.x[row] = v + r;
        });
    }
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// the instantiated (np, gate|up type, su, down np, down type, down su): 1.7B Q4_K_M (down Q4_K
// or Q6_K) and BF16, 0.1B Q8_0, 2.6B Q8_0 (and LFM2-2.6B), the tiny test presets' shapes
#define MIO_FFN_SHAPES(X) \
    X(1, 12, 6, 3, 12, 3)  \
    X(1, 12, 6, 3, 14, 3)  \
    X(1, 30, 6, 3, 30, 3)  \
    X(1, 8, 2, 1, 8, 1)    \
    X(1, 8, 0, 6, 8, 0)

struct FfnShape {
    int np, t, su, npd, td, sud, GI, GD;
};
FfnShape ffn_shape(const LlmDims &d, const LayerW &L) {
    FfnShape f{};
    f.GI = matvec_grid(d, L.gate.rows), f.GD = matvec_grid(d, L.down.rows);
    f.np = pick_np(d.n_embd), f.t = L.gate.type;
    f.su = pick_su(max_wave_units(L.gate.rows, f.GI, f.np, 2), f.np);
    f.npd = pick_np(L.down.k), f.td = L.down.type;
    f.sud = pick_su(max_wave_units(L.down.rows, f.GD, f.npd, 1), f.npd);
    return f;
}

template <bool DG>
bool launch_ffn(const LlmDims &d, const LayerW &L, const LlmBuffers &b, int adv, hipStream_t st, bool dry) {
    if (L.up.type != L.gate.type) return false;
    const FfnShape f = ffn_shape(d, L);
    const size_t lds = std::max(smem_bytes(d.n_embd), smem_bytes(L.down.k));
    bool found = false;
#define MIO_FFN_CASE(NP, T, SU, NPD, TD, SUD)                                                                     \
    if (!found && f.np == NP && f.t == T && f.su == SU && f.npd == NPD && f.td == TD && f.sud == SUD) {          \
        found = true;                                                                                            \
        if (!dry)                                                                                                \
            hipLaunchKernelGGL((k_ffn<NP, T, SU, NPD, TD, SUD, DG>), dim3(f.GI + f.GD), dim3(MT), lds, st, d,       \
                               L.ffn_norm, L.gate, L.up, L.down, b, adv, f.GI);                                  \
    }
    MIO_FFN_SHAPES(MIO_FFN_CASE)
#undef MIO_FFN_CASE
    return found;
}

// final RMSNorm (once per CU) + logits + per-workgroup Gumbel-max partial. A wave's rows
// (<= 128) are parked one per lane (two registers) and the noise is drawn for 64 rows at
// a time after the stream.
template <int NP, int T, bool DG>
__global__ __launch_bounds__(MT) void k_lm_head(LlmDims d, const float *norm_w, QMat lm, LlmBuffers b) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float bs_[MW];
    __shared__ int bi_[MW];
    const int K = d.n_embd;
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    if (blockIdx.x == 2 && MIO_TIDX < 2 * kFfnShards)  // the previous k_ffn's h counters (kernel boundary ordered)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kFfnOff + kFfnStride * MIO_TIDX), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 3) zero_layer_sets(b.att_cnt);  // the k_layer counter sets (the last layer's is in use)
    const Smem s = carve(smem, K);
    XRegs<NP> xr;
    load_x(b.x, norm_w, K, xr);
    x_gate();
    int lo, hi;
    wave_range(d, lm.rows, lo, hi);
    Frag ga[Cfg<NP>::U], gb[Cfg<NP>::U];
    load_first<T, NP, 1, 0, MIO_LM_AUX>(lm, lm, lo, hi, ga, gb);
    x_after_weights(xr);
    // the sampling configuration and step are needed only by the epilogue: loaded behind the
    // first weight group (in front of it, their scalar-load wait held the weight stream back)
    asm volatile("" ::: "memory");
    const SampleCfg sc = *b.cfg;
    const int step = b.st->step;
    if (b.st->done) return;  // no pending sample: the next step's attn_in returns too
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    rmsnorm_quant(xr, K, d.eps, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    const int lane = threadIdx.x & 63;
    float r0 = -INFINITY, r1 = -INFINITY;
    stream_rows<T, NP, 1, 0, MIO_LM_AUX>(lm, lm, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        const int k = row - lo;
        r0 = lane == k ? v : r0;
        r1 = lane + 64 == k ? v : r1;
    });
    MIO_TRACE(b, 3);
    const uint64_t seed = ((uint64_t)sc.seed_hi << 32) | sc.seed_lo;
    float best = -INFINITY;
    int bi = INT_MAX;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int row = lo + lane + 64 * h;
        const float v = h ? r1 : r0;
        if (row < hi) {
            b.logits[row] = v;
            if (row >= sc.lo && row < sc.hi) {
                const float t = sc.temp > 0.0f ? v / sc.temp + gumbel(seed, step, row) : v;
                if (t > best || (t == best && row < bi)) best = t, bi = row;
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float ov = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ov > best || (ov == best && oi < bi)) best = ov, bi = oi;
    }
    const int wave = threadIdx.x >> 6;
    if (lane == 0) bs_[wave] = best, bi_[wave] = bi;
    lds_barrier();
    if (threadIdx.x == 0) {
        for (int w = 1; w < MW; ++w)
            if (bs_[w] > best || (bs_[w] == best && bi_[w] < bi)) best = bs_[w], bi = bi_[w];
        b.smp[2 * blockIdx.x] = best;
        b.smp[2 * blockIdx.x + 1] = __int_as_float(bi);
        if (blockIdx.x == 0) b.st->pending = 1;  // sampled by the next step's attn_in or the flush
    }
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// ------------------------------------------------------------------ attention
// One workgroup per (chunk of ATT_CHUNK positions, kv head): q/k RMSNorm (qwen3) + RoPE +
// f16 rounding, the chunk owning `pos` appends the new k/v row to the F16 cache, then a
// softmax over the chunk for the G q heads sharing the kv head, whose partial records
// {O[HD], m, l} the last chunk workgroup to arrive merges into b.att (attn_merge_last):
// ATT_CHUNK (64) -position chunks spread the K/V rows of position ~400 over 7 x n_kv
// workgroups (32 KB each at hd 128), and k_attn_out (or the O workgroups of k_att_o) reads
// the n_head * hd merged values.
template <int HD, int G, bool DG>
__global__ __launch_bounds__(AttCfg<HD>::NT) void k_attention(LlmDims d, const float *q_norm, const float *k_norm,
                                                      const float *bqkv, _Float16 *kc, _Float16 *vc, LlmBuffers b) {
    constexpr bool kDiag = DG;
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    // every kernel argument the workgroup uses is loaded in the round trip that fetches
    // b.st (without this the compiler sinks them below the pos-dependent exit: a third
    // scalar-load round trip before the first K/V load)
    asm volatile("" ::"s"(kc), "s"(vc), "s"(d.n_ctx), "s"(b.qkv), "s"(b.rope), "s"(q_norm), "s"(k_norm),
                 "s"(b.part), "s"(d.max_splits), "s"(bqkv), "s"(b.att), "s"(b.att_cnt));
    const int pos = cur_pos(b.st, d);
    if (!attention_wg<HD, G, DG>(d, q_norm, k_norm, bqkv, kc, vc, b, blockIdx.x, blockIdx.y, pos, nullptr)) return;
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

template <int HD, bool DG>
void launch_attention(int G, dim3 grid, hipStream_t s, const LlmDims &d, const LayerW &L, _Float16 *kc,
                      _Float16 *vc, const LlmBuffers &b) {
    const float *qn = L.q_norm, *kn = L.k_norm, *bi = L.bqkv;
    switch (G) {
        case 1: hipLaunchKernelGGL((k_attention<HD, 1, DG>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, b); break;
        case 2: hipLaunchKernelGGL((k_attention<HD, 2, DG>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, b); break;
        case 3: hipLaunchKernelGGL((k_attention<HD, 3, DG>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, b); break;
        case 4: hipLaunchKernelGGL((k_attention<HD, 4, DG>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, b); break;
        case 8: hipLaunchKernelGGL((k_attention<HD, 8, DG>), grid, dim3(AttCfg<HD>::NT), 0, s, d, qn, kn, bi, kc, vc, b); break;
        default: break;
    }
}

template <int HD, int G, int NP, int T, int SU, bool DG>
__global__ __launch_bounds__(MT) void k_att_o(LlmDims d, const float *q_norm, const float *k_norm, const float *bqkv,
                                              _Float16 *kc, _Float16 *vc, QMat wo, LlmBuffers b) {
    constexpr bool kDiag = DG;
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    asm volatile("" ::"s"(kc), "s"(vc), "s"(d.n_ctx), "s"(b.qkv), "s"(b.rope), "s"(q_norm), "s"(k_norm),
                 "s"(b.part), "s"(d.max_splits), "s"(bqkv), "s"(b.att), "s"(b.att_cnt));
    const int pos = cur_pos(b.st, d);
    if (b.st->done) return;  // no merge is signalled after an end token: nobody may wait
    const int bid = blockIdx.x, n_act = (pos / ATT_CHUNK + 1) * d.n_kv;
    if (bid < n_act) {
        if (MIO_TIDX >= AttCfg<HD>::NT) return;  // whole waves; s_barrier counts the live ones
        if (!attention_wg<HD, G, DG>(d, q_norm, k_norm, bqkv, kc, vc, b, bid / d.n_kv, bid % d.n_kv, pos,
                                     b.att_cnt + kRdyOff))
            return;
    } else {
        const int no = matvec_grid_n(d.n_wg, wo.rows), ob = bid - n_act;
        if (ob >= no) return;
        o_consumer<NP, T, SU, DG>(d, wo, b, ob, no);
    }
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

template <int NP, int T, int SU, bool DG>
void launch_att_o(int G, int grid, size_t lds, hipStream_t s, const LlmDims &d, const LayerW &L, _Float16 *kc,
                  _Float16 *vc, const LlmBuffers &b) {
    const float *qn = L.q_norm, *kn = L.k_norm, *bi = L.bqkv;
#define MIO_ATT_O(HH, GG) \
    hipLaunchKernelGGL((k_att_o<HH, GG, NP, T, SU, DG>), dim3(grid), dim3(MT), lds, s, d, qn, kn, bi, kc, vc, L.wo, b)
    if (d.hd == 128 && G == 2) MIO_ATT_O(128, 2);
    if (d.hd == 64 && G == 3) MIO_ATT_O(64, 3);
    if (d.hd == 64 && G == 4) MIO_ATT_O(64, 4);
#undef MIO_ATT_O
}

// ------------------------------------------------------------------ sampler / embedding
// The flush sampler (after the last step of a run; the step graph samples inside the next
// step's layer-0 attn_in): the pending token, its embedding into b.x, the state advance.
template <bool DG>
__global__ __launch_bounds__(ST) void k_sample(LlmDims d, QMat emb, int nblk, LlmBuffers b) {
    constexpr bool kDiag = DG;
    __shared__ float rs_[ST / 64];
    __shared__ int ri_[ST / 64];
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    StepState *st = b.st;
    if (!st->pending) return;
    const SampleCfg sc = *b.cfg;
    const int step = st->step;
    const int tok = sample_token<ST>(b.smp, nblk, sc, step, rs_, ri_);
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    embed_row(emb, tok, d.n_embd, b.x);
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
    if (MIO_TIDX == 0) {
        if (step < sc.max_steps) sc.out_tokens[step] = tok;
        if (tok == sc.eos0 || tok == sc.eos1) st->done = 1, signal_host_done(sc);
        st->token = tok;
        // a full context ends generation (host-side step budget); the state never points
        // past the cache, so later diagnostic launches stay in bounds
        st->pos = min(st->pos + 1, d.n_ctx - 1);
        st->step = step + 1;
        st->pending = 0;
    }
}

__global__ __launch_bounds__(ST) void k_embed(LlmDims d, QMat emb, LlmBuffers b) {
    embed_row(emb, b.st->token, d.n_embd, b.x);
}

}  // namespace

// ------------------------------------------------------------------ host launchers
int pick_np(int K) { return K <= 2048 ? 1 : (K <= 6144 ? 3 : 6); }

// at least MW rows per workgroup (every wave owns >= 1 row), at most one workgroup per CU
static_assert(MW == 8, "matvec_grid_n assumes 8 waves per workgroup");
// (hd, G) of the fused launch: 1.7B qwen3 (128, 2), 0.1B (64, 3), 2.6B (64, 4); other shapes
// keep the two launches
bool att_o_supported(int hd, int G) { return (hd == 128 && G == 2) || (hd == 64 && (G == 3 || G == 4)); }
bool ffn_fused_supported(const LlmDims &d, const LayerW &L) {
    return launch_ffn<false>(d, L, LlmBuffers{}, 0, nullptr, true);
}

int matvec_grid(const LlmDims &d, int rows) { return matvec_grid_n(d.n_wg, rows); }

// lm_head workgroups per CU (MIO_LM_WGM, 1..4): the lm_head launch sees n_wg scaled. Two
// per CU (16 waves) stream the 255 MB output matrix in 47.5 us against 49.5 us for one
// (same-box A/B, 1.7B Q4_K_M).
LlmDims lm_dims(const LlmDims &d) {
    static const int mult = [] {
        const char *e = getenv("MIO_LM_WGM");
        const int v = e ? atoi(e) : 2;
        return v < 1 ? 1 : (v > 4 ? 4 : v);
    }();
    LlmDims l = d;
    l.n_wg = d.n_wg * mult;
    return l;
}
int lm_head_blocks(const LlmDims &d) { const LlmDims l = lm_dims(d); return matvec_grid(l, l.n_vocab); }

size_t matvec_lds(int K) { return smem_bytes(K); }


// An empty one-workgroup launch: the reference of mio_hip_llm_time_kernel's launch timing (what
// a launch costs the stream besides its own work)
__global__ void k_nop() {}
void launch_nop(hipStream_t s) { hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s); }

void launch_embed_token(const LlmDims &d, const QMat &tok_embd, const LlmBuffers &b, hipStream_t s) {
    hipLaunchKernelGGL(k_embed, dim3(1), dim3(ST), 0, s, d, tok_embd, b);
}

inline size_t mv_lds(int K) { return smem_bytes(K); }
// lm_head dynamic LDS, optionally padded (MIO_LM_LDS_KB, A/B knob) so that no more than
// 160 KB / size of its workgroups fit on one CU: the dispatcher then has to spread them
size_t lm_lds(int K) {
    static const size_t kb = [] {
        const char *e = getenv("MIO_LM_LDS_KB");
        return e ? (size_t)atoi(e) : (size_t)0;
    }();
    const size_t b = smem_bytes(K);
    return kb * 1024 > b ? std::min(kb * 1024, (size_t)64 * 1024) : b;
}

// Units (row passes) of the busiest wave of a matvec over `rows` rows on `grid` workgroups
// (wave_range), and the single-group size that covers them (0 = streaming groups).
int max_wave_units(int rows, int grid, int np, int nm) {
    const int rg = (rows + grid - 1) / grid, rw = (rg + MW - 1) / MW;
    return rw * np * nm;
}
int pick_su(int units, int np) {
    if (np == 1 && units <= 4) return units;
    if (np == 1 && units <= 6) return 6;
    if (np == 3 && units <= 3) return 3;
    return 0;
}
// Launch one kernel of the step: which = 0 attn_in, 1 attention, 2 attn_out (+ chunk
// merge), 3 ffn_in, 4 ffn_down (layer il), 5 (unused: the final norm is fused into
// lm_head), 6 lm_head, 7 flush sampler; lfm2 short-conv layer il: 8 conv_in (RMSNorm +
// in_proj, the attn_in kernel), 9 conv_out (gated conv + out_proj). Layer 0's attn_in samples the pending token of the
// previous step and layer 0's ffn_in advances pos / step (StepState.pending).
void launch_step_kernel(int which, const LlmDims &d, const LayerW *layers, int il, _Float16 *kcache,
                        _Float16 *vcache, const float *out_norm, const QMat &lm, const QMat &tok_embd,
                        const LlmBuffers &b, hipStream_t s) {
    const size_t layer_kv = (size_t)d.n_kv * d.n_ctx * d.hd;
    const int G = d.n_head / d.n_kv;
    // diagnostic instantiations only when a trace / timeline buffer is attached
    auto go_dg = [&]<bool DG>() {
    switch (which) {
        case 0: {
            launch_attn_in(d, layers[il], il, tok_embd, b, DG, s);
            break;
        }
        case 1: {
            const LayerW &L = layers[il];
            const dim3 grid(d.max_splits, d.n_kv);
            if (d.hd == 128)
                launch_attention<128, DG>(G, grid, s, d, L, kcache + il * layer_kv, vcache + il * layer_kv, b);
            else
                launch_attention<64, DG>(G, grid, s, d, L, kcache + il * layer_kv, vcache + il * layer_kv, b);
            break;
        }
        case 2: {
            const LayerW &L = layers[il];
            const int grid = matvec_grid(d, L.wo.rows);
            dispatch_nt(L.wo.k, L.wo.type, [&]<int NP, int T>() {
                dispatch_su<NP>(pick_su(max_wave_units(L.wo.rows, grid, NP, 1), NP), [&]<int SU>() {
                    hipLaunchKernelGGL((k_attn_out<NP, T, SU, DG>), dim3(grid), dim3(MT), mv_lds(L.wo.k), s, d, L.wo, b);
                });
            });
            break;
        }
        case 10: {  // attention + O in one launch (k_att_o)
            const LayerW &L = layers[il];
            const int grid = d.max_splits * d.n_kv + matvec_grid(d, L.wo.rows);
            dispatch_nt(L.wo.k, L.wo.type, [&]<int NP, int T>() {
                if constexpr (NP == 1)
                    dispatch_su<NP>(pick_su(max_wave_units(L.wo.rows, matvec_grid(d, L.wo.rows), NP, 1), NP), [&]<int SU>() {
                        launch_att_o<NP, T, SU, DG>(G, grid, mv_lds(L.wo.k), s, d, L, kcache + il * layer_kv,
                                                    vcache + il * layer_kv, b);
                    });
            });
            break;
        }
        case 11:  // the attention block in one launch (k_layer_att)
            launch_layer_att(d, layers[il], kcache + il * layer_kv, vcache + il * layer_kv, b, DG, s);
            break;
        case 3: {
            const LayerW &L = layers[il];
            const int grid = matvec_grid(d, L.gate.rows);
            dispatch_nt(d.n_embd, L.gate.type, [&]<int NP, int T>() {
                dispatch_su<NP>(pick_su(max_wave_units(L.gate.rows, grid, NP, 2), NP), [&]<int SU>() {
                    hipLaunchKernelGGL((k_ffn_in<NP, T, SU, DG>), dim3(grid), dim3(MT), mv_lds(d.n_embd), s, d, L.ffn_norm,
                                       L.gate, L.up, b, il == 0 ? 1 : 0);
                });
            });
            break;
        }
        case 4: {
            const LayerW &L = layers[il];
            const int grid = matvec_grid(d, L.down.rows);
            dispatch_nt(L.down.k, L.down.type, [&]<int NP, int T>() {
                dispatch_su<NP>(pick_su(max_wave_units(L.down.rows, grid, NP, 1), NP), [&]<int SU>() {
                    hipLaunchKernelGGL((k_ffn_down<NP, T, SU, DG>), dim3(grid), dim3(MT), mv_lds(L.down.k), s, d, L.down,
                                       b);
                });
            });
            break;
        }
        case 12:  // the FFN pair in one launch (k_ffn)
            launch_ffn<DG>(d, layers[il], b, il == 0 ? 1 : 0, s, false);
            break;
        case 13:  // the whole layer in one launch (k_layer, layers >= 1)
            launch_layer(d, layers[il], il, kcache + il * layer_kv, vcache + il * layer_kv, b, DG, s);
            break;
        case 8: {  // lfm2 conv_in: RMSNorm + in_proj as the attn_in launch (B | C rows, X rows)
            const LayerW &L = layers[il];
            const int n = d.n_embd;
            LayerW V = L;
            V.wq = qmat_rows(L.in_proj, 0, 2 * n);
            V.wk = qmat_rows(L.in_proj, 2 * n, 0);
            V.wv = qmat_rows(L.in_proj, 2 * n, n);
            V.q_norm = V.k_norm = V.bqkv = nullptr;
            launch_attn_in(d, V, il, tok_embd, b, DG, s);
            break;
        }
        case 9: {
            const LayerW &L = layers[il];
            const int grid = matvec_grid(d, L.out_proj.rows);
            float *ring = b.ring + (size_t)il * kConvSlots * d.n_embd;
            dispatch_nt(L.out_proj.k, L.out_proj.type, [&]<int NP, int T>() {
                dispatch_su<NP>(pick_su(max_wave_units(L.out_proj.rows, grid, NP, 1), NP), [&]<int SU>() {
                    hipLaunchKernelGGL((k_conv_out<NP, T, SU, DG>), dim3(grid), dim3(MT), mv_lds(L.out_proj.k), s, d,
                                       L.out_proj, L.conv_w, ring, b);
                });
            });
            break;
        }
        case 6: {
            const LlmDims dl = lm_dims(d);
            dispatch_nt(d.n_embd, lm.type, [&]<int NP, int T>() {
                hipLaunchKernelGGL((k_lm_head<NP, T, DG>), dim3(lm_head_blocks(d)), dim3(MT), lm_lds(d.n_embd), s, dl,
                                   out_norm, lm, b);
            });
            break;
        }
        case 7:
            hipLaunchKernelGGL(k_sample<DG>, dim3(1), dim3(ST), 0, s, d, tok_embd, lm_head_blocks(d), b);
            break;
        default: break;
    }
    };
    if (b.tl || b.trace)
        go_dg.template operator()<true>();
    else
        go_dg.template operator()<false>();
}


}  // namespace mio
