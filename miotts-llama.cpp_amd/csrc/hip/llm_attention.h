// Workgroup bodies shared by the decode step's attention launches (llm_kernels.hip: k_attention,
// k_att_o; llm_layer_att.hip: k_layer_att): the attention chunk workgroup, the O-projection
// consumer of the fused launches and two small register helpers.
#pragma once
#include "llm_device.h"

namespace mio {
namespace {

// residual rows of this wave (<= 64) in one register: lane i holds x[lo + i]
__device__ inline float load_resid(const float *x, int lo, int hi) {
    const int lane = threadIdx.x & 63;
    return lo + lane < hi ? x[lo + lane] : 0.0f;
}
__device__ inline float lane_value(float v, int i) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i));
}

// The body of one (chunk ch, kv head kvh) workgroup at position pos (first AttCfg<HD>::NT
// threads). rdy: the fused attention + O launch's merge counter (attn_merge_last), or null.
// WQ (k_layer_att: q|k|v produced in the same launch): the K/V rows are loaded and staged
// first, then one lane waits until the kv head's q|k|v row counter (b.att_cnt + kQkvOff +
// kQkvStride * kvh) reaches (G + 2) * HD rows, and the head rows are loaded sc1.
// Returns false for a workgroup with no positions (or after an end token).
template <int HD, int G, bool DG, bool WQ = false>
__device__ __forceinline__ bool attention_wg(const LlmDims &d, const float *q_norm, const float *k_norm,
                                             const float *bqkv, _Float16 *kc, _Float16 *vc, const LlmBuffers &b,
                                             int ch, int kvh, int pos, int *rdy) {
    static_assert(!WQ || MIO_ATT_MFMA, "the q|k|v wait is on the MFMA attention path");
    constexpr bool kDiag = DG;
    using C = AttCfg<HD>;
    constexpr int PER = HD / 64;
    __shared__ float qs[G][HD];
    __shared__ float knew[HD], vnew[HD];
#if MIO_ATT_MFMA
    using A = AttM<HD>;
    static_assert(C::NT == A::NT, "attention workgroup size");
    __shared__ __attribute__((aligned(16))) char img[2 * A::IMG];
    __shared__ __attribute__((aligned(16))) _Float16 qh[G][HD];
#else
    __shared__ float wres[C::NW][G][HD + 2];
#endif

    const int t0 = ch * ATT_CHUNK;
    if (t0 > pos || b.st->done) return false;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float2 *rope = b.rope + (size_t)pos * (HD / 2);
    // q heads (waves 0..G-1) and, for the chunk owning `pos`, the new k/v row (wave G); the
    // loads of each wave's first head go out before its K/V rows (row `pos` is never consumed
    // from the cache)
    const bool owner = pos < t0 + ATT_CHUNK;
    auto head_src = [&](int hh, HeadIn<HD> &in) {
        const bool isk = hh == G;
        const size_t so = isk ? (size_t)(d.n_head + kvh) * HD : (size_t)(kvh * G + hh) * HD;
        const size_t vo = (size_t)(d.n_head + d.n_kv + kvh) * HD;
        head_load<HD, WQ ? 16 : 0>(b.qkv + so, bqkv ? bqkv + so : nullptr, isk ? k_norm : q_norm, rope, d, in,
                                   isk ? b.qkv + vo : nullptr, isk && bqkv ? bqkv + vo : nullptr);
    };
    HeadIn<HD> hin;
#if MIO_ATT_MFMA
    h8 kr[A::VI], vr[A::VI];
    if constexpr (WQ) {
        kv_issue<HD>(kc + (size_t)kvh * d.n_ctx * HD, vc + (size_t)kvh * d.n_ctx * HD, t0, pos, kr, vr);
        kv_stage<HD>(kr, vr, owner ? pos - t0 : -1, img, img + A::IMG);
        MIO_TL_MARK(b, 4);  // K / V staged
        if (MIO_TIDX == 0)
            wait_count(b.att_cnt + kQkvOff + kQkvStride * kvh, (G + 2) * HD, b.att_cnt + kRdyFlag);
        asm volatile("s_barrier" ::: "memory");
        MIO_TL_MARK(b, 3);  // q|k|v rows of this kv head written
        if (wave < G + (owner ? 1 : 0)) head_src(wave, hin);
    } else {
        if (wave < G + (owner ? 1 : 0)) head_src(wave, hin);
        kv_issue<HD>(kc + (size_t)kvh * d.n_ctx * HD, vc + (size_t)kvh * d.n_ctx * HD, t0, pos, kr, vr);
    }
#else
    if (wave < G + (owner ? 1 : 0)) head_src(wave, hin);
    h8 kr[C::IT], vr[C::IT];
    load_kv_rows<HD>(kc + (size_t)kvh * d.n_ctx * HD, vc + (size_t)kvh * d.n_ctx * HD, t0, pos, kr, vr);
#endif
    MIO_TRACE(b, 1);
    MIO_TL_MARK1(b);
    for (int hh = wave; hh < G + (owner ? 1 : 0); hh += C::NW) {
        const bool isk = hh == G;
        if (hh != wave) head_src(hh, hin);
        head_prep<HD>(hin, d, isk ? knew : qs[hh]);
        if (isk) {
            _Float16 *kd = kc + ((size_t)kvh * d.n_ctx + pos) * HD;
            _Float16 *vd = vc + ((size_t)kvh * d.n_ctx + pos) * HD;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int p = lane + 64 * i;
                const float vr16 = f16r(hin.vv[i]);
                vnew[p] = vr16;
                kd[p] = (_Float16)knew[p];
                vd[p] = (_Float16)vr16;
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
    MIO_TRACE(b, 6);  // this wave's head prepared
    if constexpr (!WQ) kv_stage<HD>(kr, vr, owner ? pos - t0 : -1, img, img + A::IMG);
    MIO_TRACE(b, 7);  // this thread's K / V rows arrived and staged
    lds_barrier();
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    const uint32_t gs = (uint32_t)(d.max_splits * C::REC), head0 = (uint32_t)(kvh * G) * gs;
    attend_chunk_mfma<HD, G>(qh, img, img + A::IMG, t0, pos, d.scale, b.part + head0 + (uint32_t)ch * C::REC, gs,
                             DG ? b.trace : nullptr);
#else
    lds_barrier();
    MIO_TRACE(b, 2);
    MIO_TL_MARK(b, 2);
    // the slot owning row `pos` takes it from LDS (exact f16 values, the cache row's bits)
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
    const uint32_t gs = (uint32_t)(d.max_splits * C::REC), head0 = (uint32_t)(kvh * G) * gs;
    attend_chunk<HD, G>(qs, kr, vr, t0, pos, d.scale, wres, b.part + head0 + (uint32_t)ch * C::REC, gs,
                        DG ? b.trace : nullptr, MIO_TL_DIAGSLOT(b));
#endif
    attn_merge_last<HD, G>(b.part, head0, gs, pos / ATT_CHUNK + 1, b.att_cnt + kvh, b.att + (size_t)kvh * G * HD, -1,
                           {}, 0, rdy, (kDiag && b.tl) ? MIO_TL_SLOT(b) : nullptr);
    return true;
}

// ------------------------------------------------------------------ attention + O, one launch
// k_att_o: the attention workgroups and the O-projection workgroups of a layer in ONE launch
// (MI355X_MICROARCH "boundary": a dependent launch boundary costs ~1.2-1.5 us, and the O
// workgroups' weights and residual rows are loaded while the attention runs). Roles are taken
// from the position (every workgroup reads it): workgroups [0, n_act) with n_act =
// (pos / ATT_CHUNK + 1) * n_kv are the attention chunks (chunk bid / n_kv, kv head bid % n_kv;
// their first AttCfg::NT threads), the next matvec_grid(wo) are k_attn_out's workgroups, the
// rest return. The n_kv merging workgroups store the head outputs write-through and add 1 to
// each of the 8 counter shards at b.att_cnt + kRdyOff (attn_merge_last); an O workgroup issues
// its weight group, waits for n_kv on its shard (one lane, wait_count), then loads the outputs
// sc1. Deadlock-free by dispatch
// order: every producer has a lower workgroup index than every consumer and never waits, so
// it is dispatched (and finishes) whatever the residency. The counter is zeroed by the next
// launch, k_ffn_in (kernel boundary ordered), and by reset_tickets.
// Two-level arrival counter of an in-launch hand-off with n signalling workgroups (r = the
// signaller's index among them; first wave, after every wave's stores drained and a workgroup
// barrier): one add to arrival shard r % 8 (<= n / 8 adds per word); the workgroup whose add
// returns its shard's last count adds 1 to each of the 8 ready replicas (one instruction, 8
// lanes), where a consumer polls replica r' % 8 until min(n, 8) (MI355X_MICROARCH hand-off
// rows 1-2; k_ffn's h counter).
__device__ __forceinline__ void signal_two_level(int *arr, int *rdy, int r, int n) {
    if (MIO_TIDX < 64) {
        int last = 0;
        if (MIO_TIDX == 0) {
            const int sh = r & (kFfnShards - 1), n_sh = (n - sh + kFfnShards - 1) / kFfnShards;
            last = __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(arr + kFfnStride * sh), 1,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_sh - 1;
        }
        if (__builtin_amdgcn_readfirstlane(last) && MIO_TIDX < kFfnShards)
            __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(rdy + kFfnStride * MIO_TIDX), 1,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ __forceinline__ void wait_two_level(int *rdy, int r, int n, int *flag) {
    if (MIO_TIDX == 0) wait_count(rdy + kFfnStride * (r & (kFfnShards - 1)), min(n, kFfnShards), flag);
    asm volatile("s_barrier" ::: "memory");
}

// residual rows [lo, hi) of this wave, lane i holding x[lo + i], by sc1 loads (x was stored
// write-through by other workgroups of the launch); lanes past hi read 0 (out of range)
__device__ __forceinline__ float load_resid_sc1(const float *x, int lo, int hi) {
    const int lane = threadIdx.x & 63;
    return __uint_as_float(
        __builtin_amdgcn_raw_buffer_load_b32(rsrc(x, (uint32_t)hi * 4u), (uint32_t)(lo + lane) * 4u, 0, 16));
}

// XS (the whole-layer launch, k_layer): the x rows are stored write-through and, once every
// wave's stores drained, the workgroup signals the two-level x counter (kXOff / kXRdy of
// b.att_cnt) for the launch's gate|up workgroups
template <int NP, int T, int SU, bool DG, bool XS = false>
__device__ __forceinline__ void o_consumer(const LlmDims &d, const QMat &wo, const LlmBuffers &b, int ob, int no) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = wo.k;
    const Smem s = carve(smem, K);
    int lo, hi;
    wave_range(wo.rows, lo, hi, ob, no);
    const float xres = load_resid(b.x, lo, hi);
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 1, SU, MIO_SMALL_AUX>(wo, wo, lo, hi, ga, gb);
    if (MIO_TIDX == 0)
        wait_count(b.att_cnt + kRdyOff + kRdyStride * (blockIdx.x & (kRdyShards - 1)), d.n_kv, b.att_cnt + kRdyFlag);
    asm volatile("s_barrier" ::: "memory");
    MIO_TL_MARK(b, 3);
    XRegs<NP> xr;
    load_x<NP, 16>(b.att, nullptr, K, xr);
    x_after_weights(xr);
    MIO_TL_MARK1(b);
    plain_quant(xr, K, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 1, SU, MIO_SMALL_AUX>(wo, wo, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        const float r = lane_value(xres, row - lo);
        if ((threadIdx.x & 63) == 0) {
            if constexpr (XS)
                st1_sc1(b.x, (uint32_t)row * 4u, v + r);
            else
                b.x[row] = v + r;
        }
    });
    if constexpr (XS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        MIO_TL_MARK(b, 6);  // x rows written through
        signal_two_level(b.att_cnt + kXOff, b.att_cnt + kXRdy, ob, no);
    }
}

}  // namespace
}  // namespace mio
