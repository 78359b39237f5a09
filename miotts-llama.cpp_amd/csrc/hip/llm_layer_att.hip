// A decoder layer's attention block as ONE launch of the single-token decode step (layers >= 1;
// llama_decode for one token, test-to-speech.cpp:178-185): RMSNorm + q|k|v matvec, the
// attention chunks and their merge, and the O projection + residual, which are k_attn_in,
// k_attention and k_attn_out's bodies as three workgroup roles of one grid:
//   [0, GW)                q|k|v producers (k_attn_in's body; rows stored write-through, then
//                          the rows each workgroup wrote per kv head added to that head's
//                          counter at b.att_cnt + kQkvOff + kQkvStride * kvh)
//   [GW, GW + n_act)       attention chunks (n_act = (pos / ATT_CHUNK + 1) * n_kv): K/V rows
//                          of the chunk loaded and staged in LDS first, then one lane waits
//                          for the kv head's (G + 2) * hd rows, the head rows are loaded sc1
//                          (attention_wg<..., WQ = true>); the mergers signal the O counters
//   [GW + n_act, + no)     O workgroups (o_consumer, as in k_att_o)
// Every consumer has a higher workgroup index than the producers it waits for, and producers
// never wait, so in-order dispatch makes progress whatever the residency (MI355X_MICROARCH
// "Persistent kernels": hand-offs inside a launch instead of a ~1.2-1.5 us boundary each).
// Layer 0 keeps k_attn_in (its sampler may end the step) + k_att_o. The counters are zeroed by
// the next launch, k_ffn_in. Instantiated for the shipped head shapes and weight types only
// (layer_att_supported); everything else runs the separate launches, whose math is the same.
#include "llm_attention.h"

#pragma clang fp contract(off)

namespace mio {
#if MIO_ATT_MFMA
namespace {

template <int NP, int TQ, int TV, int SU, int HD, int G, bool DG>
__device__ __forceinline__ void qkv_producer(const LlmDims &d, const float *norm_w, const QMat &wq, const QMat &wk,
                                             const QMat &wv, int g_qk, int GW, const LlmBuffers &b) {
    constexpr bool kDiag = DG;
    const int o1 = wq.rows, o2 = wq.rows + wk.rows;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    const uint32_t dn = done_issue(b);
    XRegs<NP> xr;
    load_x(b.x, norm_w, K, xr);
    x_gate();
    auto put = [&](int row, float v) {
        if ((threadIdx.x & 63) == 0) st1_sc1(b.qkv, (uint32_t)row * 4, v);
    };
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    int lo, hi, ra, rb;
    const int bid = blockIdx.x;
    if (bid < g_qk) {
        wave_range(o2, lo, hi, bid, g_qk);
        ra = o2 * bid / g_qk, rb = o2 * (bid + 1) / g_qk;
        load_first<TQ, NP, 1, SU, MIO_SMALL_AUX>(wq, wk, lo, hi, ga, gb, o1);
        x_after_weights(xr);
        if (done_now(dn)) return;
        MIO_TL_MARK1(b);
        rmsnorm_quant(xr, K, d.eps, akind(TQ), s, MIO_TL_DIAGSLOT(b));
        MIO_TL_MARK(b, 2);
        stream_rows<TQ, NP, 1, SU, MIO_SMALL_AUX>(wq, wk, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
            put(row, v);
        }, o1);
    } else {
        const int bv = bid - g_qk, gv = GW - g_qk;
        wave_range(wv.rows, lo, hi, bv, gv);
        ra = o2 + wv.rows * bv / gv, rb = o2 + wv.rows * (bv + 1) / gv;
        load_first<TV, NP, 1, SU, MIO_SMALL_AUX>(wv, wv, lo, hi, ga, gb);
        x_after_weights(xr);
        if (done_now(dn)) return;
        MIO_TL_MARK1(b);
        rmsnorm_quant(xr, K, d.eps, akind(TV), s, MIO_TL_DIAGSLOT(b));
        MIO_TL_MARK(b, 2);
        stream_rows<TV, NP, 1, SU, MIO_SMALL_AUX>(wv, wv, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
            put(o2 + row, v);
        });
    }
    // every row of the workgroup written through, then per kv head ONE add of the workgroup's
    // row count there (runs of equal heads over rows ra .. rb - 1 <= 64, host-checked)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (MIO_TIDX < 64) {
        const int i = MIO_TIDX, r = ra + i;
        auto head_of = [&](int rr) { return rr < o1 ? rr / (HD * G) : (rr < o2 ? (rr - o1) / HD : (rr - o2) / HD); };
        const bool ok = r < rb;
        const int h = ok ? head_of(r) : -1;
        const bool start = ok && (i == 0 || head_of(r - 1) != h);
        const uint64_t m = __ballot(start);
        if (start) {
            const uint64_t nx = i < 63 ? m >> (i + 1) : 0;
            const int end = nx ? i + 1 + __builtin_ctzll(nx) : rb - ra;
            __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(b.att_cnt + kQkvOff + kQkvStride * h),
                                   end - i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int NP, int TQ, int TV, int SU, int HD, int G, int TO, int SUO, bool DG>
__global__ __launch_bounds__(MT) void k_layer_att(LlmDims d, const float *norm_w, QMat wq, QMat wk, QMat wv, int g_qk,
                                                  int GW, const float *q_norm, const float *k_norm, const float *bqkv,
                                                  _Float16 *kc, _Float16 *vc, QMat wo, LlmBuffers b) {
    constexpr bool kDiag = DG;
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    if (blockIdx.x == 2 && MIO_TIDX < 2 * kFfnShards)  // the previous k_ffn's h counters (kernel boundary ordered)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kFfnOff + kFfnStride * MIO_TIDX), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int bid = blockIdx.x;
    if (bid < GW) {
        qkv_producer<NP, TQ, TV, SU, HD, G, DG>(d, norm_w, wq, wk, wv, g_qk, GW, b);
    } else {
        asm volatile("" ::"s"(kc), "s"(vc), "s"(d.n_ctx), "s"(b.qkv), "s"(b.rope), "s"(q_norm), "s"(k_norm),
                     "s"(b.part), "s"(d.max_splits), "s"(bqkv), "s"(b.att), "s"(b.att_cnt));
        const int pos = cur_pos(b.st, d);
        if (b.st->done) return;  // the producers return too: nobody signals, nobody waits
        const int ab = bid - GW, n_act = (pos / ATT_CHUNK + 1) * d.n_kv;
        if (ab < n_act) {
            if (MIO_TIDX >= AttCfg<HD>::NT) return;  // whole waves; s_barrier counts the live ones
            if (!attention_wg<HD, G, DG, true>(d, q_norm, k_norm, bqkv, kc, vc, b, ab / d.n_kv, ab % d.n_kv, pos,
                                               b.att_cnt + kRdyOff))
                return;
        } else {
            const int no = matvec_grid_n(d.n_wg, wo.rows), ob = ab - n_act;
            if (ob >= no) return;
            o_consumer<1, TO, SUO, DG>(d, wo, b, ob, no);
        }
    }
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// ------------------------------------------------------------------ the whole layer as one launch
// k_layer (which = 13, MIO_LAYER_FUSE): k_layer_att's three roles followed by k_ffn's two in ONE
// grid, so the FFN's weights stream while the attention chain runs (MI355X_MICROARCH
// "engine-vs-launches" / "prefetch-credit": the attention block leaves most of the chip idle for
// ~8 us; in the two-launch form the FFN started its 24.6 MB stream only after a boundary):
//   [0, GW)                       q|k|v producers                          (as k_layer_att)
//   [GW, GW + n_act)              attention chunks + mergers               (as k_layer_att)
//   [O0 = GW + n_act, O0 + no)    O workgroups; their x rows are stored write-through and each
//                                 signals the two-level x counter (o_consumer<XS>)
//   [F0 = O0 + no, F0 + GI)       gate|up workgroups: every weight unit of the wave issued at
//                                 dispatch (SU: the whole share is one register group), then the
//                                 x wait, x loaded sc1, RMSNorm + quant, SwiGLU; h stored
//                                 write-through + the two-level h counter (k_ffn's producer)
//   [F0 + GI, F0 + GI + GD)       down workgroups: weights at dispatch, h wait, h and the residual
//                                 rows loaded sc1, x += down h (plain stores: the next launch reads)
//   the rest (slots of inactive attention chunks) returns.
// Every workgroup waits only for workgroups with lower indices, none of which waits for it, so
// in-order dispatch makes progress whatever the residency; the FFN roles are dispatched as the
// producers and chunks retire, well before x is ready. Counters: b.att_cnt is counter set il & 1;
// workgroup 3 zeroes the other set (the previous k_layer's; kernel boundary), workgroup 2 the
// base h counters of a k_ffn before (layer 0). Arithmetic = k_layer_att + k_ffn (bit-identical).
// fgate (MIO_LAYER_GATE): 1 = the FFN workgroups first wait for their kv head's q|k|v rows, so
// their weight burst does not sit in front of the producers' stream; 2 = gate|up waits for the
// chunk merge, down for x, before issuing weights (the attention chain runs without them).
template <int NP, int T, int SU, bool DG>
__device__ __forceinline__ void gate_up_role(const LlmDims &d, const float *norm_w, const QMat &gate, const QMat &up,
                                             const LlmBuffers &b, int r, int GI, int no, int fgate) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    if (fgate == 1) {
        const int kvh = r % d.n_kv;
        if (MIO_TIDX == 0)
            wait_count(b.att_cnt + kQkvOff + kQkvStride * kvh, (d.n_head / d.n_kv + 2) * d.hd, b.att_cnt + kRdyFlag);
        asm volatile("s_barrier" ::: "memory");
    } else if (fgate == 2) {  // the chunk merge is done (the O workgroups' counter)
        if (MIO_TIDX == 0)
            wait_count(b.att_cnt + kRdyOff + kRdyStride * (r & (kRdyShards - 1)), d.n_kv, b.att_cnt + kRdyFlag);
        asm volatile("s_barrier" ::: "memory");
    }
    int lo, hi;
    wave_range(gate.rows, lo, hi, r, GI);
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 2, SU>(gate, up, lo, hi, ga, gb);
    wait_two_level(b.att_cnt + kXRdy, r, no, b.att_cnt + kRdyFlag);
    MIO_TL_MARK(b, 3);
    XRegs<NP> xr;
    load_x<NP, 16>(b.x, norm_w, K, xr);
    x_after_weights(xr);
    MIO_TL_MARK1(b);
    rmsnorm_quant(xr, K, d.eps, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 2, SU>(gate, up, lo, hi, ga, gb, s.a, [&](int row, float g, float u) {
        if ((threadIdx.x & 63) == 0) st1_sc1(b.h, (uint32_t)row * 4u, silu_f(g) * u);
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    signal_two_level(b.att_cnt + kFfnOff, b.att_cnt + kFfnRdy, r, GI);
}

template <int NP, int T, int SU, bool DG>
__device__ __forceinline__ void down_role(const LlmDims &d, const QMat &down, const LlmBuffers &b, int r, int GD,
                                          int GI, int no, int fgate) {
    constexpr bool kDiag = DG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = down.k;
    const Smem s = carve(smem, K);
    if (fgate == 1) {
        const int kvh = r % d.n_kv;
        if (MIO_TIDX == 0)
            wait_count(b.att_cnt + kQkvOff + kQkvStride * kvh, (d.n_head / d.n_kv + 2) * d.hd, b.att_cnt + kRdyFlag);
        asm volatile("s_barrier" ::: "memory");
    } else if (fgate == 2) {  // x is ready (the gate|up workgroups' counter)
        wait_two_level(b.att_cnt + kXRdy, r, no, b.att_cnt + kRdyFlag);
    }
    int lo, hi;
    wave_range(down.rows, lo, hi, r, GD);
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    load_first<T, NP, 1, SU>(down, down, lo, hi, ga, gb);
    wait_two_level(b.att_cnt + kFfnRdy, r, GI, b.att_cnt + kRdyFlag);
    MIO_TL_MARK(b, 3);
    const float xres = load_resid_sc1(b.x, lo, hi);
    XRegs<NP> xr;
    load_x<NP, 16>(b.h, nullptr, K, xr);
    x_after_weights(xr);
    MIO_TL_MARK1(b);
    plain_quant(xr, K, akind(T), s, MIO_TL_DIAGSLOT(b));
    MIO_TL_MARK(b, 2);
    stream_rows<T, NP, 1, SU>(down, down, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        const float rr = lane_value(xres, row - lo);
        if ((threadIdx.x & 63) == 0) b.x[row] = v + rr;
    });
}

template <int NP, int TQ, int TV, int SU, int HD, int G, int TO, int SUO, int FNP, int FT, int FSU, int FNPD, int FTD,
          int FSUD, bool DG>
__global__ __launch_bounds__(MT) void k_layer(LlmDims d, const float *norm_w, QMat wq, QMat wk, QMat wv, int g_qk,
                                              int GW, const float *q_norm, const float *k_norm, const float *bqkv,
                                              _Float16 *kc, _Float16 *vc, QMat wo, const float *ffn_norm, QMat gate,
                                              QMat up, QMat down, int GI, int GD, int *base_cnt, int *other_set,
                                              int fgate, LlmBuffers b) {
    constexpr bool kDiag = DG;
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    if (blockIdx.x == 2 && MIO_TIDX < 2 * kFfnShards)  // a layer-0 k_ffn's h counters (kernel boundary ordered)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(base_cnt + kFfnOff + kFfnStride * MIO_TIDX), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 3) {  // the other counter set (the previous k_layer's): every counter but the flag
        for (int i = MIO_TIDX; i < kRdyShards + kQkvMax + 4 * kFfnShards; i += MT) {
            const int o = i < kRdyShards ? kRdyOff + kRdyStride * i
                        : i < kRdyShards + kQkvMax ? kQkvOff + kQkvStride * (i - kRdyShards)
                                                   : kFfnOff + kFfnStride * (i - kRdyShards - kQkvMax);
            __hip_atomic_store((__attribute__((address_space(1))) int *)(other_set + o), 0, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const int bid = blockIdx.x;
    if (bid < GW) {
        qkv_producer<NP, TQ, TV, SU, HD, G, DG>(d, norm_w, wq, wk, wv, g_qk, GW, b);
    } else {
        asm volatile("" ::"s"(kc), "s"(vc), "s"(d.n_ctx), "s"(b.qkv), "s"(b.rope), "s"(q_norm), "s"(k_norm),
                     "s"(b.part), "s"(d.max_splits), "s"(bqkv), "s"(b.att), "s"(b.att_cnt));
        const int pos = cur_pos(b.st, d);
        if (b.st->done) return;  // the producers return too: nobody signals, nobody waits
        const int ab = bid - GW, n_act = (pos / ATT_CHUNK + 1) * d.n_kv;
        const int no = matvec_grid_n(d.n_wg, wo.rows);
        if (ab < n_act) {
            if (MIO_TIDX >= AttCfg<HD>::NT) return;  // whole waves; s_barrier counts the live ones
            if (!attention_wg<HD, G, DG, true>(d, q_norm, k_norm, bqkv, kc, vc, b, ab / d.n_kv, ab % d.n_kv, pos,
                                               b.att_cnt + kRdyOff))
                return;
        } else if (ab < n_act + no) {
            o_consumer<1, TO, SUO, DG, true>(d, wo, b, ab - n_act, no);
        } else if (ab < n_act + no + GI) {
            gate_up_role<FNP, FT, FSU, DG>(d, ffn_norm, gate, up, b, ab - n_act - no, GI, no, fgate);
        } else if (ab < n_act + no + GI + GD) {
            down_role<FNPD, FTD, FSUD, DG>(d, down, b, ab - n_act - no - GI, GD, GI, no, fgate);
        } else {
            return;
        }
    }
    MIO_TL_END(b);
    MIO_TRACE(b, 15);
}

// the instantiated (np, q|k type, v type, su, hd, G, o type, o su): 1.7B Q4_K_M (v Q4_K or
// Q6_K) and BF16, 0.1B Q8_0, 2.6B Q8_0 (and the LFM2-2.6B attention layers)
#define MIO_LAYER_ATT_SHAPES(X)   \
    X(1, 12, 12, 2, 128, 2, 12, 1) \
    X(1, 12, 14, 2, 128, 2, 12, 1) \
    X(1, 30, 30, 2, 128, 2, 30, 1) \
    X(1, 8, 8, 1, 64, 3, 8, 1)     \
    X(1, 8, 8, 2, 64, 4, 8, 1)

struct Shape {
    int np, tq, tv, su, hd, g, to, suo;
    int GW, g_qk;
};

Shape shape_of(const LlmDims &d, const LayerW &L) {
    Shape s{};
    attn_in_grid(d, L, s.GW, s.g_qk);
    s.np = pick_np(d.n_embd);
    s.tq = L.wq.type, s.tv = L.wv.type, s.to = L.wo.type;
    s.su = pick_su(std::max(max_wave_units(L.wq.rows + L.wk.rows, s.g_qk, s.np, 1),
                            max_wave_units(L.wv.rows, s.GW - s.g_qk, s.np, 1)),
                   s.np);
    s.suo = pick_su(max_wave_units(L.wo.rows, matvec_grid(d, L.wo.rows), pick_np(L.wo.k), 1), pick_np(L.wo.k));
    s.hd = d.hd, s.g = d.n_head / d.n_kv;
    if (pick_np(L.wo.k) != 1) s.suo = -1;
    return s;
}

template <bool DG>
bool launch(const LlmDims &d, const LayerW &L, _Float16 *kc, _Float16 *vc, const LlmBuffers &b, hipStream_t st,
            bool dry) {
    const Shape s = shape_of(d, L);
    const int rows = L.wq.rows + L.wk.rows + L.wv.rows;
    // the producer's per-head signal covers <= 64 rows per workgroup
    if ((L.wq.rows + L.wk.rows + s.g_qk - 1) / s.g_qk > 64 || (L.wv.rows + s.GW - s.g_qk - 1) / (s.GW - s.g_qk) > 64 ||
        d.n_kv > kQkvMax || rows != (d.n_head + 2 * d.n_kv) * d.hd || L.conv)
        return false;
    const int grid = s.GW + d.max_splits * d.n_kv + matvec_grid(d, L.wo.rows);
    const size_t lds = std::max(matvec_lds(d.n_embd), matvec_lds(L.wo.k));
    bool found = false;
#define MIO_LA_CASE(NP, TQ, TV, SU, HD, G, TO, SUO)                                                                   \
    if (!found && s.np == NP && s.tq == TQ && s.tv == TV && s.su == SU && s.hd == HD && s.g == G && s.to == TO &&   \
        s.suo == SUO) {                                                                                                \
        found = true;                                                                                                  \
        if (!dry)                                                                                                      \
            hipLaunchKernelGGL((k_layer_att<NP, TQ, TV, SU, HD, G, TO, SUO, DG>), dim3(grid), dim3(MT), lds, st, d,   \
                               L.attn_norm, L.wq, L.wk, L.wv, s.g_qk, s.GW, L.q_norm, L.k_norm, L.bqkv, kc, vc, L.wo, \
                               b);                                                                                     \
    }
    MIO_LAYER_ATT_SHAPES(MIO_LA_CASE)
#undef MIO_LA_CASE
    return found;
}

// the instantiated whole-layer shapes (attention shape as above, then the FFN's np, gate|up
// type, su, down np, down type, down su): 1.7B Q4_K_M (attn_v and ffn_down Q4_K or Q6_K)
#define MIO_LAYER_SHAPES(X)                             \
    X(1, 12, 12, 2, 128, 2, 12, 1, 1, 12, 6, 3, 12, 3) \
    X(1, 12, 14, 2, 128, 2, 12, 1, 1, 12, 6, 3, 14, 3) \
    X(1, 12, 12, 2, 128, 2, 12, 1, 1, 12, 6, 3, 14, 3) \
    X(1, 12, 14, 2, 128, 2, 12, 1, 1, 12, 6, 3, 12, 3)

template <bool DG>
bool launch_whole(const LlmDims &d, const LayerW &L, int il, _Float16 *kc, _Float16 *vc, const LlmBuffers &b,
                  hipStream_t st, bool dry) {
    const Shape s = shape_of(d, L);
    const int rows = L.wq.rows + L.wk.rows + L.wv.rows;
    if ((L.wq.rows + L.wk.rows + s.g_qk - 1) / s.g_qk > 64 || (L.wv.rows + s.GW - s.g_qk - 1) / (s.GW - s.g_qk) > 64 ||
        d.n_kv > kQkvMax || rows != (d.n_head + 2 * d.n_kv) * d.hd || L.conv || L.up.type != L.gate.type)
        return false;
    const int GI = matvec_grid(d, L.gate.rows), GD = matvec_grid(d, L.down.rows);
    const int fnp = pick_np(d.n_embd), fsu = pick_su(max_wave_units(L.gate.rows, GI, fnp, 2), fnp);
    const int fnpd = pick_np(L.down.k), fsud = pick_su(max_wave_units(L.down.rows, GD, fnpd, 1), fnpd);
    const int grid = s.GW + d.max_splits * d.n_kv + matvec_grid(d, L.wo.rows) + GI + GD;
    const size_t lds = std::max({matvec_lds(d.n_embd), matvec_lds(L.wo.k), matvec_lds(L.down.k)});
    LlmBuffers lb = b;
    int *base = b.att_cnt, *other = nullptr;
    if (!dry) lb.att_cnt = base + kLayOff + (il & 1) * kLaySet, other = base + kLayOff + ((il & 1) ^ 1) * kLaySet;
    const int fgate = layer_ffn_gate();
    bool found = false;
#define MIO_LY_CASE(NP, TQ, TV, SU, HD, G, TO, SUO, FNP, FT, FSU, FNPD, FTD, FSUD)                                  \
    if (!found && s.np == NP && s.tq == TQ && s.tv == TV && s.su == SU && s.hd == HD && s.g == G && s.to == TO &&   \
        s.suo == SUO && fnp == FNP && L.gate.type == FT && fsu == FSU && fnpd == FNPD && L.down.type == FTD &&      \
        fsud == FSUD) {                                                                                             \
        found = true;                                                                                               \
        if (!dry)                                                                                                   \
            hipLaunchKernelGGL((k_layer<NP, TQ, TV, SU, HD, G, TO, SUO, FNP, FT, FSU, FNPD, FTD, FSUD, DG>), dim3(grid), \
                               dim3(MT), lds, st, d, L.attn_norm, L.wq, L.wk, L.wv, s.g_qk, s.GW, L.q_norm, L.k_norm,   \
                               L.bqkv, kc, vc, L.wo, L.ffn_norm, L.gate, L.up, L.down, GI, GD, base, other, fgate, lb); \
    }
    MIO_LAYER_SHAPES(MIO_LY_CASE)
#undef MIO_LY_CASE
    return found;
}

}  // namespace

int layer_ffn_gate() {
    static const int v = [] {
        const char *e = getenv("MIO_LAYER_GATE");
        return e ? atoi(e) : 0;
    }();
    return v;
}

bool layer_fused_supported(const LlmDims &d, const LayerW &L) {
    return launch_whole<false>(d, L, 0, nullptr, nullptr, LlmBuffers{}, nullptr, true);
}

void launch_layer(const LlmDims &d, const LayerW &L, int il, _Float16 *kc, _Float16 *vc, const LlmBuffers &b, bool dg,
                  hipStream_t s) {
    if (dg)
        launch_whole<true>(d, L, il, kc, vc, b, s, false);
    else
        launch_whole<false>(d, L, il, kc, vc, b, s, false);
}

bool layer_att_supported(const LlmDims &d, const LayerW &L) {
    return launch<false>(d, L, nullptr, nullptr, LlmBuffers{}, nullptr, true);
}

void launch_layer_att(const LlmDims &d, const LayerW &L, _Float16 *kc, _Float16 *vc, const LlmBuffers &b, bool dg,
                      hipStream_t s) {
    if (dg)
        launch<true>(d, L, kc, vc, b, s, false);
    else
        launch<false>(d, L, kc, vc, b, s, false);
}
#else
bool layer_att_supported(const LlmDims &, const LayerW &) { return false; }
void launch_layer_att(const LlmDims &, const LayerW &, _Float16 *, _Float16 *, const LlmBuffers &, bool, hipStream_t) {}
int layer_ffn_gate() { return 0; }
bool layer_fused_supported(const LlmDims &, const LayerW &) { return false; }
void launch_layer(const LlmDims &, const LayerW &, int, _Float16 *, _Float16 *, const LlmBuffers &, bool, hipStream_t) {}
#endif

}  // namespace mio
