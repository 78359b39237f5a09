// First launch of a decoder layer in the single-token decode step (llama_decode for one
// token, test-to-speech.cpp:178-185 / :589-596): RMSNorm(x) -> q|k|v dequant-matvec.
//
// Matvec workgroups: q|k rows (type TQ) on the first g_qk workgroups, v rows (type TV) on the
// rest; each branch is WG-uniform and runs its own prologue, so neither path merges load
// counts. FS (layer 0 only): the previous step's sampler runs here when st->pending. Every
// workgroup reduces the lm_head partials to the same token and dequantizes its embedding
// row into its x registers while its first weight group is in flight; workgroup 0 also
// stores x (attn_out's residual) and the token / token ring / EOS flag. pos and step are
// advanced by layer 0's ffn_in (no kernel before it writes a StepState field it reads).
#include "llm_device.h"

#pragma clang fp contract(off)

namespace mio {
namespace {

template <int NP, int TQ, int TV, int SU, bool DG, bool FS>
__global__ __launch_bounds__(MT) void k_attn_in(LlmDims d, const float *norm_w, QMat wq, QMat wk, QMat wv,
                                                int g_qk, LlmBuffers b, QMat emb, int nblk) {
    constexpr bool kDiag = DG;
    const int o1 = wq.rows, o2 = wq.rows + wk.rows;
    const int GW = matvec_grid_n(d.n_wg, o2 + wv.rows);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float rs_[MW];
    __shared__ int ri_[MW];
    const int K = d.n_embd;
    const Smem s = carve(smem, K);
    MIO_TRACE(b, 0);
    MIO_TL_BEGIN(b);
    if (blockIdx.x == 2 && MIO_TIDX < 2 * kFfnShards)  // the previous k_ffn's h counters (kernel boundary ordered)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(b.att_cnt + kFfnOff + kFfnStride * MIO_TIDX), 0,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int pend = 0, step = 0;
    if constexpr (FS) {
        // after an end token every decode launch returns at entry (test-to-speech.cpp:168-170
        // breaks before the next llama_decode); layer 0 reads the flag with pending / step
        pend = b.st->pending;
        step = b.st->step;
        if (b.st->done) return;
    }
    uint32_t dn = 0;
    if constexpr (!FS) dn = done_issue(b);
    XRegs<NP> xr;
    load_x(pend ? nullptr : b.x, norm_w, K, xr);
    x_gate();
    // returns true when the sampled token ends generation (the rest of the step is skipped)
    auto sample_prologue = [&]() -> bool {
        if constexpr (FS) {
            if (pend) {
                const SampleCfg sc = *b.cfg;
                const int tok = sample_token<MT>(b.smp, nblk, sc, step, rs_, ri_);
                embed_regs(emb, tok, K, xr);
                if (blockIdx.x == 0) {
#pragma unroll
                    for (int i = 0; i < NP; ++i) {
                        const int e = (MIO_TIDX + i * MT) * 4;
                        if (e < K) *reinterpret_cast<float4 *>(b.x + e) = xr.v[i];
                    }
                    if (MIO_TIDX == 0) {
                        if (step < sc.max_steps) sc.out_tokens[step] = tok;
                        if (tok == sc.eos0 || tok == sc.eos1) b.st->done = 1, signal_host_done(sc);
                        b.st->token = tok;
                    }
                }
                return tok == sc.eos0 || tok == sc.eos1;
            }
        }
        return false;
    };
    auto put = [&](int row, float v) {
        if ((threadIdx.x & 63) == 0) b.qkv[row] = v;
    };
    Frag ga[Cfg<NP, SU>::U], gb[Cfg<NP, SU>::U];
    int lo, hi;
    if ((int)blockIdx.x < g_qk) {
        wave_range(o2, lo, hi, blockIdx.x, g_qk);
        load_first<TQ, NP, 1, SU, MIO_SMALL_AUX>(wq, wk, lo, hi, ga, gb, o1);
        if (sample_prologue()) return;
        x_after_weights(xr);
        if (!FS && done_now(dn)) return;
        MIO_TRACE(b, 1);
        MIO_TL_MARK1(b);
        rmsnorm_quant(xr, K, d.eps, akind(TQ), s, MIO_TL_DIAGSLOT(b));
        MIO_TRACE(b, 2);
        MIO_TL_MARK(b, 2);
        stream_rows<TQ, NP, 1, SU, MIO_SMALL_AUX>(wq, wk, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
            put(row, v);
        }, o1);
        MIO_TL_END(b);
        MIO_TRACE(b, 15);
    } else {
        const int bv = (int)blockIdx.x - g_qk, gv = GW - g_qk;
        wave_range(wv.rows, lo, hi, bv, gv);
        load_first<TV, NP, 1, SU, MIO_SMALL_AUX>(wv, wv, lo, hi, ga, gb);
        if (sample_prologue()) return;
        x_after_weights(xr);
        if (!FS && done_now(dn)) return;
        rmsnorm_quant(xr, K, d.eps, akind(TV), s, MIO_TL_DIAGSLOT(b));
        stream_rows<TV, NP, 1, SU, MIO_SMALL_AUX>(wv, wv, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
            put(o2 + row, v);
        });
        MIO_TL_END(b);
    }
}

template <bool DG>
void launch(const LlmDims &d, const LayerW &L, int il, const QMat &tok_embd, const LlmBuffers &b, hipStream_t s) {
    int GW, g_qk;
    attn_in_grid(d, L, GW, g_qk);
    const size_t lds = matvec_lds(d.n_embd);
    const int np = pick_np(d.n_embd);
    const int un = std::max(max_wave_units(L.wq.rows + L.wk.rows, g_qk, np, 1),
                            max_wave_units(L.wv.rows, GW - g_qk, np, 1));
    const int nblk = lm_head_blocks(d);
    const int grid = GW;
    dispatch_nt(d.n_embd, L.wq.type, [&]<int NP, int TQ>() {
        auto go = [&]<int TV>() {
            dispatch_su<NP>(pick_su(un, NP), [&]<int SU>() {
                if (il == 0)
                    hipLaunchKernelGGL((k_attn_in<NP, TQ, TV, SU, DG, true>), dim3(grid), dim3(MT), lds, s, d,
                                       L.attn_norm, L.wq, L.wk, L.wv, g_qk, b, tok_embd, nblk);
                else
                    hipLaunchKernelGGL((k_attn_in<NP, TQ, TV, SU, DG, false>), dim3(grid), dim3(MT), lds, s, d,
                                       L.attn_norm, L.wq, L.wk, L.wv, g_qk, b, tok_embd, nblk);
            });
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
}

}  // namespace

void launch_attn_in(const LlmDims &d, const LayerW &L, int il, const QMat &tok_embd, const LlmBuffers &b, bool dg,
                    hipStream_t s) {
    if (dg)
        launch<true>(d, L, il, tok_embd, b, s);
    else
        launch<false>(d, L, il, tok_embd, b, s);
}

}  // namespace mio
