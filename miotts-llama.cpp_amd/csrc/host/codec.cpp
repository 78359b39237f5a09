// MioCodec decoder on one MI355X (replaces miocodec_load / miocodec_decode,
// miocodec.cpp:426-810).
//
// Differences in *mechanism* from the reference (numerics are the same functions):
//  * weights are read from the GGUF once and uploaded once at load, re-laid-out for the
//    kernels (fused q|k|v, gate/up interleaved per 16 rows, ConvT taps as GEMM panels,
//    conv kernels pre-rounded to f16 as ggml_cast does), instead of a graph rebuild +
//    full weight memcpy on every call (miocodec.cpp:558-782);
//  * the local attention mask is a band (|i-j| <= window/2) instead of a dense S x S
//    -inf tensor (miocodec.cpp:233-242);
//  * activations stay in [rows][channels] layout, so the reference's transposes
//    (:623, :638, :663, :712) and the host interleave (:801-808) disappear: the head
//    GEMM writes the [frame][bin][re,im] spectrogram directly, and decode_pcm feeds it
//    to the fused iSTFT without leaving the GPU.
#include <cmath>
#include <cstring>
#include <initializer_list>
#include <string>
#include <vector>

#include "codec_kernels.h"
#include "common.h"
#include "gguf.h"

int mio_istft_launch_device(mio_hip_istft *h, const float *d_spec, int n_frames, int hop,
                            float *d_out, hipStream_t s);

namespace {

struct ResW {
    float *gn1_w, *gn1_b, *gn2_w, *gn2_b, *b1, *b2;
    _Float16 *w1, *w2;
};
// h16_*: the matrix came from an F16 GGUF tensor, so its GEMM rounds the activation to f16
// (GemmArgs::a_f16; ggml mul_mat's F16 vec_dot_type)
struct PreW {
    float *ln1_w, *ln1_b, *ln2_w, *ln2_b, *qkv, *wo, *gu, *wd;
    int h16_qkv, h16_wo, h16_gu, h16_wd;
};
struct DecW {
    float *qkv, *wo, *gu, *wd;
    int h16_qkv, h16_wo, h16_gu, h16_wd;
};
struct UpW {
    float *w, *b, *alpha_e, *beta_e;
    int f, K, taps, trim, Cin, Cout;
    int h16;
    ResW res;
};

}  // namespace

struct mio_hip_codec {
    mio_hip_device *d = nullptr;
    // hyper-parameters (miocodec.cpp:58-89 defaults, read at :448-474)
    int sample_rate = 44100, n_fft = 392, hop = 98, n_freq = 197, spt = 1764, head_out = 394;
    int pre_layers = 6, pre_dim = 768, pre_heads = 12, pre_ff = 2048, pre_win = 65;
    int dec_layers = 8, dec_dim = 512, dec_heads = 8, dec_ff = 1536, dec_win = 65, adaln = 128;
    int res_blocks = 2, groups = 32, up_stages = 2;
    float theta = 10000.f, eps = 1e-5f, gn_eps = 1e-6f;
    int n_codes = 0, nfp = 0;

    float *tok = nullptr;
    std::vector<PreW> pre;
    float *pre_norm_w = nullptr, *pre_norm_b = nullptr, *pre_out_w = nullptr, *pre_out_b = nullptr;
    float *ups_w = nullptr, *ups_b = nullptr;
    int h16_pre_out = 0, h16_ups = 0, h16_cond = 0, h16_op = 0, h16_head = 0;
    std::vector<ResW> prior, post;
    std::vector<DecW> dec;
    float *cond_w = nullptr, *cond_b = nullptr;
    int cond_rows = 0;
    std::vector<UpW> ups;
    float *op_w = nullptr, *op_b = nullptr, *op_ae = nullptr, *op_be = nullptr;
    float *head_w = nullptr, *head_b = nullptr;
    int c_last = 0;

    float2 *rope = nullptr;
    int rope_cap = 0;
    char *ws = nullptr;
    size_t ws_cap = 0;
    // mio_hip_codec_decode_pcm_batch: lane k >= 1 decodes on stream xs[k - 1] in workspace
    // xws[k - 1] (lane 0: the caller's stream and ws), joined through xev
    std::vector<hipStream_t> xs;
    std::vector<hipEvent_t> xev;
    std::vector<char *> xws;
    std::vector<size_t> xws_cap;
    mio_hip_istft *ist = nullptr;
    std::vector<void *> allocs;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    float last_ms[2] = {0, 0};
    bool timed = false;
    // streaming prenet cache (MIO_CODEC_INCREMENTAL): prenet + projection rows [0, pc_exact)
    // of the previous incremental decode, whose ±pre_layers*(pre_win/2) receptive field lay
    // inside that decode (so they equal the full-context rows), and that decode's codes
    float *pc = nullptr;
    int pc_cap = 0, pc_exact = 0;
    std::vector<int32_t> pc_codes;
    int pc_last_reused = 0;  // rows the last decode took from the cache (diagnostic)
    double last_flops = 0.0;  // algorithmic FLOPs of the last decode_pcm (codec_roofline)

    ~mio_hip_codec() {
        if (d) hipSetDevice(d->dev);
        for (void *p : allocs) hipFree(p);
        if (rope) hipFree(rope);
        if (ws) hipFree(ws);
        for (char *p : xws)
            if (p) hipFree(p);
        for (auto e : xev) hipEventDestroy(e);
        for (auto q : xs) hipStreamDestroy(q);
        if (pc) hipFree(pc);
        if (ist) mio_hip_istft_destroy(ist);
        for (auto e : ev)
            if (e) hipEventDestroy(e);
    }
};

namespace {

// Algorithmic FLOPs of the decode being issued (2 per multiply-add of every GEMM, conv and
// banded-attention dot product), read back by mio_hip_codec_last_flops for bench.py's
// codec_roofline. Counted at issue, so an incremental re-decode counts only what it runs.
thread_local double t_flops = 0.0;
void gemm_launch(const mio::GemmArgs &a, int epi, hipStream_t s) {
    t_flops += 2.0 * a.M * a.N * a.K;
    mio::launch_gemm_f32(a, epi, s);
}
void conv_launch(const mio::ConvArgs &a, hipStream_t s) {
    t_flops += 2.0 * a.L * a.Cout * a.taps * a.Cin;
    mio::launch_conv_f16(a, s);
}
void band_launch(const float *qkv, float *out, int S, int H, int win, const float2 *rope, hipStream_t s) {
    const int h = win / 2;
    double pairs = 0;
    for (int i = 0; i < S; ++i) pairs += std::min(S - 1, i + h) - std::max(0, i - h) + 1;
    t_flops += 4.0 * pairs * H * 64;  // q.k and p.v over the band, head dim 64
    mio::launch_band_attention(qkv, out, S, H, win, rope, s);
}
void cond_launch(const float *W, const float *b, const float *e, int R, int A, float *y, int e_f16, hipStream_t s) {
    t_flops += 2.0 * R * A;
    mio::launch_cond_gemv(W, b, e, R, A, y, e_f16, s);
}

struct Loader {
    mio_hip_codec *c;
    const mio::GgufFile &g;
    bool ok = true;

    std::vector<float> f32(const std::string &name, size_t expect) {
        const mio::GgufTensor *t = g.tensor(name);
        std::vector<float> v;
        if (!t) {
            if (ok) mio::set_error("miocodec: missing tensor: %s", name.c_str());
            ok = false;
            return v;
        }
        const size_t n = (size_t)t->nelements();
        if (expect && n != expect) {
            if (ok) mio::set_error("miocodec: tensor %s has %zu elements, expected %zu", name.c_str(), n, expect);
            ok = false;
            return v;
        }
        v.resize(n);
        if (t->type == mio::GGML_F32) {
            std::memcpy(v.data(), t->data, n * 4);
        } else if (t->type == mio::GGML_F16) {
            const _Float16 *h = (const _Float16 *)t->data;
            for (size_t i = 0; i < n; ++i) v[i] = (float)h[i];
        } else {
            if (ok) mio::set_error("miocodec: tensor %s type %s unsupported", name.c_str(), mio::ggml_type_name(t->type));
            ok = false;
        }
        return v;
    }
    template <class T>
    T *up(const std::vector<T> &v) {
        if (!ok || v.empty()) return nullptr;
        void *p = nullptr;
        if (hipMalloc(&p, v.size() * sizeof(T)) != hipSuccess) {
            mio::set_error("miocodec: hipMalloc failed");
            ok = false;
            return nullptr;
        }
        c->allocs.push_back(p);
        if (hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) {
            mio::set_error("miocodec: upload failed");
            ok = false;
        }
        return (T *)p;
    }
    float *vec(const std::string &name, size_t n) { return up(f32(name, n)); }
    // 1 when every named tensor is F16, 0 when none is; a mix (one GEMM can round its
    // activation one way only) is refused
    int f16(std::initializer_list<std::string> names) {
        int n16 = 0, n = 0;
        for (const std::string &nm : names) {
            const mio::GgufTensor *t = g.tensor(nm);
            n += t != nullptr;
            n16 += t && t->type == mio::GGML_F16;
        }
        if (n16 && n16 != n) {
            if (ok) mio::set_error("miocodec: %s and the matrices fused with it mix F16 and F32", names.begin()->c_str());
            ok = false;
        }
        return n16 ? 1 : 0;
    }
    // exp of a (log-scale) snake parameter; ggml_exp of an F16 tensor stays F16
    std::vector<float> snake_exp(const std::string &name, size_t n) {
        std::vector<float> v = f32(name, n);
        const bool h = f16({name});
        for (auto &x : v) x = h ? (float)(_Float16)expf(x) : expf(x);
        return v;
    }

    // conv1d kernel ggml [K][Cin][Cout] (mem [co][ci][k]) -> f16 [co][k*Cin + ci]
    _Float16 *conv_w(const std::string &name, int K, int Cin, int Cout) {
        std::vector<float> w = f32(name, (size_t)K * Cin * Cout);
        if (!ok) return nullptr;
        std::vector<_Float16> o((size_t)Cout * K * Cin);
        for (int co = 0; co < Cout; ++co)
            for (int ci = 0; ci < Cin; ++ci)
                for (int k = 0; k < K; ++k)
                    o[(size_t)co * K * Cin + (size_t)k * Cin + ci] = (_Float16)w[((size_t)co * Cin + ci) * K + k];
        return up(o);
    }
    ResW resnet(const std::string &p, int ch) {
        ResW r{};
        r.gn1_w = vec(p + "norm1.weight", ch);
        r.gn1_b = vec(p + "norm1.bias", ch);
        r.w1 = conv_w(p + "conv1.weight", 3, ch, ch);
        r.b1 = vec(p + "conv1.bias", ch);
        r.gn2_w = vec(p + "norm2.weight", ch);
        r.gn2_b = vec(p + "norm2.bias", ch);
        r.w2 = conv_w(p + "conv2.weight", 3, ch, ch);
        r.b2 = vec(p + "conv2.bias", ch);
        return r;
    }
    // gate/up -> rows interleaved per 16 (EPI_SWIGLU pairs lane l with l^16)
    float *gate_up(const std::string &gname, const std::string &uname, int in, int ff) {
        std::vector<float> g = f32(gname, (size_t)in * ff), u = f32(uname, (size_t)in * ff);
        if (!ok) return nullptr;
        std::vector<float> o((size_t)2 * ff * in);
        for (int p = 0; p < ff / 16; ++p)
            for (int r = 0; r < 16; ++r) {
                std::memcpy(&o[((size_t)32 * p + r) * in], &g[((size_t)16 * p + r) * in], in * 4);
                std::memcpy(&o[((size_t)32 * p + 16 + r) * in], &u[((size_t)16 * p + r) * in], in * 4);
            }
        return up(o);
    }
    float *qkv(const std::string &p, int D) {
        std::vector<float> q = f32(p + "attn_q.weight", (size_t)D * D), k = f32(p + "attn_k.weight", (size_t)D * D),
                           v = f32(p + "attn_v.weight", (size_t)D * D);
        if (!ok) return nullptr;
        std::vector<float> o;
        o.reserve((size_t)3 * D * D);
        o.insert(o.end(), q.begin(), q.end());
        o.insert(o.end(), k.begin(), k.end());
        o.insert(o.end(), v.begin(), v.end());
        return up(o);
    }
};

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ggml rope cache for mode 0 (test: ggml_rope_cache_init): theta = p, *= theta_scale per pair
std::vector<float2> rope_table(int S, int hd, float base) {
    std::vector<float2> t((size_t)S * (hd / 2));
    const float theta_scale = powf(base, -2.0f / hd);
    for (int p = 0; p < S; ++p) {
        float theta = (float)p;
        for (int i = 0; i < hd / 2; ++i) {
            t[(size_t)p * (hd / 2) + i] = make_float2(cosf(theta), sinf(theta));
            theta *= theta_scale;
        }
    }
    return t;
}

struct Ws {
    int T = 0, S = 0;
    float *xT, *hT, *qkvT, *aT, *fT, *yT;
    float *xS, *hS, *qkvS, *aS, *fS;
    std::vector<float *> u, t;
    std::vector<int> uL;
    float *op, *spec, *pcm, *cond, *emb;
    mio::GnScratch gns;
    _Float16 *xa;
    int *codes;
    int Lf;
};

int plan_ws(mio_hip_codec *c, int T, Ws &w, bool alloc, size_t *bytes = nullptr, int lane = 0) {
    char *&ws = lane ? c->xws[lane - 1] : c->ws;
    size_t &ws_cap = lane ? c->xws_cap[lane - 1] : c->ws_cap;
    const int S = 2 * T;
    size_t off = 0;
    std::vector<size_t> sizes;
    auto take = [&](size_t nfloats) {
        size_t o = off;
        off = align_up(off + nfloats * 4, 256);
        return o;
    };
    struct Slot { float **p; size_t o; };
    std::vector<std::pair<float **, size_t>> slots;
    auto F = [&](float **p, size_t n) { slots.push_back({p, take(n)}); };
    F(&w.xT, (size_t)T * c->pre_dim);
    F(&w.hT, (size_t)T * c->pre_dim);
    F(&w.qkvT, (size_t)T * 3 * c->pre_dim);
    F(&w.aT, (size_t)T * c->pre_dim);
    F(&w.fT, (size_t)T * c->pre_ff);
    F(&w.yT, (size_t)T * c->dec_dim);
    F(&w.xS, (size_t)S * c->dec_dim);
    F(&w.hS, (size_t)S * c->dec_dim);
    F(&w.qkvS, (size_t)S * 3 * c->dec_dim);
    F(&w.aS, (size_t)S * c->dec_dim);
    F(&w.fS, (size_t)S * c->dec_ff);
    w.u.assign(c->up_stages, nullptr);
    w.t.assign(c->up_stages, nullptr);
    w.uL.assign(c->up_stages, 0);
    int L = S;
    for (int s = 0; s < c->up_stages; ++s) {
        const UpW &u = c->ups[s];
        L = (L - 1) * u.f + u.K - 2 * u.trim;
        w.uL[s] = L;
        F(&w.u[s], (size_t)L * u.Cout);
        F(&w.t[s], (size_t)L * u.Cout);
    }
    w.Lf = L;
    F(&w.op, (size_t)L * c->dec_dim);
    F(&w.spec, (size_t)L * 2 * c->n_freq);
    F(&w.pcm, (size_t)L * c->hop + c->n_fft);
    // GroupNorm slice partials (doubles) and the f16 conv operand of the widest ResNet
    size_t xa_n = (size_t)S * c->dec_dim;
    for (int st = 0; st < c->up_stages; ++st) xa_n = std::max(xa_n, (size_t)w.uL[st] * c->ups[st].Cout);
    float *gnp_f = nullptr, *gns_f = nullptr, *xa_f = nullptr;
    F(&gnp_f, (size_t)mio::kGnPartDoubles * 2);
    F(&gns_f, 2 * 64);
    F(&xa_f, (xa_n + 1) / 2);
    F(&w.cond, (size_t)c->cond_rows);
    F(&w.emb, (size_t)c->adaln);
    float *codes_f = nullptr;
    F(&codes_f, (size_t)T);
    if (bytes) *bytes = off;
    if (alloc && off > ws_cap) {
        // sized for at least 1024 codes: streaming re-decodes grow T every call, and each
        // re-allocation (hipFree) would wait for whatever else runs on the device
        size_t want = off;
        if (T < 1024) {
            Ws big;
            plan_ws(c, 1024, big, false, &want);
        }
        if (ws) hipFree(ws);
        ws = nullptr;
        ws_cap = 0;
        if (hipMalloc(&ws, want) != hipSuccess) {
            mio::set_error("miocodec: workspace of %zu bytes failed", want);
            return MIO_ERR_OOM;
        }
        ws_cap = want;
    }
    for (auto &s : slots) *s.first = (float *)(ws + s.second);
    w.codes = (int *)codes_f;
    w.gns.part = (double *)gnp_f;
    w.gns.stat = (float2 *)gns_f;
    w.xa = (_Float16 *)xa_f;
    w.T = T;
    w.S = S;
    if (alloc && S > c->rope_cap) {
        if (c->rope) hipFree(c->rope);
        c->rope = nullptr;
        const int cap = S < 4096 ? 4096 : S;
        std::vector<float2> r = rope_table(cap, 64, c->theta);
        MIO_HIP_CHECK(hipMalloc(&c->rope, r.size() * sizeof(float2)));
        MIO_HIP_CHECK(hipMemcpy(c->rope, r.data(), r.size() * sizeof(float2), hipMemcpyHostToDevice));
        c->rope_cap = cap;
    }
    return MIO_OK;
}

mio::GemmArgs gemm(const float *A, int K, int M, const float *B, int N, float *C, int ldc, int a_f16 = 0) {
    mio::GemmArgs g{};
    g.a_f16 = a_f16;
    g.A = A;
    g.a_seg = K;
    g.a_row_off = 0;
    g.a_rows = M;
    g.B = B;
    g.M = M;
    g.N = N;
    g.K = K;
    g.C = C;
    g.ldc = ldc;
    return g;
}

void resnet(mio_hip_codec *c, const ResW &r, float *x, float *t, int L, int C, const Ws &w,
            hipStream_t s) {
    mio::ConvArgs a{};
    a.L = L, a.Cin = C, a.taps = 3, a.pad = 1, a.Cout = C, a.Xa = w.xa;
    // t = conv1(silu(GN1(x))) + b1
    mio::launch_groupnorm_apply(x, L, C, c->groups, c->gn_eps, r.gn1_w, r.gn1_b, w.gns, w.xa, s);
    a.B = r.w1, a.bias = r.b1, a.Y = t, a.resid = nullptr;
    conv_launch(a, s);
    // x = conv2(silu(GN2(t))) + b2 + x
    mio::launch_groupnorm_apply(t, L, C, c->groups, c->gn_eps, r.gn2_w, r.gn2_b, w.gns, w.xa, s);
    a.B = r.w2, a.bias = r.b2, a.Y = x, a.resid = x;
    conv_launch(a, s);
}

// Prenet receptive field in codes: each layer's banded attention reaches pre_win/2 each way.
int prenet_radius(const mio_hip_codec *c) { return c->pre_layers * (c->pre_win / 2); }

// Runs the decoder; if stop_stage >= 0, returns after that stage with *stage_buf/rows/cols set.
// cached > 0: rows [0, cached) of the prenet output are taken from c->pc; the prenet then runs
// only over codes [cached - radius, T) (RoPE at absolute positions), whose rows from `cached`
// on have their whole receptive field inside that window.
int run_decode(mio_hip_codec *c, Ws &w, hipStream_t s, int stop_stage, const float **stage_buf,
               int *rows, int *cols, int cached = 0) {
    const int T = w.T, S = w.S, Dp = c->pre_dim, Dd = c->dec_dim;
    const int s0 = cached > 0 ? std::max(0, cached - prenet_radius(c)) : 0, Tw = T - s0;
    const float2 *rope_w = c->rope + (size_t)s0 * 32;  // [pos][hd/2], hd = 64
    int stage = 0;
    auto done = [&](const float *buf, int r, int cc) {
        if (stage == stop_stage) {
            *stage_buf = buf, *rows = r, *cols = cc;
            return true;
        }
        ++stage;
        return false;
    };
    // 1. embedding (:599-600) of codes [s0, T)
    mio::launch_embed(c->tok, w.codes + s0, Tw, Dp, w.xT, s);
    if (done(w.xT, Tw, Dp)) return MIO_OK;
    // 2. prenet (:604-618) over the window's Tw rows
    for (int i = 0; i < c->pre_layers; ++i) {
        const PreW &p = c->pre[i];
        mio::launch_rownorm(w.xT, w.hT, Tw, Dp, c->eps, 1, p.ln1_w, p.ln1_b, s);
        gemm_launch(gemm(w.hT, Dp, Tw, p.qkv, 3 * Dp, w.qkvT, 3 * Dp, p.h16_qkv), mio::EPI_STORE, s);
        band_launch(w.qkvT, w.aT, Tw, c->pre_heads, c->pre_win, rope_w, s);
        gemm_launch(gemm(w.aT, Dp, Tw, p.wo, Dp, w.xT, Dp, p.h16_wo), mio::EPI_RESID, s);
        mio::launch_rownorm(w.xT, w.hT, Tw, Dp, c->eps, 1, p.ln2_w, p.ln2_b, s);
        gemm_launch(gemm(w.hT, Dp, Tw, p.gu, 2 * c->pre_ff, w.fT, c->pre_ff, p.h16_gu), mio::EPI_SWIGLU, s);
        gemm_launch(gemm(w.fT, c->pre_ff, Tw, p.wd, Dp, w.xT, Dp, p.h16_wd), mio::EPI_RESID, s);
    }
    mio::launch_rownorm(w.xT, w.hT, Tw, Dp, c->eps, 1, c->pre_norm_w, c->pre_norm_b, s);
    {
        mio::GemmArgs g = gemm(w.hT, Dp, Tw, c->pre_out_w, Dd, w.yT + (size_t)s0 * Dd, Dd, c->h16_pre_out);
        g.bias = c->pre_out_b;
        gemm_launch(g, mio::EPI_STORE, s);
    }
    // the cached rows replace the window's left edge (whose context was cut)
    if (cached > 0)
        MIO_HIP_CHECK(hipMemcpyAsync(w.yT, c->pc, (size_t)cached * Dd * 4, hipMemcpyDeviceToDevice, s));
    if (done(w.yT, T, Dd)) return MIO_OK;
    // 3. wave_upsample ConvT k=2 s=2 (:622-626): one GEMM, N = 2*Dd, remapped rows
    {
        mio::GemmArgs g = gemm(w.yT, Dd, T, c->ups_w, 2 * Dd, w.xS, Dd, c->h16_ups);
        g.bias = c->ups_b, g.f = 2, g.trim = 0, g.cout = Dd, g.rows_out = S;
        gemm_launch(g, mio::EPI_CONVT, s);
    }
    if (done(w.xS, S, Dd)) return MIO_OK;
    // 4. wave_prior (:629-637)
    for (auto &r : c->prior) resnet(c, r, w.xS, w.hS, S, Dd, w, s);
    if (done(w.xS, S, Dd)) return MIO_OK;
    // 5. AdaLN-Zero decoder (:640-660); all conditioning vectors in one GEMV
    cond_launch(c->cond_w, c->cond_b, w.emb, c->cond_rows, c->adaln, w.cond, c->h16_cond, s);
    for (int i = 0; i < c->dec_layers; ++i) {
        const DecW &p = c->dec[i];
        const float *ca = w.cond + (size_t)i * 6 * Dd, *cf = ca + 3 * Dd;
        mio::launch_rownorm(w.xS, w.hS, S, Dd, c->eps, 2, ca, ca + Dd, s);
        gemm_launch(gemm(w.hS, Dd, S, p.qkv, 3 * Dd, w.qkvS, 3 * Dd, p.h16_qkv), mio::EPI_STORE, s);
        band_launch(w.qkvS, w.aS, S, c->dec_heads, c->dec_win, c->rope, s);
        {
            mio::GemmArgs g = gemm(w.aS, Dd, S, p.wo, Dd, w.xS, Dd, p.h16_wo);
            g.aux = ca + 2 * Dd;
            gemm_launch(g, mio::EPI_GATED, s);
        }
        mio::launch_rownorm(w.xS, w.hS, S, Dd, c->eps, 2, cf, cf + Dd, s);
        gemm_launch(gemm(w.hS, Dd, S, p.gu, 2 * c->dec_ff, w.fS, c->dec_ff, p.h16_gu), mio::EPI_SWIGLU, s);
        {
            mio::GemmArgs g = gemm(w.fS, c->dec_ff, S, p.wd, Dd, w.xS, Dd, p.h16_wd);
            g.aux = cf + 2 * Dd;
            gemm_launch(g, mio::EPI_GATED, s);
        }
    }
    {
        const float *nc = w.cond + (size_t)c->dec_layers * 6 * Dd;
        mio::launch_rownorm(w.xS, w.xS, S, Dd, c->eps, 2, nc, nc + Dd, s);
    }
    if (done(w.xS, S, Dd)) return MIO_OK;
    // 6. wave_post (:663-672)
    for (auto &r : c->post) resnet(c, r, w.xS, w.hS, S, Dd, w, s);
    if (done(w.xS, S, Dd)) return MIO_OK;
    // 7. upsampler stages (:677-708): ConvT(+trim)+Snake as one tap-window GEMM, then ResNet
    const float *src = w.xS;
    int Lin = S;
    for (int st = 0; st < c->up_stages; ++st) {
        const UpW &u = c->ups[st];
        const int Lout = w.uL[st];
        const int M = (Lout - 1 + u.trim) / u.f + 1;
        mio::GemmArgs g{};
        g.A = src, g.a_seg = u.Cin, g.a_row_off = -(u.taps - 1), g.a_rows = Lin;
        g.B = u.w, g.M = M, g.N = u.f * u.Cout, g.K = u.taps * u.Cin;
        g.C = w.u[st], g.ldc = u.Cout, g.bias = u.b, g.aux = u.alpha_e, g.aux2 = u.beta_e;
        g.f = u.f, g.trim = u.trim, g.cout = u.Cout, g.rows_out = Lout, g.a_f16 = u.h16;
        gemm_launch(g, mio::EPI_CONVT_SNAKE, s);
        resnet(c, u.res, w.u[st], w.t[st], Lout, u.Cout, w, s);
        src = w.u[st];
        Lin = Lout;
        if (done(w.u[st], Lout, u.Cout)) return MIO_OK;
    }
    const int L = Lin;
    // 8. out_proj + out_snake (:711-725)
    {
        mio::GemmArgs g = gemm(src, c->c_last, L, c->op_w, Dd, w.op, Dd, c->h16_op);
        g.bias = c->op_b, g.aux = c->op_ae, g.aux2 = c->op_be;
        gemm_launch(g, mio::EPI_SNAKE, s);
    }
    if (done(w.op, L, Dd)) return MIO_OK;
    // 9. iSTFT head (:728-737) written as [frame][bin][re,im] (:801-808)
    {
        mio::GemmArgs g = gemm(w.op, Dd, L, c->head_w, 2 * c->nfp, w.spec, 2 * c->n_freq, c->h16_head);
        g.bias = c->head_b, g.cout = c->n_freq;
        gemm_launch(g, mio::EPI_HEAD, s);
    }
    if (done(w.spec, L, 2 * c->n_freq)) return MIO_OK;
    return MIO_OK;
}

int prepare_inputs(mio_hip_codec *c, Ws &w, const int32_t *codes, int n, const float *emb,
                   unsigned flags, hipStream_t s) {
    if (flags & MIO_IN_DEVICE) {
        MIO_HIP_CHECK(hipMemcpyAsync(w.codes, codes, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        MIO_HIP_CHECK(hipMemcpyAsync(w.emb, emb, (size_t)c->adaln * 4, hipMemcpyDeviceToDevice, s));
    } else {
        for (int i = 0; i < n; ++i)
            MIO_REQUIRE(codes[i] >= 0 && codes[i] < c->n_codes, MIO_ERR_INVALID,
                        "miocodec: code %d at %d outside [0, %d)", codes[i], i, c->n_codes);
        MIO_HIP_CHECK(hipMemcpyAsync(w.codes, codes, (size_t)n * 4, hipMemcpyHostToDevice, s));
        MIO_HIP_CHECK(hipMemcpyAsync(w.emb, emb, (size_t)c->adaln * 4, hipMemcpyHostToDevice, s));
    }
    return MIO_OK;
}

}  // namespace

extern "C" int mio_hip_codec_load(mio_hip_device *d, const char *path, mio_hip_codec **out) {
    MIO_REQUIRE(d && path && out, MIO_ERR_INVALID, "codec_load: null argument");
    int rc = mio::bind(d);
    if (rc) return rc;
    mio::GgufFile g;
    if (!g.open(path)) return MIO_ERR_IO;
    auto *c = new mio_hip_codec();
    c->d = d;
    auto U = [&](const char *k, int def) { return (int)g.get_int(k, def); };
    c->sample_rate = U("miocodec.sample_rate", 44100);
    c->n_fft = U("miocodec.n_fft", 392);
    c->hop = U("miocodec.hop_length", 98);
    c->n_freq = c->n_fft / 2 + 1;
    c->spt = U("miocodec.samples_per_token", 1764);
    c->head_out = U("embedding_length_out", 394);
    c->pre_layers = U("miocodec.prenet_layers", 6);
    c->pre_dim = U("miocodec.prenet_dim", 768);
    c->pre_heads = U("miocodec.prenet_heads", 12);
    c->pre_ff = U("miocodec.prenet_ff", 2048);
    c->pre_win = U("miocodec.prenet_window", 65);
    c->dec_layers = U("miocodec.decoder_layers", 8);
    c->dec_dim = U("miocodec.decoder_dim", 512);
    c->dec_heads = U("miocodec.decoder_heads", 8);
    c->dec_ff = U("miocodec.decoder_ff", 1536);
    c->dec_win = U("miocodec.decoder_window", 65);
    c->adaln = U("miocodec.decoder_adanorm_dim", 128);
    c->res_blocks = U("miocodec.resnet_blocks", 2);
    c->groups = U("miocodec.resnet_groups", 32);
    c->up_stages = U("miocodec.wave_upsampler_layers", 2);
    c->theta = (float)g.get_float("miocodec.rope_theta", 10000.0);
    c->eps = (float)g.get_float("miocodec.norm_eps", 1e-5);
    c->gn_eps = (float)g.get_float("miocodec.group_norm_eps", 1e-6);
    auto fail = [&](int code) {
        delete c;
        return code;
    };
    // shapes this implementation supports (all MioCodec checkpoints: head_dim 64, window 65)
    if (c->pre_dim % c->pre_heads || c->pre_dim / c->pre_heads != 64 || c->dec_dim % c->dec_heads ||
        c->dec_dim / c->dec_heads != 64 || c->pre_win / 2 > 32 || c->dec_win / 2 > 32 ||
        c->pre_dim % 64 || c->dec_dim % 64 || c->pre_dim > 1024 || c->dec_dim > 1024 || c->pre_ff % 16 || c->dec_ff % 16 || c->groups > 64 ||
        c->head_out != 2 * c->n_freq || c->up_stages < 0 || c->up_stages > 4) {
        mio::set_error("miocodec: unsupported hyper-parameters (head_dim must be 64, window <= 65)");
        return fail(MIO_ERR_UNSUPPORTED);
    }
    Loader ld{c, g};
    const int Dp = c->pre_dim, Dd = c->dec_dim;
    const mio::GgufTensor *te = g.tensor("token_embd");
    if (!te || te->ne[0] != Dp) {
        mio::set_error("miocodec: token_embd missing or wrong width");
        return fail(MIO_ERR_FORMAT);
    }
    c->n_codes = (int)te->ne[1];
    c->tok = ld.vec("token_embd", (size_t)Dp * c->n_codes);
    for (int i = 0; i < c->pre_layers; ++i) {
        const std::string p = "wave_prenet.blk." + std::to_string(i) + ".";
        PreW w{};
        w.ln1_w = ld.vec(p + "attn_norm.weight", Dp);
        w.ln1_b = ld.vec(p + "attn_norm.bias", Dp);
        w.qkv = ld.qkv(p, Dp);
        w.wo = ld.vec(p + "attn_output.weight", (size_t)Dp * Dp);
        w.ln2_w = ld.vec(p + "ffn_norm.weight", Dp);
        w.ln2_b = ld.vec(p + "ffn_norm.bias", Dp);
        w.gu = ld.gate_up(p + "ffn_gate.weight", p + "ffn_up.weight", Dp, c->pre_ff);
        w.wd = ld.vec(p + "ffn_down.weight", (size_t)c->pre_ff * Dp);
        w.h16_qkv = ld.f16({p + "attn_q.weight", p + "attn_k.weight", p + "attn_v.weight"});
        w.h16_wo = ld.f16({p + "attn_output.weight"});
        w.h16_gu = ld.f16({p + "ffn_gate.weight", p + "ffn_up.weight"});
        w.h16_wd = ld.f16({p + "ffn_down.weight"});
        c->pre.push_back(w);
    }
    c->pre_norm_w = ld.vec("wave_prenet.norm.weight", Dp);
    c->pre_norm_b = ld.vec("wave_prenet.norm.bias", Dp);
    c->pre_out_w = ld.vec("wave_prenet.output.weight", (size_t)Dp * Dd);
    c->pre_out_b = ld.vec("wave_prenet.output.bias", Dd);
    c->h16_pre_out = ld.f16({"wave_prenet.output.weight"});
    c->h16_ups = ld.f16({"wave_upsample.weight"});
    {   // ConvT k=2 s=2: ggml [2][Cout][Cin] (mem [ci][co][k]) -> B[(k*Cout+co)][ci]
        const mio::GgufTensor *tu = g.tensor("wave_upsample.weight");
        if (!tu || tu->ne[0] != 2 || tu->ne[1] != Dd || tu->ne[2] != Dd) {
            mio::set_error("miocodec: wave_upsample.weight must be [2, %d, %d]", Dd, Dd);
            return fail(MIO_ERR_FORMAT);
        }
        std::vector<float> w = ld.f32("wave_upsample.weight", (size_t)2 * Dd * Dd), o((size_t)2 * Dd * Dd);
        for (int ci = 0; ci < Dd && ld.ok; ++ci)
            for (int co = 0; co < Dd; ++co)
                for (int k = 0; k < 2; ++k) o[((size_t)k * Dd + co) * Dd + ci] = w[((size_t)ci * Dd + co) * 2 + k];
        c->ups_w = ld.up(o);
        c->ups_b = ld.vec("wave_upsample.bias", Dd);
    }
    for (int b = 0; b < c->res_blocks; ++b) c->prior.push_back(ld.resnet("wave_prior." + std::to_string(b) + ".", Dd));
    {
        std::vector<float> cw, cb;
        for (int i = 0; i < c->dec_layers; ++i) {
            const std::string p = "wave_decoder.blk." + std::to_string(i) + ".";
            for (const char *n : {"attn_cond", "ffn_cond"}) {
                std::vector<float> w = ld.f32(p + n + ".weight", (size_t)c->adaln * 3 * Dd);
                std::vector<float> bb = ld.f32(p + n + ".bias", (size_t)3 * Dd);
                cw.insert(cw.end(), w.begin(), w.end());
                cb.insert(cb.end(), bb.begin(), bb.end());
            }
            DecW w{};
            w.qkv = ld.qkv(p, Dd);
            w.wo = ld.vec(p + "attn_output.weight", (size_t)Dd * Dd);
            w.gu = ld.gate_up(p + "ffn_gate.weight", p + "ffn_up.weight", Dd, c->dec_ff);
            w.wd = ld.vec(p + "ffn_down.weight", (size_t)c->dec_ff * Dd);
            w.h16_qkv = ld.f16({p + "attn_q.weight", p + "attn_k.weight", p + "attn_v.weight"});
            w.h16_wo = ld.f16({p + "attn_output.weight"});
            w.h16_gu = ld.f16({p + "ffn_gate.weight", p + "ffn_up.weight"});
            w.h16_wd = ld.f16({p + "ffn_down.weight"});
            c->dec.push_back(w);
        }
        std::vector<float> w = ld.f32("wave_decoder.norm_cond.weight", (size_t)c->adaln * 2 * Dd);
        std::vector<float> bb = ld.f32("wave_decoder.norm_cond.bias", (size_t)2 * Dd);
        cw.insert(cw.end(), w.begin(), w.end());
        cb.insert(cb.end(), bb.begin(), bb.end());
        c->cond_rows = (int)cb.size();
        {   // every conditioning matrix shares one GEMV: one rounding rule for all of them
            std::vector<std::string> names{"wave_decoder.norm_cond.weight"};
            for (int i = 0; i < c->dec_layers; ++i)
                for (const char *n : {"attn_cond", "ffn_cond"})
                    names.push_back("wave_decoder.blk." + std::to_string(i) + "." + n + ".weight");
            int n16 = 0;
            for (const std::string &nm : names) n16 += ld.f16({nm});
            if (n16 && n16 != (int)names.size()) {
                mio::set_error("miocodec: the AdaLN conditioning matrices mix F16 and F32");
                return fail(MIO_ERR_UNSUPPORTED);
            }
            c->h16_cond = n16 ? 1 : 0;
        }
        c->cond_w = ld.up(cw);
        c->cond_b = ld.up(cb);
    }
    for (int b = 0; b < c->res_blocks; ++b) c->post.push_back(ld.resnet("wave_post." + std::to_string(b) + ".", Dd));
    // upsampler stages: factors / kernels from int tensors (:480-481)
    std::vector<int> fac(c->up_stages), ker(c->up_stages);
    {
        const mio::GgufTensor *tf = g.tensor("miocodec.wave_upsampler.factors");
        const mio::GgufTensor *tk = g.tensor("miocodec.wave_upsampler.kernel_sizes");
        if (c->up_stages && (!tf || !tk || tf->type != mio::GGML_I32 || tk->type != mio::GGML_I32 ||
                             tf->nelements() < c->up_stages || tk->nelements() < c->up_stages)) {
            mio::set_error("miocodec: upsampler factors/kernel_sizes tensors missing");
            return fail(MIO_ERR_FORMAT);
        }
        if (c->up_stages) {
            std::memcpy(fac.data(), tf->data, 4 * c->up_stages);
            std::memcpy(ker.data(), tk->data, 4 * c->up_stages);
        }
    }
    int cin = Dd;
    for (int s = 0; s < c->up_stages; ++s) {
        const std::string ss = std::to_string(s);
        const mio::GgufTensor *tw = g.tensor("wave_upsampler.up." + ss + ".weight");
        if (!tw || tw->ne[0] != ker[s] || tw->ne[2] != cin) {
            mio::set_error("miocodec: wave_upsampler.up.%d.weight shape mismatch", s);
            return fail(MIO_ERR_FORMAT);
        }
        UpW u{};
        u.f = fac[s], u.K = ker[s], u.Cin = cin, u.Cout = (int)tw->ne[1];
        u.taps = (u.K + u.f - 1) / u.f;
        u.trim = (u.K - u.f) / 2 > 0 ? (u.K - u.f) / 2 : 0;
        if (u.Cout % 4 || u.Cin % 4) {
            mio::set_error("miocodec: upsampler channels must be multiples of 4");
            return fail(MIO_ERR_UNSUPPORTED);
        }
        std::vector<float> w = ld.f32("wave_upsampler.up." + ss + ".weight", (size_t)u.K * u.Cout * u.Cin);
        std::vector<float> o((size_t)u.f * u.Cout * u.taps * u.Cin, 0.0f);
        for (int r = 0; r < u.f && ld.ok; ++r)
            for (int co = 0; co < u.Cout; ++co)
                for (int j = 0; j < u.taps; ++j) {
                    const int m = u.taps - 1 - j, k = r + u.f * m;
                    if (k >= u.K) continue;
                    for (int ci = 0; ci < u.Cin; ++ci)
                        o[((size_t)r * u.Cout + co) * u.taps * u.Cin + (size_t)j * u.Cin + ci] =
                            w[((size_t)ci * u.Cout + co) * u.K + k];
                }
        u.w = ld.up(o);
        u.h16 = ld.f16({"wave_upsampler.up." + ss + ".weight"});
        u.b = ld.vec("wave_upsampler.up." + ss + ".bias", u.Cout);
        u.alpha_e = ld.up(ld.snake_exp("wave_upsampler.snake." + ss + ".alpha", u.Cout));
        u.beta_e = ld.up(ld.snake_exp("wave_upsampler.snake." + ss + ".beta", u.Cout));
        u.res = ld.resnet("wave_upsampler.resblk." + ss + ".", u.Cout);
        c->ups.push_back(u);
        cin = u.Cout;
    }
    c->c_last = cin;
    c->op_w = ld.vec("wave_upsampler.out_proj.weight", (size_t)cin * Dd);
    c->op_b = ld.vec("wave_upsampler.out_proj.bias", Dd);
    c->h16_op = ld.f16({"wave_upsampler.out_proj.weight"});
    c->op_ae = ld.up(ld.snake_exp("wave_upsampler.out_snake.alpha", Dd));
    c->op_be = ld.up(ld.snake_exp("wave_upsampler.out_snake.beta", Dd));
    c->h16_head = ld.f16({"istft_head.out.weight"});
    {   // head rows interleaved per 16: [logmag 16p.., phase 16p..], zero-padded to nfp bins
        const int nf = c->n_freq;
        c->nfp = (nf + 15) / 16 * 16;
        std::vector<float> w = ld.f32("istft_head.out.weight", (size_t)Dd * 2 * nf);
        std::vector<float> bb = ld.f32("istft_head.out.bias", (size_t)2 * nf);
        std::vector<float> o((size_t)2 * c->nfp * Dd, 0.0f), ob((size_t)2 * c->nfp, 0.0f);
        for (int p = 0; p < c->nfp / 16 && ld.ok; ++p)
            for (int r = 0; r < 16; ++r) {
                const int k = 16 * p + r;
                if (k >= nf) continue;
                std::memcpy(&o[((size_t)32 * p + r) * Dd], &w[(size_t)k * Dd], Dd * 4);
                std::memcpy(&o[((size_t)32 * p + 16 + r) * Dd], &w[(size_t)(nf + k) * Dd], Dd * 4);
                ob[32 * p + r] = bb[k];
                ob[32 * p + 16 + r] = bb[nf + k];
            }
        c->head_w = ld.up(o);
        c->head_b = ld.up(ob);
    }
    if (!ld.ok) return fail(MIO_ERR_FORMAT);
    {   // ResNet widths: f16 conv operand in 8-channel chunks, GroupNorm groups inside 64 lanes
        auto gn_ok = [&](int C) {
            return C % 8 == 0 && C <= 1024 && C % c->groups == 0 && 64 % (C / c->groups) == 0;
        };
        bool ok = gn_ok(Dd);
        for (const UpW &u : c->ups) ok = ok && gn_ok(u.Cout);
        if (!ok) {
            mio::set_error("miocodec: ResNet widths must be multiples of 8 (<= 1024) with C/groups dividing 64");
            return fail(MIO_ERR_UNSUPPORTED);
        }
    }
    rc = mio_hip_istft_create(d, c->n_fft, c->n_fft, &c->ist);
    if (rc) return fail(rc);
    *out = c;
    return MIO_OK;
}

extern "C" void mio_hip_codec_free(mio_hip_codec *c) { delete c; }

extern "C" int mio_hip_codec_info(const mio_hip_codec *c, int *info) {
    MIO_REQUIRE(c && info, MIO_ERR_INVALID, "codec_info: null");
    int up = 1;
    for (auto &u : c->ups) up *= u.f;
    info[0] = c->sample_rate, info[1] = c->n_fft, info[2] = c->hop, info[3] = c->spt;
    info[4] = c->n_freq, info[5] = c->up_stages, info[6] = 2 * up, info[7] = c->n_codes;
    return MIO_OK;
}

extern "C" int mio_hip_codec_decode_stage(mio_hip_codec *c, const int32_t *codes, int n_codes,
                                          const float *emb, int stage, float *out, int *rows,
                                          int *cols) {
    MIO_REQUIRE(c && codes && emb && out && n_codes > 0, MIO_ERR_INVALID, "codec_decode_stage: bad args");
    int rc = mio::bind(c->d);
    if (rc) return rc;
    hipStream_t s = c->d->stream;
    Ws w;
    if ((rc = plan_ws(c, n_codes, w, true))) return rc;
    if ((rc = prepare_inputs(c, w, codes, n_codes, emb, 0, s))) return rc;
    const float *buf = nullptr;
    int r = 0, cc = 0;
    if ((rc = run_decode(c, w, s, stage, &buf, &r, &cc))) return rc;
    MIO_REQUIRE(buf, MIO_ERR_INVALID, "codec_decode_stage: stage %d out of range", stage);
    MIO_HIP_CHECK(hipGetLastError());
    MIO_HIP_CHECK(hipMemcpyAsync(out, buf, (size_t)r * cc * 4, hipMemcpyDeviceToHost, s));
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    if (rows) *rows = r;
    if (cols) *cols = cc;
    return MIO_OK;
}

extern "C" int mio_hip_codec_decode(mio_hip_codec *c, const int32_t *codes, int n_codes,
                                    const float *emb, float *out_spec, int *out_frames,
                                    unsigned flags, void *stream) {
    MIO_REQUIRE(c && codes && emb && out_spec && n_codes > 0, MIO_ERR_INVALID, "codec_decode: bad args");
    int rc = mio::bind(c->d);
    if (rc) return rc;
    hipStream_t s = mio::pick_stream(c->d, stream);
    Ws w;
    if ((rc = plan_ws(c, n_codes, w, true))) return rc;
    if ((rc = prepare_inputs(c, w, codes, n_codes, emb, flags, s))) return rc;
    const float *buf = nullptr;
    int r = 0, cc = 0;
    if ((rc = run_decode(c, w, s, 1 << 20, &buf, &r, &cc))) return rc;
    MIO_HIP_CHECK(hipGetLastError());
    const size_t bytes = (size_t)w.Lf * 2 * c->n_freq * 4;
    if (out_frames) *out_frames = w.Lf;
    if (flags & MIO_OUT_DEVICE) {
        MIO_HIP_CHECK(hipMemcpyAsync(out_spec, w.spec, bytes, hipMemcpyDeviceToDevice, s));
    } else {
        MIO_HIP_CHECK(hipMemcpyAsync(out_spec, w.spec, bytes, hipMemcpyDeviceToHost, s));
        MIO_HIP_CHECK(hipStreamSynchronize(s));
    }
    return MIO_OK;
}

extern "C" int mio_hip_codec_decode_pcm(mio_hip_codec *c, const int32_t *codes, int n_codes,
                                        const float *emb, float *out_pcm, int *out_len,
                                        unsigned flags, void *stream) {
    MIO_REQUIRE(c && codes && emb && out_pcm && n_codes > 0, MIO_ERR_INVALID, "codec_decode_pcm: bad args");
    int rc = mio::bind(c->d);
    if (rc) return rc;
    hipStream_t s = mio::pick_stream(c->d, stream);
    Ws w;
    if ((rc = plan_ws(c, n_codes, w, true))) return rc;
    if ((rc = prepare_inputs(c, w, codes, n_codes, emb, flags, s))) return rc;
    const float *buf = nullptr;
    int r = 0, cc = 0;
    if (!c->ev[0])
        for (auto &e : c->ev) MIO_HIP_CHECK(hipEventCreate(&e));
    const bool incr = (flags & MIO_CODEC_INCREMENTAL) && !(flags & MIO_IN_DEVICE);
    int cached = 0;
    if (incr) {
        int prefix = 0;
        const int lim = std::min(n_codes, (int)c->pc_codes.size());
        while (prefix < lim && c->pc_codes[prefix] == codes[prefix]) ++prefix;
        // a cached row is valid while every code of its receptive field is unchanged
        cached = std::min(c->pc_exact, std::max(0, prefix - prenet_radius(c)));
        if (n_codes > c->pc_cap) {  // grow the cache before this decode reads it
            float *np = nullptr;
            const int cap = std::max(2 * n_codes, 1024);
            MIO_HIP_CHECK(hipMalloc(&np, (size_t)cap * c->dec_dim * 4));
            if (cached > 0)
                MIO_HIP_CHECK(hipMemcpyAsync(np, c->pc, (size_t)cached * c->dec_dim * 4, hipMemcpyDeviceToDevice, s));
            MIO_HIP_CHECK(hipStreamSynchronize(s));
            if (c->pc) hipFree(c->pc);
            c->pc = np;
            c->pc_cap = cap;
        }
    }
    c->pc_last_reused = cached;
    MIO_HIP_CHECK(hipEventRecord(c->ev[0], s));
    t_flops = 0.0;
    if ((rc = run_decode(c, w, s, 1 << 20, &buf, &r, &cc, cached))) return rc;
    c->last_flops = t_flops;
    if (incr) {  // rows whose receptive field this decode held completely become the cache
        const int exact = std::max(0, n_codes - prenet_radius(c));
        if (exact > cached)
            MIO_HIP_CHECK(hipMemcpyAsync(c->pc + (size_t)cached * c->dec_dim, w.yT + (size_t)cached * c->dec_dim,
                                         (size_t)(exact - cached) * c->dec_dim * 4, hipMemcpyDeviceToDevice, s));
        c->pc_exact = exact;
        c->pc_codes.assign(codes, codes + n_codes);
    }
    MIO_HIP_CHECK(hipEventRecord(c->ev[1], s));
    int len = 0;
    if ((rc = mio_hip_istft_out_len(c->ist, w.Lf, c->hop, &len))) return rc;
    if ((rc = mio_istft_launch_device(c->ist, w.spec, w.Lf, c->hop, w.pcm, s))) return rc;
    MIO_HIP_CHECK(hipEventRecord(c->ev[2], s));
    c->timed = true;
    MIO_HIP_CHECK(hipGetLastError());
    if (out_len) *out_len = len;
    if (flags & MIO_OUT_DEVICE) {
        MIO_HIP_CHECK(hipMemcpyAsync(out_pcm, w.pcm, (size_t)len * 4, hipMemcpyDeviceToDevice, s));
    } else {
        MIO_HIP_CHECK(hipMemcpyAsync(out_pcm, w.pcm, (size_t)len * 4, hipMemcpyDeviceToHost, s));
        MIO_HIP_CHECK(hipStreamSynchronize(s));
    }
    return MIO_OK;
}

// Concurrent decodes of independent utterances (header: mio_hip_codec_decode_pcm_batch). Every
// lane's workspace and the RoPE table are sized before the first kernel is issued, so no
// hipFree runs while another lane's kernels read a buffer.
extern "C" int mio_hip_codec_decode_pcm_batch(mio_hip_codec *c, const int32_t *const *codes, const int *n_codes,
                                              int B, const float *emb, float *const *out_pcm, int *out_len,
                                              unsigned flags, void *stream) {
    MIO_REQUIRE(c && codes && n_codes && emb && out_pcm && B > 0, MIO_ERR_INVALID, "codec_decode_pcm_batch: bad args");
    MIO_REQUIRE(!(flags & MIO_CODEC_INCREMENTAL), MIO_ERR_INVALID, "codec_decode_pcm_batch: no incremental decodes");
    for (int b = 0; b < B; ++b)
        MIO_REQUIRE(codes[b] && out_pcm[b] && n_codes[b] > 0, MIO_ERR_INVALID, "codec_decode_pcm_batch: utterance %d", b);
    int rc = mio::bind(c->d);
    if (rc) return rc;
    hipStream_t s = mio::pick_stream(c->d, stream);
    static const int kLanes = [] {
        const char *e = getenv("MIO_CODEC_STREAMS");
        const int v = e ? atoi(e) : 3;  // 8 x 700 codes: 23.1 / 17.8 / 16.9 / 18.8 ms at 1-4 (r06)
        return v < 1 ? 1 : (v > 8 ? 8 : v);
    }();
    const int NS = std::min(B, kLanes);
    if (!c->ev[0])
        for (auto &e : c->ev) MIO_HIP_CHECK(hipEventCreate(&e));
    while ((int)c->xs.size() < NS - 1) {
        hipStream_t q = nullptr;
        hipEvent_t e = nullptr;
        MIO_HIP_CHECK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
        MIO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->xs.push_back(q), c->xev.push_back(e), c->xws.push_back(nullptr), c->xws_cap.push_back(0);
    }
    // size every lane for its longest utterance first (allocations wait for the device)
    for (int k = 0; k < NS; ++k) {
        int tmax = 0;
        for (int b = k; b < B; b += NS) tmax = std::max(tmax, n_codes[b]);
        Ws w;
        if ((rc = plan_ws(c, tmax, w, true, nullptr, k))) return rc;
    }
    MIO_HIP_CHECK(hipEventRecord(c->ev[0], s));
    for (int k = 1; k < NS; ++k) MIO_HIP_CHECK(hipStreamWaitEvent(c->xs[k - 1], c->ev[0], 0));
    double flops = 0.0;
    for (int b = 0; b < B; ++b) {
        const int k = b % NS;
        hipStream_t ls = k ? c->xs[k - 1] : s;
        Ws w;
        if ((rc = plan_ws(c, n_codes[b], w, false, nullptr, k))) return rc;
        if ((rc = prepare_inputs(c, w, codes[b], n_codes[b], emb, flags, ls))) return rc;
        const float *buf = nullptr;
        int r = 0, cc = 0;
        t_flops = 0.0;
        if ((rc = run_decode(c, w, ls, 1 << 20, &buf, &r, &cc))) return rc;
        flops += t_flops;
        int len = 0;
        if ((rc = mio_hip_istft_out_len(c->ist, w.Lf, c->hop, &len))) return rc;
        if (flags & MIO_OUT_DEVICE) {
            if ((rc = mio_istft_launch_device(c->ist, w.spec, w.Lf, c->hop, out_pcm[b], ls))) return rc;
        } else {
            if ((rc = mio_istft_launch_device(c->ist, w.spec, w.Lf, c->hop, w.pcm, ls))) return rc;
            MIO_HIP_CHECK(hipMemcpyAsync(out_pcm[b], w.pcm, (size_t)len * 4, hipMemcpyDeviceToHost, ls));
        }
        if (out_len) out_len[b] = len;
    }
    for (int k = 1; k < NS; ++k) {
        MIO_HIP_CHECK(hipEventRecord(c->xev[k - 1], c->xs[k - 1]));
        MIO_HIP_CHECK(hipStreamWaitEvent(s, c->xev[k - 1], 0));
    }
    MIO_HIP_CHECK(hipGetLastError());
    // last_timings: codec = the whole batch (decodes and iSTFTs overlap), iSTFT 0
    MIO_HIP_CHECK(hipEventRecord(c->ev[1], s));
    MIO_HIP_CHECK(hipEventRecord(c->ev[2], s));
    c->timed = true;
    c->last_flops = flops;
    if (!(flags & MIO_OUT_DEVICE)) MIO_HIP_CHECK(hipStreamSynchronize(s));
    return MIO_OK;
}

// Device memory a decode of up to n_codes codes needs (workspace, RoPE table, the
// incremental prenet cache, timing events), allocated now: the ggml_gallocr reserve of
// miocodec_load (miocodec.cpp:424-516) happens at load too, so no decode pays a hipMalloc
// (and a hipFree that waits for the whole device) in its own time.
extern "C" int mio_hip_codec_reserve(mio_hip_codec *c, int n_codes) {
    MIO_REQUIRE(c && n_codes > 0, MIO_ERR_INVALID, "codec_reserve: bad args");
    int rc = mio::bind(c->d);
    if (rc) return rc;
    Ws w;
    if ((rc = plan_ws(c, n_codes, w, true))) return rc;
    if (!c->ev[0])
        for (auto &e : c->ev) MIO_HIP_CHECK(hipEventCreate(&e));
    if (n_codes > c->pc_cap) {
        const int cap = std::max(2 * n_codes, 1024);
        float *np = nullptr;
        MIO_HIP_CHECK(hipMalloc(&np, (size_t)cap * c->dec_dim * 4));
        if (c->pc) {
            MIO_HIP_CHECK(hipDeviceSynchronize());
            hipFree(c->pc);
        }
        c->pc = np;
        c->pc_cap = cap;
        c->pc_exact = 0;
        c->pc_codes.clear();
    }
    return MIO_OK;
}

extern "C" int mio_hip_codec_last_reused(const mio_hip_codec *c, int *rows) {
    MIO_REQUIRE(c && rows, MIO_ERR_INVALID, "codec_last_reused: null");
    *rows = c->pc_last_reused;
    return MIO_OK;
}

extern "C" int mio_hip_codec_last_flops(const mio_hip_codec *c, double *flops) {
    MIO_REQUIRE(c && flops, MIO_ERR_INVALID, "codec_last_flops: null");
    *flops = c->last_flops;
    return MIO_OK;
}

extern "C" int mio_hip_codec_last_timings(const mio_hip_codec *c, float *ms2) {
    MIO_REQUIRE(c && ms2 && c->timed, MIO_ERR_INVALID, "codec_last_timings: no timed decode yet");
    MIO_HIP_CHECK(hipEventSynchronize(c->ev[2]));
    MIO_HIP_CHECK(hipEventElapsedTime(&ms2[0], c->ev[0], c->ev[1]));
    MIO_HIP_CHECK(hipEventElapsedTime(&ms2[1], c->ev[1], c->ev[2]));
    return MIO_OK;
}
