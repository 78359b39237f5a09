/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of miocodec_decode (/root/reference/src/miocodec.cpp:519-810) with the
 * ggml CPU op semantics the reference runs through (ggml is absent here, SURVEY F1, so
 * this oracle is "parity unpinned": it follows the documented ggml semantics below).
 *
 * Layout: activations are kept row-major [rows][channels] ("transformer format");
 * the reference's transposes (miocodec.cpp:228-230) are layout-only and omitted.
 *
 * Op semantics followed (ggml CPU backend):
 *   norm        mean/var accumulated in double, y=(x-mean)*(1/sqrtf(var+eps))   (:212-217)
 *   group_norm  per group of ceil(C/G) channels x all positions, double sums      (:358-371)
 *   rope mode 0 adjacent pairs, theta_p,i = p * theta_scale^i by repeated float
 *               multiplication (ggml rope cache), theta_scale = powf(base,-2/n_dims) (:260-263)
 *   soft_max    scores*0.125 + mask(0/-inf), exp(x-max), sum in double, * (1/sum)  (:271-275)
 *   mul_mat     f32 weight: f32 dot products; F16 weight: the input rounded to f16 first
 *               (ggml's vec_dot_type of F16 is F16), products summed in f32          (:204-209)
 *   conv_1d     kernel AND im2col input rounded to f16, products summed in f32    (:381-386)
 *   conv_transpose_1d dst[t*s+k] += dot_ci(x[t], W_k) in ascending t; an F16 kernel rounds
 *               the input to f16 like mul_mat                                   (:624, :685)
 *   snake       x + sin(exp(a)*x)^2 / exp(b); F16 a / b: ggml_exp keeps F16, so exp is
 *               rounded to f16                                                   (:410-420, :717-725)
 *   other F16 tensors (norm / bias / embedding) enter as their exact f32 values
 *   head        mag = clamp(exp(.),0,100), (re,im) = mag*(cos,sin)(phase)         (:728-737)
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gguf_ref.h"
#include "mio_oracle.h"

struct mo_codec {
    mo_gguf *g;
    float **f32_of; /* per GGUF tensor: f32 copy of an F16 tensor, else NULL */
    int sr, n_fft, hop, n_freq, spt, head_out;
    int pre_layers, pre_dim, pre_heads, pre_ff, pre_win;
    int dec_layers, dec_dim, dec_heads, dec_ff, dec_win, adaln;
    int res_blocks, groups, up_stages;
    float theta, eps, gn_eps;
    int factors[8], kernels[8];
    int n_codes;
};

static const float *W(const mo_codec *c, const char *name) {
    const mo_tensor *t = mo_gguf_tensor(c->g, name);
    if (!t) return NULL;
    if (t->type == 0) return (const float *)t->data;
    if (t->type == 1) return c->f32_of[t - c->g->tensors];
    return NULL;
}

/* a matrix operand and whether it was stored F16 (mul_mat then rounds its input to f16) */
typedef struct {
    const float *w;
    int f16;
} wref;

static wref WR(const mo_codec *c, const char *name) {
    const mo_tensor *t = mo_gguf_tensor(c->g, name);
    wref r = {W(c, name), t && t->type == 1};
    return r;
}

static int is_f16(const mo_codec *c, const char *name) {
    const mo_tensor *t = mo_gguf_tensor(c->g, name);
    return t && t->type == 1;
}

float mo_fp16_to_f32(uint16_t h);

static int WN(const mo_codec *c, const char *name, int dim) {
    const mo_tensor *t = mo_gguf_tensor(c->g, name);
    return t ? (int)t->ne[dim] : 0;
}

mo_codec *mo_codec_load(const char *path) {
    mo_gguf *g = mo_gguf_open(path);
    if (!g) return NULL;
    mo_codec *c = (mo_codec *)calloc(1, sizeof(mo_codec));
    c->g = g;
    /* miocodec.cpp:448-474 with the same defaults */
    c->sr = (int)mo_gguf_int(g, "miocodec.sample_rate", 44100);
    c->n_fft = (int)mo_gguf_int(g, "miocodec.n_fft", 392);
    c->hop = (int)mo_gguf_int(g, "miocodec.hop_length", 98);
    c->n_freq = c->n_fft / 2 + 1;
    c->spt = (int)mo_gguf_int(g, "miocodec.samples_per_token", 1764);
    c->head_out = (int)mo_gguf_int(g, "embedding_length_out", 394);
    c->pre_layers = (int)mo_gguf_int(g, "miocodec.prenet_layers", 6);
    c->pre_dim = (int)mo_gguf_int(g, "miocodec.prenet_dim", 768);
    c->pre_heads = (int)mo_gguf_int(g, "miocodec.prenet_heads", 12);
    c->pre_ff = (int)mo_gguf_int(g, "miocodec.prenet_ff", 2048);
    c->pre_win = (int)mo_gguf_int(g, "miocodec.prenet_window", 65);
    c->dec_layers = (int)mo_gguf_int(g, "miocodec.decoder_layers", 8);
    c->dec_dim = (int)mo_gguf_int(g, "miocodec.decoder_dim", 512);
    c->dec_heads = (int)mo_gguf_int(g, "miocodec.decoder_heads", 8);
    c->dec_ff = (int)mo_gguf_int(g, "miocodec.decoder_ff", 1536);
    c->dec_win = (int)mo_gguf_int(g, "miocodec.decoder_window", 65);
    c->adaln = (int)mo_gguf_int(g, "miocodec.decoder_adanorm_dim", 128);
    c->res_blocks = (int)mo_gguf_int(g, "miocodec.resnet_blocks", 2);
    c->groups = (int)mo_gguf_int(g, "miocodec.resnet_groups", 32);
    c->up_stages = (int)mo_gguf_int(g, "miocodec.wave_upsampler_layers", 2);
    c->theta = (float)mo_gguf_float(g, "miocodec.rope_theta", 10000.0);
    c->eps = (float)mo_gguf_float(g, "miocodec.norm_eps", 1e-5);
    c->gn_eps = (float)mo_gguf_float(g, "miocodec.group_norm_eps", 1e-6);
    const mo_tensor *tf = mo_gguf_tensor(g, "miocodec.wave_upsampler.factors");
    const mo_tensor *tk = mo_gguf_tensor(g, "miocodec.wave_upsampler.kernel_sizes");
    if (!tf || !tk || c->up_stages > 8) { mo_gguf_close(g); free(c); return NULL; }
    memcpy(c->factors, tf->data, sizeof(int) * c->up_stages);
    memcpy(c->kernels, tk->data, sizeof(int) * c->up_stages);
    c->n_codes = WN(c, "token_embd", 1);
    c->f32_of = (float **)calloc(g->n_tensors, sizeof(float *));
    for (int i = 0; i < g->n_tensors; i++) {
        const mo_tensor *t = &g->tensors[i];
        if (t->type != 1) continue;
        size_t n = 1;
        for (int d = 0; d < t->n_dims; d++) n *= (size_t)t->ne[d];
        float *f = (float *)malloc(n * sizeof(float));
        const uint16_t *h = (const uint16_t *)t->data;
        for (size_t j = 0; j < n; j++) f[j] = mo_fp16_to_f32(h[j]);
        c->f32_of[i] = f;
    }
    return c;
}

void mo_codec_free(mo_codec *c) {
    if (!c) return;
    for (int i = 0; i < c->g->n_tensors; i++) free(c->f32_of[i]);
    free(c->f32_of);
    mo_gguf_close(c->g);
    free(c);
}

void mo_codec_info(const mo_codec *c, int *info) {
    info[0] = c->sr; info[1] = c->n_fft; info[2] = c->hop; info[3] = c->spt;
    info[4] = c->n_freq; info[5] = c->up_stages;
    int up = 1;
    for (int i = 0; i < c->up_stages; i++) up *= c->factors[i];
    info[6] = 2 * up; /* frames per code */
    info[7] = c->n_codes;
}

/* ------------------------------------------------------------------ helpers */

static float dot_f32(const float *a, const float *b, int n) {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
    for (; i + 8 <= n; i += 8)
        for (int j = 0; j < 8; j++) s[j] += a[i + j] * b[i + j];
    float r = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    for (; i < n; i++) r += a[i] * b[i];
    return r;
}

float mo_f16_round(float f);

/* x rounded to f16 (a fresh buffer) when rx, else x itself */
static const float *round_in(const float *x, size_t n, int rx, float **tmp) {
    *tmp = NULL;
    if (!rx) return x;
    float *r = (float *)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; i++) r[i] = mo_f16_round(x[i]);
    *tmp = r;
    return r;
}

/* y[m][n] = x[m][:] . w[n][:] (+ b[n]);  w is ggml [K, N] = row-major [N][K] */
static void linear(const float *x_in, int M, int K, wref wr, const float *b, int N, float *y) {
    const int NB = 64;
    float *tmp;
    const float *x = round_in(x_in, (size_t)M * K, wr.f16, &tmp);
    const float *w = wr.w;
#pragma omp parallel for collapse(2) schedule(static)
    for (int n0 = 0; n0 < N; n0 += NB)
        for (int m = 0; m < M; m++) {
            const int n1 = n0 + NB < N ? n0 + NB : N;
            for (int n = n0; n < n1; n++) {
                float v = dot_f32(x + (size_t)m * K, w + (size_t)n * K, K);
                y[(size_t)m * N + n] = b ? v + b[n] : v;
            }
        }
    free(tmp);
}

/* ggml_norm (+ optional affine w,b applied as separate mul/add) */
static void norm_rows(const float *x, int M, int D, float eps, float *y) {
#pragma omp parallel for schedule(static)
    for (int m = 0; m < M; m++) {
        const float *xr = x + (size_t)m * D;
        float *yr = y + (size_t)m * D;
        double sum = 0.0;
        for (int i = 0; i < D; i++) sum += (double)xr[i];
        const float mean = (float)(sum / D);
        double sum2 = 0.0;
        for (int i = 0; i < D; i++) {
            const float v = xr[i] - mean;
            yr[i] = v;
            sum2 += (double)(v * v);
        }
        const float variance = (float)(sum2 / D);
        const float scale = 1.0f / sqrtf(variance + eps);
        for (int i = 0; i < D; i++) yr[i] *= scale;
    }
}

static void layer_norm(const float *x, int M, int D, const float *w, const float *b, float eps,
                       float *y) {
    norm_rows(x, M, D, eps, y);
#pragma omp parallel for schedule(static)
    for (int m = 0; m < M; m++)
        for (int i = 0; i < D; i++) {
            float v = y[(size_t)m * D + i] * w[i];
            y[(size_t)m * D + i] = b ? v + b[i] : v;
        }
}

/* adaln_norm (miocodec.cpp:322-330): norm(x) * (1 + scale) + shift */
static void adaln_norm(const float *x, int M, int D, const float *shift, const float *scale,
                       float eps, float *y) {
    norm_rows(x, M, D, eps, y);
    float *s = (float *)malloc(sizeof(float) * D);
    for (int i = 0; i < D; i++) s[i] = 1.0f + scale[i];
#pragma omp parallel for schedule(static)
    for (int m = 0; m < M; m++)
        for (int i = 0; i < D; i++) {
            float v = y[(size_t)m * D + i] * s[i];
            y[(size_t)m * D + i] = v + shift[i];
        }
    free(s);
}

static inline float silu(float x) { return x / (1.0f + expf(-x)); }

/* ggml rope cache: theta = p, theta *= theta_scale per pair (float) */
static void rope_table(int S, int hd, float base, float *ct, float *st) {
    const float theta_scale = powf(base, -2.0f / hd);
    for (int p = 0; p < S; p++) {
        float theta = (float)p;
        for (int i = 0; i < hd / 2; i++) {
            ct[(size_t)p * (hd / 2) + i] = cosf(theta);
            st[(size_t)p * (hd / 2) + i] = sinf(theta);
            theta *= theta_scale;
        }
    }
}

/* mha_rope (miocodec.cpp:245-286) on qkv [S][3D] (q | k | v), out attn [S][D] */
static void attention(const float *q_in, const float *k_in, const float *v_in, int ld, int S,
                      int H, int hd, int window, float base, float *out /*[S][H*hd]*/) {
    const int D = H * hd, half = hd / 2, hw = window / 2;
    float *ct = (float *)malloc(sizeof(float) * (size_t)S * half);
    float *st = (float *)malloc(sizeof(float) * (size_t)S * half);
    rope_table(S, hd, base, ct, st);
    float *q = (float *)malloc(sizeof(float) * (size_t)S * D);
    float *k = (float *)malloc(sizeof(float) * (size_t)S * D);
#pragma omp parallel for schedule(static)
    for (int p = 0; p < S; p++)
        for (int h = 0; h < H; h++)
            for (int i = 0; i < half; i++) {
                const float c = ct[(size_t)p * half + i], s = st[(size_t)p * half + i];
                const float *qs = q_in + (size_t)p * ld + h * hd;
                const float *ks = k_in + (size_t)p * ld + h * hd;
                float *qd = q + (size_t)p * D + h * hd, *kd = k + (size_t)p * D + h * hd;
                qd[2 * i] = qs[2 * i] * c - qs[2 * i + 1] * s;
                qd[2 * i + 1] = qs[2 * i] * s + qs[2 * i + 1] * c;
                kd[2 * i] = ks[2 * i] * c - ks[2 * i + 1] * s;
                kd[2 * i + 1] = ks[2 * i] * s + ks[2 * i + 1] * c;
            }
    const float scale = 1.0f / sqrtf((float)hd);
#pragma omp parallel for collapse(2) schedule(static)
    for (int h = 0; h < H; h++)
        for (int i = 0; i < S; i++) {
            float sc[1024];
            const int j0 = i - hw < 0 ? 0 : i - hw;
            const int j1 = i + hw > S - 1 ? S - 1 : i + hw;
            float mx = -INFINITY;
            for (int j = j0; j <= j1; j++) {
                float s = dot_f32(k + (size_t)j * D + h * hd, q + (size_t)i * D + h * hd, hd);
                s = s * scale;
                sc[j - j0] = s;
                if (s > mx) mx = s;
            }
            double sum = 0.0;
            for (int j = j0; j <= j1; j++) {
                const float e = expf(sc[j - j0] - mx);
                sc[j - j0] = e;
                sum += (double)e;
            }
            const float inv = (float)(1.0 / sum);
            for (int j = j0; j <= j1; j++) sc[j - j0] *= inv;
            for (int d = 0; d < hd; d++) {
                float a = 0.0f;
                for (int j = j0; j <= j1; j++) a += v_in[(size_t)j * ld + h * hd + d] * sc[j - j0];
                out[(size_t)i * D + h * hd + d] = a;
            }
        }
    free(ct); free(st); free(q); free(k);
}

/* ggml_group_norm over [L][C] (transformer layout) + per-channel affine */
static void group_norm(const float *x, int L, int C, int G, const float *w, const float *b,
                       float eps, float *y) {
    const int cpg = (C + G - 1) / G;
#pragma omp parallel for schedule(static)
    for (int g = 0; g < G; g++) {
        const int c0 = g * cpg, c1 = c0 + cpg < C ? c0 + cpg : C;
        if (c0 >= c1) continue;
        const double n = (double)L * (c1 - c0);
        double sum = 0.0;
        for (int c = c0; c < c1; c++)
            for (int l = 0; l < L; l++) sum += (double)x[(size_t)l * C + c];
        const float mean = (float)(sum / n);
        double sum2 = 0.0;
        for (int c = c0; c < c1; c++)
            for (int l = 0; l < L; l++) {
                const float v = x[(size_t)l * C + c] - mean;
                y[(size_t)l * C + c] = v;
                sum2 += (double)(v * v);
            }
        const float variance = (float)(sum2 / n);
        const float scale = 1.0f / sqrtf(variance + eps);
        for (int c = c0; c < c1; c++)
            for (int l = 0; l < L; l++) y[(size_t)l * C + c] *= scale;
    }
#pragma omp parallel for schedule(static)
    for (int l = 0; l < L; l++)
        for (int c = 0; c < C; c++) {
            float v = y[(size_t)l * C + c] * w[c];
            y[(size_t)l * C + c] = v + b[c];
        }
}

/* round-to-nearest-even f32 -> f16 -> f32 (ggml F16 storage / F16C cvtps2ph) */
static float f16_round(float f) {
    unsigned int x;
    memcpy(&x, &f, 4);
    const unsigned int sign = x & 0x80000000u;
    unsigned int ax = x & 0x7fffffffu;
    unsigned short h;
    if (ax >= 0x7f800000u) {
        h = (unsigned short)((sign >> 16) | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    } else if (ax >= 0x477ff000u) { /* >= 65520 rounds to inf */
        h = (unsigned short)((sign >> 16) | 0x7c00u);
    } else if (ax < 0x38800000u) { /* subnormal half */
        float af;
        memcpy(&af, &ax, 4);
        const float t = af * 16777216.0f; /* / 2^-24 */
        unsigned int q = (unsigned int)nearbyintf(t);
        h = (unsigned short)((sign >> 16) | q);
    } else {
        unsigned int mant = ax & 0x7fffffu;
        int exp = (int)(ax >> 23) - 127 + 15;
        unsigned int hm = mant >> 13, rem = mant & 0x1fffu;
        unsigned int hv = ((unsigned int)exp << 10) | hm;
        if (rem > 0x1000u || (rem == 0x1000u && (hv & 1u))) hv++;
        h = (unsigned short)((sign >> 16) | hv);
    }
    /* back to f32 */
    const unsigned int hs = (h & 0x8000u) << 16, he = (h >> 10) & 0x1f, hm2 = h & 0x3ff;
    unsigned int out;
    if (he == 0) {
        float v = (float)hm2 * (1.0f / 16777216.0f);
        memcpy(&out, &v, 4);
        out |= hs;
    } else if (he == 31) {
        out = hs | 0x7f800000u | (hm2 << 13);
    } else {
        out = hs | ((he - 15 + 127) << 23) | (hm2 << 13);
    }
    float r;
    memcpy(&r, &out, 4);
    return r;
}

float mo_f16_round(float f) { return f16_round(f); }

/* conv_1d k=K, stride 1, pad p (miocodec.cpp:382-386): f16 kernel and f16 im2col */
static void conv1d(const float *x, int L, int Cin, const float *w /*[Cout][Cin][K]*/, int K,
                   int Cout, int pad, const float *bias, float *y) {
    const int KK = Cin * K;
    float *wh = (float *)malloc(sizeof(float) * (size_t)Cout * KK);
    for (size_t i = 0; i < (size_t)Cout * KK; i++) wh[i] = f16_round(w[i]);
#pragma omp parallel
    {
        float *col = (float *)malloc(sizeof(float) * KK);
#pragma omp for schedule(static)
        for (int l = 0; l < L; l++) {
            for (int ci = 0; ci < Cin; ci++)
                for (int k = 0; k < K; k++) {
                    const int src = l + k - pad;
                    col[ci * K + k] = (src >= 0 && src < L) ? f16_round(x[(size_t)src * Cin + ci]) : 0.0f;
                }
            for (int co = 0; co < Cout; co++) {
                const float v = dot_f32(col, wh + (size_t)co * KK, KK);
                y[(size_t)l * Cout + co] = v + bias[co];
            }
        }
        free(col);
    }
    free(wh);
}

/* conv_transpose_1d (f32 kernel ggml [K][Cout][Cin] = mem [Cin][Cout][K]) + bias + trim */
static void conv_transpose1d(const float *x_in, int L, int Cin, wref wr, int K, int Cout,
                             int stride, int trim, const float *bias, float *y /*[L*stride][Cout]*/) {
    float *tmp;
    const float *x = round_in(x_in, (size_t)L * Cin, wr.f16, &tmp);
    const float *w = wr.w;
    const int Lraw = (L - 1) * stride + K;
    const int Lout = Lraw - 2 * trim;
    /* permute kernel to [Cout][K][Cin] as ggml does */
    float *wp = (float *)malloc(sizeof(float) * (size_t)Cout * K * Cin);
    for (int ci = 0; ci < Cin; ci++)
        for (int co = 0; co < Cout; co++)
            for (int k = 0; k < K; k++)
                wp[((size_t)co * K + k) * Cin + ci] = w[((size_t)ci * Cout + co) * K + k];
#pragma omp parallel
    {
        float *acc = (float *)malloc(sizeof(float) * Lraw);
#pragma omp for schedule(static)
        for (int co = 0; co < Cout; co++) {
            memset(acc, 0, sizeof(float) * Lraw);
            for (int t = 0; t < L; t++)
                for (int k = 0; k < K; k++) {
                    const float v = dot_f32(x + (size_t)t * Cin, wp + ((size_t)co * K + k) * Cin, Cin);
                    acc[t * stride + k] += v;
                }
            for (int p = 0; p < Lout; p++) y[(size_t)p * Cout + co] = acc[p + trim] + bias[co];
        }
        free(acc);
    }
    free(wp);
    free(tmp);
}

static void snake_rows(float *x, int M, int C, const float *la, const float *lb, int fa, int fb) {
    float *a = (float *)malloc(sizeof(float) * C), *b = (float *)malloc(sizeof(float) * C);
    for (int c = 0; c < C; c++) {
        a[c] = fa ? mo_f16_round(expf(la[c])) : expf(la[c]);
        b[c] = fb ? mo_f16_round(expf(lb[c])) : expf(lb[c]);
    }
#pragma omp parallel for schedule(static)
    for (int m = 0; m < M; m++)
        for (int c = 0; c < C; c++) {
            const float v = x[(size_t)m * C + c];
            const float ax = v * a[c];
            const float s = sinf(ax);
            const float s2 = s * s;
            const float sc = s2 / b[c];
            x[(size_t)m * C + c] = v + sc;
        }
    free(a); free(b);
}

static void resnet_block(const mo_codec *c, const char *prefix, float *x, int L, int C, float *t1,
                         float *t2) {
    char n[256];
#define WP(s) (snprintf(n, sizeof n, "%s%s", prefix, s), W(c, n))
    group_norm(x, L, C, c->groups, WP("norm1.weight"), WP("norm1.bias"), c->gn_eps, t1);
    for (size_t i = 0; i < (size_t)L * C; i++) t1[i] = silu(t1[i]);
    conv1d(t1, L, C, WP("conv1.weight"), 3, C, 1, WP("conv1.bias"), t2);
    group_norm(t2, L, C, c->groups, WP("norm2.weight"), WP("norm2.bias"), c->gn_eps, t1);
    for (size_t i = 0; i < (size_t)L * C; i++) t1[i] = silu(t1[i]);
    conv1d(t1, L, C, WP("conv2.weight"), 3, C, 1, WP("conv2.bias"), t2);
    for (size_t i = 0; i < (size_t)L * C; i++) x[i] = t2[i] + x[i];
#undef WP
}

/* Runs the decoder up to `stop_stage` (see mio_oracle.h) and copies that stage's
 * activation into out. Returns 0 on success. */
/* start_stage > 0 (teacher forcing, tests only): the stages from start_stage on run on `in`, the
 * output of stage start_stage - 1 (its rows x cols as mo_codec_decode_stage returns them), in
 * place of the stages before it; codes still give T. */
static int decode_stages(mo_codec *c, const int *codes, int T, const float *emb, int start_stage, const float *in,
                         int stop_stage, float *out, int *out_rows, int *out_cols) {
    if (T <= 0) return -1;
    for (int i = 0; i < T; i++)
        if (codes[i] < 0 || codes[i] >= c->n_codes) return -2;
    const int Dp = c->pre_dim, Dd = c->dec_dim;
    const int S = 2 * T;
    int Lmax = S;
    for (int s = 0; s < c->up_stages; s++) Lmax *= c->factors[s];
    size_t big = (size_t)T * (3 * Dp > c->pre_ff ? 3 * Dp : c->pre_ff);
    const size_t dec_need = (size_t)S * (3 * Dd > c->dec_ff ? 3 * Dd : c->dec_ff);
    if (dec_need > big) big = dec_need;
    int cw = Dd > c->head_out ? Dd : c->head_out;
    if (2 * c->n_freq > cw) cw = 2 * c->n_freq;
    {
        int L = S;
        for (int s = 0; s < c->up_stages; s++) {
            L *= c->factors[s];
            char nm[96];
            snprintf(nm, sizeof nm, "wave_upsampler.up.%d.weight", s);
            const size_t need = (size_t)L * WN(c, nm, 1);
            if (need > big) big = need;
        }
    }
    if ((size_t)Lmax * cw > big) big = (size_t)Lmax * cw;
    big += 64;
    float *x = (float *)calloc(big, sizeof(float));
    float *h = (float *)calloc(big, sizeof(float));
    float *a = (float *)calloc(big, sizeof(float));
    float *b = (float *)calloc(big, sizeof(float));
    float *f = (float *)calloc(big, sizeof(float));
    int stage = 0, rows = 0, cols = 0;
    char n[256];
#define DONE(buf, r, cc)                                                           \
    do {                                                                           \
        rows = (r), cols = (cc);                                                   \
        if (stage == stop_stage) {                                                 \
            memcpy(out, (buf), sizeof(float) * (size_t)rows * cols);               \
            goto finish;                                                           \
        }                                                                          \
        stage++;                                                                   \
    } while (0)

    int L = S, C = Dd, s_up0 = 0;
    if (start_stage > 0) {
        /* shape of stage start_stage - 1's output, then jump to stage start_stage */
        if (start_stage > mo_codec_n_stages(c) - 1) goto finish;
        int r = T, cc = Dp;
        if (start_stage >= 2) r = T, cc = Dd;
        if (start_stage >= 3) r = S, cc = Dd;
        if (start_stage >= 7) {
            s_up0 = start_stage - 6;
            if (s_up0 > c->up_stages) s_up0 = c->up_stages;
            for (int s = 0; s < s_up0; s++) {
                const int K = c->kernels[s], fac = c->factors[s], trim = (K - fac) / 2;
                snprintf(n, sizeof n, "wave_upsampler.up.%d.weight", s);
                L = (L - 1) * fac + K - 2 * (trim > 0 ? trim : 0);
                C = WN(c, n, 1);
            }
            r = L, cc = C;
        }
        memcpy(x, in, sizeof(float) * (size_t)r * cc);
        stage = start_stage;
        switch (start_stage) {
            case 1: goto st_prenet;
            case 2: goto st_upsample;
            case 3: goto st_prior;
            case 4: goto st_decoder;
            case 5: goto st_post;
            default: break;
        }
        if (start_stage == 7 + c->up_stages) {
            memcpy(h, in, sizeof(float) * (size_t)L * Dd);
            goto st_head;
        }
        if (start_stage == 6 + c->up_stages) goto st_outproj;
        goto st_up;
    }

    /* 1. token embedding (:599-600) */
    {
        const float *emb_tbl = W(c, "token_embd");
        for (int t = 0; t < T; t++) memcpy(x + (size_t)t * Dp, emb_tbl + (size_t)codes[t] * Dp, sizeof(float) * Dp);
    }
    DONE(x, T, Dp);

    /* 2. prenet (:604-618) */
st_prenet:
    {
        const int H = c->pre_heads, hd = Dp / H;
        for (int i = 0; i < c->pre_layers; i++) {
#define PW(s) (snprintf(n, sizeof n, "wave_prenet.blk.%d.%s", i, s), W(c, n))
#define PWR(s) (snprintf(n, sizeof n, "wave_prenet.blk.%d.%s", i, s), WR(c, n))
            layer_norm(x, T, Dp, PW("attn_norm.weight"), PW("attn_norm.bias"), c->eps, h);
            float *q = a, *k = a + (size_t)T * Dp, *v = a + (size_t)2 * T * Dp;
            linear(h, T, Dp, PWR("attn_q.weight"), NULL, Dp, q);
            linear(h, T, Dp, PWR("attn_k.weight"), NULL, Dp, k);
            linear(h, T, Dp, PWR("attn_v.weight"), NULL, Dp, v);
            attention(q, k, v, Dp, T, H, hd, c->pre_win, c->theta, b);
            linear(b, T, Dp, PWR("attn_output.weight"), NULL, Dp, h);
            for (size_t j = 0; j < (size_t)T * Dp; j++) x[j] = x[j] + h[j];
            layer_norm(x, T, Dp, PW("ffn_norm.weight"), PW("ffn_norm.bias"), c->eps, h);
            float *g = a, *u = f;
            linear(h, T, Dp, PWR("ffn_gate.weight"), NULL, c->pre_ff, g);
            linear(h, T, Dp, PWR("ffn_up.weight"), NULL, c->pre_ff, u);
            for (size_t j = 0; j < (size_t)T * c->pre_ff; j++) g[j] = silu(g[j]) * u[j];
            linear(g, T, c->pre_ff, PWR("ffn_down.weight"), NULL, Dp, h);
            for (size_t j = 0; j < (size_t)T * Dp; j++) x[j] = x[j] + h[j];
#undef PW
        }
        layer_norm(x, T, Dp, W(c, "wave_prenet.norm.weight"), W(c, "wave_prenet.norm.bias"), c->eps, h);
        linear(h, T, Dp, WR(c, "wave_prenet.output.weight"), W(c, "wave_prenet.output.bias"), Dd, x);
    }
    DONE(x, T, Dd);

    /* 3. wave_upsample ConvT k=2 s=2 (:622-626) */
st_upsample:
    conv_transpose1d(x, T, Dd, WR(c, "wave_upsample.weight"), WN(c, "wave_upsample.weight", 0), Dd,
                     2, 0, W(c, "wave_upsample.bias"), h);
    memcpy(x, h, sizeof(float) * (size_t)S * Dd);
    DONE(x, S, Dd);

    /* 4. wave_prior ResNets (:629-637) */
st_prior:
    for (int blk = 0; blk < c->res_blocks; blk++) {
        char p[64];
        snprintf(p, sizeof p, "wave_prior.%d.", blk);
        resnet_block(c, p, x, S, Dd, a, b);
    }
    DONE(x, S, Dd);

    /* 5. AdaLN-Zero decoder (:640-660) */
st_decoder:
    {
        const int H = c->dec_heads, hd = Dd / H, A = c->adaln;
        float *se = (float *)malloc(sizeof(float) * A);
        for (int i = 0; i < A; i++) se[i] = silu(emb[i]);
        float *cond = (float *)malloc(sizeof(float) * 3 * Dd);
        for (int i = 0; i < c->dec_layers; i++) {
#define DW(s) (snprintf(n, sizeof n, "wave_decoder.blk.%d.%s", i, s), W(c, n))
#define DWR(s) (snprintf(n, sizeof n, "wave_decoder.blk.%d.%s", i, s), WR(c, n))
            linear(se, 1, A, DWR("attn_cond.weight"), DW("attn_cond.bias"), 3 * Dd, cond);
            adaln_norm(x, S, Dd, cond, cond + Dd, c->eps, h);
            float *q = a, *k = a + (size_t)S * Dd, *v = a + (size_t)2 * S * Dd;
            linear(h, S, Dd, DWR("attn_q.weight"), NULL, Dd, q);
            linear(h, S, Dd, DWR("attn_k.weight"), NULL, Dd, k);
            linear(h, S, Dd, DWR("attn_v.weight"), NULL, Dd, v);
            attention(q, k, v, Dd, S, H, hd, c->dec_win, c->theta, b);
            linear(b, S, Dd, DWR("attn_output.weight"), NULL, Dd, h);
            for (int m = 0; m < S; m++)
                for (int d = 0; d < Dd; d++) {
                    const size_t j = (size_t)m * Dd + d;
                    const float gh = h[j] * cond[2 * Dd + d];
                    x[j] = x[j] + gh;
                }
            linear(se, 1, A, DWR("ffn_cond.weight"), DW("ffn_cond.bias"), 3 * Dd, cond);
            adaln_norm(x, S, Dd, cond, cond + Dd, c->eps, h);
            float *g = a, *u = f;
            linear(h, S, Dd, DWR("ffn_gate.weight"), NULL, c->dec_ff, g);
            linear(h, S, Dd, DWR("ffn_up.weight"), NULL, c->dec_ff, u);
            for (size_t j = 0; j < (size_t)S * c->dec_ff; j++) g[j] = silu(g[j]) * u[j];
            linear(g, S, c->dec_ff, DWR("ffn_down.weight"), NULL, Dd, h);
            for (int m = 0; m < S; m++)
                for (int d = 0; d < Dd; d++) {
                    const size_t j = (size_t)m * Dd + d;
                    const float gh = h[j] * cond[2 * Dd + d];
                    x[j] = x[j] + gh;
                }
#undef DW
        }
        float *nc = (float *)malloc(sizeof(float) * 2 * Dd);
        linear(se, 1, A, WR(c, "wave_decoder.norm_cond.weight"), W(c, "wave_decoder.norm_cond.bias"), 2 * Dd, nc);
        adaln_norm(x, S, Dd, nc, nc + Dd, c->eps, h);
        memcpy(x, h, sizeof(float) * (size_t)S * Dd);
        free(nc); free(se); free(cond);
    }
    DONE(x, S, Dd);

    /* 6. wave_post ResNets (:663-672) */
st_post:
    for (int blk = 0; blk < c->res_blocks; blk++) {
        char p[64];
        snprintf(p, sizeof p, "wave_post.%d.", blk);
        resnet_block(c, p, x, S, Dd, a, b);
    }
    DONE(x, S, Dd);

    /* 7. upsampler stages (:677-708) */
st_up:
    for (int s = s_up0; s < c->up_stages; s++) {
        const int fac = c->factors[s], K = c->kernels[s], trim = (K - fac) / 2;
        snprintf(n, sizeof n, "wave_upsampler.up.%d.weight", s);
        const int Cout = WN(c, n, 1);
        const wref wt = WR(c, n);
        snprintf(n, sizeof n, "wave_upsampler.up.%d.bias", s);
        conv_transpose1d(x, L, C, wt, K, Cout, fac, trim > 0 ? trim : 0, W(c, n), h);
        L = (L - 1) * fac + K - 2 * (trim > 0 ? trim : 0);
        C = Cout;
        memcpy(x, h, sizeof(float) * (size_t)L * C);
        char na[96], nb[96];
        snprintf(na, sizeof na, "wave_upsampler.snake.%d.alpha", s);
        snprintf(nb, sizeof nb, "wave_upsampler.snake.%d.beta", s);
        snake_rows(x, L, C, W(c, na), W(c, nb), is_f16(c, na), is_f16(c, nb));
        char p[64];
        snprintf(p, sizeof p, "wave_upsampler.resblk.%d.", s);
        resnet_block(c, p, x, L, C, a, b);
        DONE(x, L, C);
    }

    /* 8. out_proj + out_snake (:711-725) */
st_outproj:
    linear(x, L, C, WR(c, "wave_upsampler.out_proj.weight"), W(c, "wave_upsampler.out_proj.bias"), Dd, h);
    snake_rows(h, L, Dd, W(c, "wave_upsampler.out_snake.alpha"), W(c, "wave_upsampler.out_snake.beta"),
               is_f16(c, "wave_upsampler.out_snake.alpha"), is_f16(c, "wave_upsampler.out_snake.beta"));
    DONE(h, L, Dd);

    /* 9. iSTFT head (:728-737) + interleave (:801-808) */
st_head:
    {
        const int nf = c->n_freq;
        linear(h, L, Dd, WR(c, "istft_head.out.weight"), W(c, "istft_head.out.bias"), c->head_out, a);
        float *spec = b;
#pragma omp parallel for schedule(static)
        for (int t = 0; t < L; t++)
            for (int k = 0; k < nf; k++) {
                float mag = expf(a[(size_t)t * c->head_out + k]);
                mag = mag < 0.0f ? 0.0f : (mag > 100.0f ? 100.0f : mag);
                const float ph = a[(size_t)t * c->head_out + nf + k];
                spec[((size_t)t * nf + k) * 2 + 0] = mag * cosf(ph);
                spec[((size_t)t * nf + k) * 2 + 1] = mag * sinf(ph);
            }
        DONE(spec, L, nf * 2);
    }

finish:
    if (out_rows) *out_rows = rows;
    if (out_cols) *out_cols = cols;
    free(x); free(h); free(a); free(b); free(f);
    return stage == stop_stage ? 0 : -3;
#undef DONE
}

int mo_codec_n_stages(const mo_codec *c) { return 8 + c->up_stages; }

int mo_codec_decode_stage(mo_codec *c, const int *codes, int T, const float *emb, int stop_stage, float *out,
                          int *out_rows, int *out_cols) {
    return decode_stages(c, codes, T, emb, 0, NULL, stop_stage, out, out_rows, out_cols);
}

int mo_codec_stage_from(mo_codec *c, const int *codes, int T, const float *emb, int start_stage, const float *in,
                        int stop_stage, float *out, int *out_rows, int *out_cols) {
    if (start_stage < 1 || stop_stage < start_stage) return -4;
    return decode_stages(c, codes, T, emb, start_stage, in, stop_stage, out, out_rows, out_cols);
}

/* Full decode -> spectrogram [S_final][n_freq][2]; returns S_final or < 0 on error. */
int mo_codec_decode(mo_codec *c, const int *codes, int T, const float *emb, float *spec) {
    int rows = 0, cols = 0;
    int rc = mo_codec_decode_stage(c, codes, T, emb, mo_codec_n_stages(c) - 1, spec, &rows, &cols);
    return rc == 0 ? rows : rc;
}
