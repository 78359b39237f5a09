/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of one llama_decode step (test-to-speech.cpp:178-185, :589-596) for the
 * GGUF architectures the synthetic models use ("llama": RoPE NORM; "qwen3": RoPE NEOX +
 * per-head q/k RMSNorm; "qwen2": RoPE NEOX + q/k/v projection biases; "lfm2": LiquidAI's
 * hybrid, RoPE NEOX + q/k RMSNorm attention layers interleaved with gated short-conv layers,
 * final norm token_embd_norm), in llama.cpp / ggml CPU semantics [upstream; parity unpinned]:
 *   rms_norm : sum x^2 in double, scale = 1/sqrtf(mean + eps), then * weight
 *   matvec   : activation re-quantized to the weight's vec_dot_type (quant_ref.c)
 *   rope     : theta = pos * base^(-2i/hd) by repeated float multiplication (ggml rope cache)
 *   KV cache : F16 (llama.cpp default cache type); q rounded to f16 for Q.K^T (ggml converts
 *              src1 to the F16 vec_dot_type), f32 accumulation; softmax(s * 1/sqrt(hd)) with the
 *              sum in double; out = sum_t p_t * v_t in f32
 *   ffn      : down(silu(gate x) * up x)
 *   shortconv: (llama.cpp build_shortconv_block) bcx = in_proj(norm(x)) split into B | C | X
 *              (rows [0,n) | [n,2n) | [2n,3n)); bx = B * X; ggml_ssm_conv over the last
 *              l_cache (3) bx of the sequence, per channel sum_j bx[t-2+j] * w[j] accumulated
 *              in f32 from j = 0 (earlier positions of the sequence, zero before it); y = C * conv;
 *              out = out_proj(y) re-quantized like every mul_mat input
 * Sampler: temperature + Gumbel-max over a counter-based hash (mo_sample). llama.cpp's
 * dist sampler draws from the same softmax(logits/T) distribution with mt19937; bit parity
 * of the RNG across backends is not attainable, so the GPU and this oracle
 * share this counter-based sampler and parity is defined on logits and sampled ids.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gguf_ref.h"
#include "mio_oracle.h"

float mo_fp16_to_f32(uint16_t h);
uint16_t mo_f32_to_fp16(float f);
void mo_quantize_q8_0(const float *x, int64_t k, uint16_t *d, int8_t *qs);
void mo_quantize_q8_K(const float *x, int64_t k, float *d, int8_t *qs, int16_t *bsums);
float mo_vec_dot_q8_0(const uint8_t *row, int64_t k, const uint16_t *ad, const int8_t *aq);
float mo_vec_dot_q45_0(uint32_t type, const uint8_t *row, int64_t k, const uint16_t *ad, const int8_t *aq);
float mo_vec_dot_bf16(const uint8_t *row, int64_t k, const uint16_t *xb);
uint16_t mo_f32_to_bf16(float f);
float mo_vec_dot_q4_K(const uint8_t *row, int64_t k, const float *ad, const int8_t *aq, const int16_t *bsums);
float mo_vec_dot_q6_K(const uint8_t *row, int64_t k, const float *ad, const int8_t *aq);
int mo_dequantize_row(uint32_t type, const uint8_t *row, int64_t k, float *y);

typedef struct {
    const mo_tensor *attn_norm, *wq, *wk, *wv, *wo, *q_norm, *k_norm, *ffn_norm, *gate, *up, *down;
    const mo_tensor *bq, *bk, *bv; /* qwen2 projection biases (or NULL) */
    const mo_tensor *conv, *in_proj, *out_proj; /* lfm2 short-conv layer (in_proj != NULL) */
} mo_layer;

struct mo_llm {
    mo_gguf *g;
    int qwen3, neox;
    int n_embd, n_layer, n_head, n_kv, hd, n_ff, n_vocab, n_ctx;
    float base, eps;
    mo_layer *L;
    const mo_tensor *tok, *out_norm, *out;
    uint16_t *kc, *vc;
    int l_cache;       /* lfm2 short-conv kernel width (shortconv.l_cache, 3) */
    float *conv_ring;  /* [n_layer][4][n_embd]: bx of position p in slot p & 3 */
    float *bcx;        /* [3 n_embd] */
    /* activation scratch */
    float *x, *h, *q, *k, *v, *att, *g1, *u1, *q8kd;
    int8_t *q8qs;
    int16_t *q8bs;
    uint16_t *q80d;
};

static const mo_tensor *T(mo_gguf *g, const char *fmt, int i) {
    char n[128];
    snprintf(n, sizeof n, fmt, i);
    return mo_gguf_tensor(g, n);
}

mo_llm *mo_llm_load(const char *path, int n_ctx) {
    mo_gguf *g = mo_gguf_open(path);
    if (!g) return NULL;
    const mo_kv *ak = mo_gguf_kv(g, "general.architecture");
    if (!ak || !ak->str) { mo_gguf_close(g); return NULL; }
    mo_llm *m = (mo_llm *)calloc(1, sizeof(mo_llm));
    m->g = g;
    const char *a = ak->str;
    m->qwen3 = strcmp(a, "qwen3") == 0;
    const int lfm2 = strcmp(a, "lfm2") == 0;
    /* llama.cpp LLM_ARCH_QWEN2 / QWEN3 / LFM2: LLAMA_ROPE_TYPE_NEOX */
    m->neox = m->qwen3 || lfm2 || strcmp(a, "qwen2") == 0;
    char key[128];
#define KI(s, def) (snprintf(key, sizeof key, "%s." s, a), (int)mo_gguf_int(g, key, def))
#define KF(s, def) (snprintf(key, sizeof key, "%s." s, a), (float)mo_gguf_float(g, key, def))
    m->n_embd = KI("embedding_length", 0);
    m->n_layer = KI("block_count", 0);
    m->n_ff = KI("feed_forward_length", 0);
    m->n_head = KI("attention.head_count", 0);
    /* head_count_kv may be a per-layer array (lfm2: 0 on the short-conv layers) */
    snprintf(key, sizeof key, "%s.attention.head_count_kv", a);
    m->n_kv = 0;
    for (int i = 0; i < m->n_layer; i++) {
        const int v = (int)mo_gguf_arr_int(g, key, i, m->n_head);
        if (v > m->n_kv) m->n_kv = v;
    }
    if (m->n_kv == 0) m->n_kv = m->n_head;
    m->l_cache = KI("shortconv.l_cache", 3);
    m->hd = KI("attention.key_length", m->n_head ? m->n_embd / m->n_head : 0);
    m->base = KF("rope.freq_base", 10000.0f);
    m->eps = KF("attention.layer_norm_rms_epsilon", 1e-6f);
#undef KI
#undef KF
    m->tok = mo_gguf_tensor(g, "token_embd.weight");
    m->out_norm = mo_gguf_tensor(g, lfm2 ? "token_embd_norm.weight" : "output_norm.weight");
    m->out = mo_gguf_tensor(g, "output.weight");
    if (!m->out) m->out = m->tok;
    if (!m->tok || !m->out_norm || m->n_layer <= 0) { mo_gguf_close(g); free(m); return NULL; }
    m->n_vocab = (int)m->tok->ne[1];
    m->n_ctx = n_ctx;
    m->L = (mo_layer *)calloc(m->n_layer, sizeof(mo_layer));
    for (int i = 0; i < m->n_layer; i++) {
        mo_layer *l = &m->L[i];
        l->attn_norm = T(g, "blk.%d.attn_norm.weight", i);
        l->wq = T(g, "blk.%d.attn_q.weight", i);
        l->wk = T(g, "blk.%d.attn_k.weight", i);
        l->wv = T(g, "blk.%d.attn_v.weight", i);
        l->wo = T(g, "blk.%d.attn_output.weight", i);
        l->q_norm = T(g, "blk.%d.attn_q_norm.weight", i);
        l->k_norm = T(g, "blk.%d.attn_k_norm.weight", i);
        l->ffn_norm = T(g, "blk.%d.ffn_norm.weight", i);
        l->gate = T(g, "blk.%d.ffn_gate.weight", i);
        l->up = T(g, "blk.%d.ffn_up.weight", i);
        l->down = T(g, "blk.%d.ffn_down.weight", i);
        l->bq = T(g, "blk.%d.attn_q.bias", i);
        l->bk = T(g, "blk.%d.attn_k.bias", i);
        l->bv = T(g, "blk.%d.attn_v.bias", i);
        l->conv = T(g, "blk.%d.shortconv.conv.weight", i);
        l->in_proj = T(g, "blk.%d.shortconv.in_proj.weight", i);
        l->out_proj = T(g, "blk.%d.shortconv.out_proj.weight", i);
        const int conv_ok = l->conv && l->in_proj && l->out_proj && l->conv->type == 0 &&
                            l->conv->ne[0] == m->l_cache;
        const int attn_ok = l->wq && l->wk && l->wv && l->wo;
        if (!l->attn_norm || !(l->in_proj ? conv_ok : attn_ok) || !l->ffn_norm || !l->gate || !l->up || !l->down) {
            mo_gguf_close(g);
            free(m->L);
            free(m);
            return NULL;
        }
    }
    const size_t kv = (size_t)m->n_layer * m->n_kv * n_ctx * m->hd;
    m->kc = (uint16_t *)calloc(kv, 2);
    m->vc = (uint16_t *)calloc(kv, 2);
    m->conv_ring = (float *)calloc((size_t)m->n_layer * 4 * m->n_embd, 4);
    m->bcx = (float *)calloc((size_t)3 * m->n_embd, 4);
    int big = m->n_embd > m->n_ff ? m->n_embd : m->n_ff;
    if (m->n_head * m->hd > big) big = m->n_head * m->hd;
    m->x = (float *)calloc(m->n_embd, 4);
    m->h = (float *)calloc(big, 4);
    m->q = (float *)calloc(m->n_head * m->hd, 4);
    m->k = (float *)calloc(m->n_kv * m->hd, 4);
    m->v = (float *)calloc(m->n_kv * m->hd, 4);
    m->att = (float *)calloc(big, 4);
    m->g1 = (float *)calloc(m->n_ff, 4);
    m->u1 = (float *)calloc(m->n_ff, 4);
    m->q8kd = (float *)calloc(big / 256 + 1, 4);
    m->q8qs = (int8_t *)calloc(big, 1);
    m->q8bs = (int16_t *)calloc(big / 16 + 1, 2);
    m->q80d = (uint16_t *)calloc(big / 32 + 1, 2);
    return m;
}

void mo_llm_free(mo_llm *m) {
    if (!m) return;
    mo_gguf_close(m->g);
    free(m->L); free(m->kc); free(m->vc); free(m->conv_ring); free(m->bcx);
    free(m->x); free(m->h); free(m->q); free(m->k); free(m->v); free(m->att);
    free(m->g1); free(m->u1); free(m->q8kd); free(m->q8qs); free(m->q8bs); free(m->q80d);
    free(m);
}

void mo_llm_info(const mo_llm *m, int *info) {
    info[0] = m->n_vocab; info[1] = m->n_embd; info[2] = m->n_layer; info[3] = m->n_head;
    info[4] = m->n_kv; info[5] = m->hd; info[6] = m->n_ff; info[7] = m->n_ctx;
}

void mo_llm_reset(mo_llm *m) {
    const size_t kv = (size_t)m->n_layer * m->n_kv * m->n_ctx * m->hd;
    memset(m->kc, 0, kv * 2);
    memset(m->vc, 0, kv * 2);
    memset(m->conv_ring, 0, (size_t)m->n_layer * 4 * m->n_embd * 4);
}

/* y = W x for all rows of W (ggml mul_mat semantics incl. activation re-quantization) */
static void matvec(mo_llm *m, const mo_tensor *W, const float *x, float *y) {
    const int64_t K = W->ne[0], R = W->ne[1];
    const size_t rb = W->nbytes / (size_t)R;
    if (W->type == 8) {
        mo_quantize_q8_0(x, K, m->q80d, m->q8qs);
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < R; r++) y[r] = mo_vec_dot_q8_0(W->data + r * rb, K, m->q80d, m->q8qs);
    } else if (W->type == 30) {  /* BF16: vec_dot_type BF16 */
        uint16_t *xh = (uint16_t *)malloc(sizeof(uint16_t) * K);
        for (int64_t i = 0; i < K; i++) xh[i] = mo_f32_to_bf16(x[i]);
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < R; r++) y[r] = mo_vec_dot_bf16(W->data + r * rb, K, xh);
        free(xh);
    } else if (W->type == 2 || W->type == 6) {  /* Q4_0 / Q5_0: vec_dot_type Q8_0 */
        mo_quantize_q8_0(x, K, m->q80d, m->q8qs);
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < R; r++) y[r] = mo_vec_dot_q45_0(W->type, W->data + r * rb, K, m->q80d, m->q8qs);
    } else if (W->type == 12 || W->type == 14) {
        mo_quantize_q8_K(x, K, m->q8kd, m->q8qs, m->q8bs);
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < R; r++)
            y[r] = W->type == 12 ? mo_vec_dot_q4_K(W->data + r * rb, K, m->q8kd, m->q8qs, m->q8bs)
                                 : mo_vec_dot_q6_K(W->data + r * rb, K, m->q8kd, m->q8qs);
    } else if (W->type == 0) {
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < R; r++) {
            const float *w = (const float *)(W->data + r * rb);
            float s = 0;
            for (int64_t i = 0; i < K; i++) s += w[i] * x[i];
            y[r] = s;
        }
    } else {
        fprintf(stderr, "oracle: unsupported weight type %u\n", W->type);
        abort();
    }
}

static void rms_norm(const float *x, int n, const float *w, float eps, float *y) {
    double sum = 0.0;
    for (int i = 0; i < n; i++) sum += (double)(x[i] * x[i]);
    const float mean = (float)(sum / n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int i = 0; i < n; i++) {
        const float v = x[i] * scale;
        y[i] = v * w[i];
    }
}

static void rope(float *x, int hd, int pos, float base, int neox) {
    const float theta_scale = powf(base, -2.0f / hd);
    float theta = (float)pos;
    for (int i = 0; i < hd / 2; i++) {
        const float c = cosf(theta), s = sinf(theta);
        const int i0 = neox ? i : 2 * i, i1 = neox ? i + hd / 2 : 2 * i + 1;
        const float x0 = x[i0], x1 = x[i1];
        x[i0] = x0 * c - x1 * s;
        x[i1] = x0 * s + x1 * c;
        theta *= theta_scale;
    }
}

static inline float silu(float x) { return x / (1.0f + expf(-x)); }

/* the token's embedding row (get_rows of token_embd) */
int mo_llm_embed(mo_llm *m, int token, float *x) {
    if (token < 0 || token >= m->n_vocab) return -1;
    const size_t rb = m->tok->nbytes / (size_t)m->n_vocab;
    return mo_dequantize_row(m->tok->type, m->tok->data + (size_t)token * rb, m->n_embd, x) ? -2 : 0;
}

/* One decoder layer at position pos: x_out = layer(x_in); writes the layer's K/V row `pos`
 * and reads rows [0, pos]. x_out may alias x_in. */
int mo_llm_layer(mo_llm *m, int il, int pos, const float *x_in, float *x_out) {
    if (il < 0 || il >= m->n_layer || pos < 0 || pos >= m->n_ctx) return -1;
    const int D = m->n_embd, H = m->n_head, Hk = m->n_kv, hd = m->hd, F = m->n_ff;
    const float scale = 1.0f / sqrtf((float)hd);
    if (m->x != x_in) memcpy(m->x, x_in, (size_t)D * 4);
    if (m->L[il].in_proj) {
        /* lfm2 gated short-conv block (llama.cpp build_shortconv_block) */
        const mo_layer *l = &m->L[il];
        rms_norm(m->x, D, (const float *)l->attn_norm->data, m->eps, m->h);
        matvec(m, l->in_proj, m->h, m->bcx);
        float *ring = m->conv_ring + (size_t)il * 4 * D;
        const float *w = (const float *)l->conv->data; /* [D][l_cache] */
        const int Lc = m->l_cache;
        for (int i = 0; i < D; i++) {
            const float bx = m->bcx[i] * m->bcx[2 * D + i];
            float sum = 0.0f;
            for (int j = 0; j < Lc; j++) {
                const int p = pos - (Lc - 1) + j;
                const float v = j == Lc - 1 ? bx : (p >= 0 ? ring[(size_t)(p & 3) * D + i] : 0.0f);
                sum += v * w[(size_t)i * Lc + j];
            }
            m->att[i] = m->bcx[D + i] * sum;
            ring[(size_t)(pos & 3) * D + i] = bx;
        }
        matvec(m, l->out_proj, m->att, m->h);
        for (int i = 0; i < D; i++) m->x[i] = m->h[i] + m->x[i];
    } else {
        const mo_layer *l = &m->L[il];
        rms_norm(m->x, D, (const float *)l->attn_norm->data, m->eps, m->h);
        matvec(m, l->wq, m->h, m->q);
        matvec(m, l->wk, m->h, m->k);
        matvec(m, l->wv, m->h, m->v);
        /* qwen2: Qcur = ggml_add(ggml_mul_mat(wq, cur), bq), likewise K and V */
        if (l->bq) for (int i = 0; i < H * hd; i++) m->q[i] += ((const float *)l->bq->data)[i];
        if (l->bk) for (int i = 0; i < Hk * hd; i++) m->k[i] += ((const float *)l->bk->data)[i];
        if (l->bv) for (int i = 0; i < Hk * hd; i++) m->v[i] += ((const float *)l->bv->data)[i];
        for (int h = 0; h < H; h++) {
            if (l->q_norm) rms_norm(m->q + h * hd, hd, (const float *)l->q_norm->data, m->eps, m->q + h * hd);
            rope(m->q + h * hd, hd, pos, m->base, m->neox);
        }
        for (int h = 0; h < Hk; h++) {
            if (l->k_norm) rms_norm(m->k + h * hd, hd, (const float *)l->k_norm->data, m->eps, m->k + h * hd);
            rope(m->k + h * hd, hd, pos, m->base, m->neox);
            uint16_t *kd = m->kc + (((size_t)il * Hk + h) * m->n_ctx + pos) * hd;
            uint16_t *vd = m->vc + (((size_t)il * Hk + h) * m->n_ctx + pos) * hd;
            for (int d = 0; d < hd; d++) {
                kd[d] = mo_f32_to_fp16(m->k[h * hd + d]);
                vd[d] = mo_f32_to_fp16(m->v[h * hd + d]);
            }
        }
#pragma omp parallel for schedule(static)
        for (int h = 0; h < H; h++) {
            const int kvh = h / (H / Hk);
            float qh[512];
            for (int d = 0; d < hd; d++) qh[d] = mo_fp16_to_f32(mo_f32_to_fp16(m->q[h * hd + d]));
            float *s = (float *)malloc(sizeof(float) * (pos + 1));
            float mx = -INFINITY;
            for (int t = 0; t <= pos; t++) {
                const uint16_t *kr = m->kc + (((size_t)il * Hk + kvh) * m->n_ctx + t) * hd;
                float a = 0;
                for (int d = 0; d < hd; d++) a += qh[d] * mo_fp16_to_f32(kr[d]);
                s[t] = a * scale;
                if (s[t] > mx) mx = s[t];
            }
            double sum = 0;
            for (int t = 0; t <= pos; t++) {
                s[t] = expf(s[t] - mx);
                sum += (double)s[t];
            }
            const float inv = (float)(1.0 / sum);
            for (int d = 0; d < hd; d++) {
                float o = 0;
                for (int t = 0; t <= pos; t++) {
                    const uint16_t *vr = m->vc + (((size_t)il * Hk + kvh) * m->n_ctx + t) * hd;
                    o += (s[t] * inv) * mo_fp16_to_f32(vr[d]);
                }
                m->att[h * hd + d] = o;
            }
            free(s);
        }
        matvec(m, l->wo, m->att, m->h);
        for (int i = 0; i < D; i++) m->x[i] = m->h[i] + m->x[i];
    }
    {
        const mo_layer *l = &m->L[il];
        rms_norm(m->x, D, (const float *)l->ffn_norm->data, m->eps, m->h);
        matvec(m, l->gate, m->h, m->g1);
        matvec(m, l->up, m->h, m->u1);
        for (int i = 0; i < F; i++) m->g1[i] = silu(m->g1[i]) * m->u1[i];
        matvec(m, l->down, m->g1, m->h);
        for (int i = 0; i < D; i++) m->x[i] = m->h[i] + m->x[i];
    }
    if (x_out != m->x) memcpy(x_out, m->x, (size_t)D * 4);
    return 0;
}

/* final norm + lm_head of the residual x */
void mo_llm_head(mo_llm *m, const float *x, float *logits) {
    rms_norm(x, m->n_embd, (const float *)m->out_norm->data, m->eps, m->h);
    matvec(m, m->out, m->h, logits);
}

/* lfm2 short-conv ring of layer il, [4][n_embd] (bx of position p in slot p & 3; get / set) */
int mo_llm_conv(mo_llm *m, int il, float *ring, int set) {
    if (il < 0 || il >= m->n_layer) return -1;
    float *r = m->conv_ring + (size_t)il * 4 * m->n_embd;
    if (set)
        memcpy(r, ring, (size_t)4 * m->n_embd * 4);
    else
        memcpy(ring, r, (size_t)4 * m->n_embd * 4);
    return 0;
}

/* 1 when layer il is an lfm2 short-conv layer */
int mo_llm_is_conv(const mo_llm *m, int il) { return il >= 0 && il < m->n_layer && m->L[il].in_proj != NULL; }

/* F16 K / V rows [0, n_pos) of layer il, [n_kv][n_pos][hd] (get: cache -> k, v; set: back) */
int mo_llm_kv(mo_llm *m, int il, int n_pos, uint16_t *k, uint16_t *v, int set) {
    if (il < 0 || il >= m->n_layer || n_pos < 0 || n_pos > m->n_ctx) return -1;
    for (int h = 0; h < m->n_kv; h++) {
        uint16_t *kc = m->kc + (((size_t)il * m->n_kv + h) * m->n_ctx) * m->hd;
        uint16_t *vc = m->vc + (((size_t)il * m->n_kv + h) * m->n_ctx) * m->hd;
        const size_t o = (size_t)h * n_pos * m->hd, n = (size_t)n_pos * m->hd * 2;
        if (set) {
            memcpy(kc, k + o, n);
            memcpy(vc, v + o, n);
        } else {
            memcpy(k + o, kc, n);
            memcpy(v + o, vc, n);
        }
    }
    return 0;
}

int mo_llm_eval(mo_llm *m, int token, int pos, float *logits) {
    if (token < 0 || token >= m->n_vocab || pos < 0 || pos >= m->n_ctx) return -1;
    if (mo_llm_embed(m, token, m->x)) return -2;
    for (int il = 0; il < m->n_layer; il++) mo_llm_layer(m, il, pos, m->x, m->x);
    if (logits) mo_llm_head(m, m->x, logits);
    return 0;
}

/* ---- counter-based Gumbel-max sampler shared with the GPU (llm_kernels.hip) ---- */
static inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

float mo_gumbel(uint64_t seed, int step, int idx) {
    const uint64_t h = mix64(seed ^ mix64(((uint64_t)(uint32_t)step << 32) | (uint32_t)idx));
    const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
    return -logf(-logf(u));
}

/* temperature + Gumbel-max over ids [lo, hi); temp <= 0 -> greedy; ties -> lowest id */
int mo_sample(const float *logits, float temp, uint64_t seed, int step, int lo, int hi) {
    int arg = lo;
    float best = -INFINITY;
    for (int i = lo; i < hi; i++) {
        const float s = temp > 0.0f ? logits[i] / temp + mo_gumbel(seed, step, i) : logits[i];
        if (s > best) {
            best = s;
            arg = i;
        }
    }
    return arg;
}

/* OpenMP threads of every oracle loop (bench.py cpu_baseline times 16 and 4 threads);
 * returns the previous maximum. */
#include <omp.h>
int mo_set_threads(int n) {
    const int prev = omp_get_max_threads();
    if (n > 0) omp_set_num_threads(n);
    return prev;
}

/* test infrastructure: the last mo_llm_layer's intermediates (0: attention output [H*hd],
 * 1: ffn activation silu(g)*u [n_ff], 2: q after norm/RoPE [H*hd]) */
int mo_llm_debug(const mo_llm *m, int which, float *out) {
    const float *src = which == 0 ? m->att : (which == 1 ? m->g1 : (which == 2 ? m->q : NULL));
    const int n = which == 1 ? m->n_ff : m->n_head * m->hd;
    if (!src) return -1;
    memcpy(out, src, (size_t)n * 4);
    return n;
}
