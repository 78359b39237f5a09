/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * ggml block formats and the CPU matmul arithmetic llama_decode runs through
 * (ggml-quants.c scalar/reference semantics, [upstream]; llama.cpp is absent, SURVEY F1,
 * so this restatement is "parity unpinned"; the block layouts are the public ggml spec,
 * SURVEY Appendix B):
 *   - activations are re-quantized to the weight's vec_dot_type before the dot:
 *       Q8_0 weights -> Q8_0 activations (quantize_row_q8_0_ref: d = amax/127 stored f16,
 *                       q = roundf(x / d_f32))
 *       Q4_K / Q6_K  -> Q8_K activations (quantize_row_q8_K_ref: iscale = -127/max_signed,
 *                       q = min(127, nearest_int(iscale*x)), d = 1/iscale f32, bsums/16)
 *   - vec_dot_q8_0_q8_0 : sum_b (float)isum_b * (dw_b * da_b)
 *   - vec_dot_bf16 (vec_dot_type BF16): the activation rounded to bf16
 *       (ggml_compute_fp32_to_bf16, nearest even), sum_i of the f32 products w_i * x_i
 *       accumulated in double (ggml_float) in element order
 *   - vec_dot_q4_0_q8_0 / vec_dot_q5_0_q8_0 (vec_dot_type Q8_0): per block
 *       (dw_b * da_b) * (isum over the low 16 codes + isum over the high 16), codes
 *       (nibble - 8) / (nibble | fifth bit from qh) - 16
 *   - vec_dot_q4_K_q8_K : per superblock d*da*sum_j sc_j*dot_j - dmin*da*sum_j m_j*bsum_j
 *   - vec_dot_q6_K_q8_K : per superblock d*da*sum_j sc_j*dot_j  (q6 - 32)
 * Integer parts are exact; the GPU reproduces them bit-for-bit per superblock.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mio_oracle.h"

float mo_fp16_to_f32(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    uint32_t o;
    if (e == 0) {
        float v = (float)m * (1.0f / 16777216.0f);
        memcpy(&o, &v, 4);
        o |= s;
    } else if (e == 31) {
        o = s | 0x7f800000u | (m << 13);
    } else {
        o = s | ((e - 15 + 127) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &o, 4);
    return f;
}

uint16_t mo_f32_to_fp16(float f) {
    /* RNE via the f16 rounding helper of codec_ref.c */
    const float r = mo_f16_round(f);
    uint32_t x;
    memcpy(&x, &r, 4);
    const uint32_t s = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(s | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    if (ax < 0x38800000u) { /* subnormal half */
        float af;
        memcpy(&af, &ax, 4);
        return (uint16_t)(s | (uint32_t)(af * 16777216.0f));
    }
    return (uint16_t)(s | (((ax >> 23) - 127 + 15) << 10) | ((ax >> 13) & 0x3ff));
}

static inline int nearest_int(float fval) {
    float val = fval + 12582912.f;
    int i;
    memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

/* Q8_0 activation block (as ggml block_q8_0) */
void mo_quantize_q8_0(const float *x, int64_t k, uint16_t *d, int8_t *qs) {
    for (int64_t i = 0; i < k / 32; i++) {
        float amax = 0.0f;
        for (int j = 0; j < 32; j++) {
            const float v = fabsf(x[i * 32 + j]);
            if (v > amax) amax = v;
        }
        const float dd = amax / 127.0f;
        const float id = dd ? 1.0f / dd : 0.0f;
        d[i] = mo_f32_to_fp16(dd);
        for (int j = 0; j < 32; j++) qs[i * 32 + j] = (int8_t)roundf(x[i * 32 + j] * id);
    }
}

/* Q8_K activation block (as ggml block_q8_K) */
void mo_quantize_q8_K(const float *x, int64_t k, float *d, int8_t *qs, int16_t *bsums) {
    for (int64_t i = 0; i < k / 256; i++) {
        float max = 0, amax = 0;
        for (int j = 0; j < 256; ++j) {
            const float ax = fabsf(x[i * 256 + j]);
            if (ax > amax) {
                amax = ax;
                max = x[i * 256 + j];
            }
        }
        if (!amax) {
            d[i] = 0;
            memset(qs + i * 256, 0, 256);
            memset(bsums + i * 16, 0, 32);
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < 256; ++j) {
            const int v = nearest_int(iscale * x[i * 256 + j]);
            qs[i * 256 + j] = (int8_t)(v < 127 ? v : 127);
        }
        for (int j = 0; j < 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += qs[i * 256 + j * 16 + ii];
            bsums[i * 16 + j] = (int16_t)sum;
        }
        d[i] = 1 / iscale;
    }
}

/* codes of element j and j + 16 of a Q4_0 (18-byte) / Q5_0 (22-byte) block (ggml
 * dequantize_row_q4_0 / _q5_0 before the scale) */
static void q45_codes(uint32_t type, const uint8_t *blk, int j, int *x0, int *x1) {
    if (type == 2) {
        const uint8_t q = blk[2 + j];
        *x0 = (q & 0x0F) - 8;
        *x1 = (q >> 4) - 8;
    } else {
        uint32_t qh;
        memcpy(&qh, blk + 2, 4);
        const uint8_t q = blk[6 + j];
        const uint32_t h0 = ((qh & (1u << j)) >> j) << 4;
        const uint32_t h1 = (qh & (1u << (j + 16))) >> (j + 12);
        *x0 = (int)((q & 0x0F) | h0) - 16;
        *x1 = (int)((q >> 4) | h1) - 16;
    }
}

/* vec_dot_q4_0_q8_0 / vec_dot_q5_0_q8_0 */
float mo_vec_dot_q45_0(uint32_t type, const uint8_t *row, int64_t k, const uint16_t *ad, const int8_t *aq) {
    const int bb = type == 2 ? 18 : 22;
    float sumf = 0;
    for (int64_t b = 0; b < k / 32; b++) {
        const uint8_t *blk = row + b * bb;
        uint16_t dw;
        memcpy(&dw, blk, 2);
        int sumi0 = 0, sumi1 = 0;
        for (int j = 0; j < 16; j++) {
            int x0, x1;
            q45_codes(type, blk, j, &x0, &x1);
            sumi0 += x0 * aq[b * 32 + j];
            sumi1 += x1 * aq[b * 32 + j + 16];
        }
        sumf += (mo_fp16_to_f32(dw) * mo_fp16_to_f32(ad[b])) * (float)(sumi0 + sumi1);
    }
    return sumf;
}

/* ggml_compute_fp32_to_bf16 / GGML_BF16_TO_FP32 */
uint16_t mo_f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    return (uint16_t)((u + (0x7fffu + ((u >> 16) & 1u))) >> 16);
}
static float bf16_to_f32(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* vec_dot_bf16 over a bf16 weight row and the bf16-rounded activation xb */
float mo_vec_dot_bf16(const uint8_t *row, int64_t k, const uint16_t *xb) {
    double sumf = 0;
    for (int64_t i = 0; i < k; i++) {
        uint16_t w;
        memcpy(&w, row + 2 * i, 2);
        sumf += (double)(bf16_to_f32(w) * bf16_to_f32(xb[i]));
    }
    return (float)sumf;
}

/* row dot products; x = one weight row in GGUF block layout */
float mo_vec_dot_q8_0(const uint8_t *row, int64_t k, const uint16_t *ad, const int8_t *aq) {
    float sumf = 0;
    for (int64_t b = 0; b < k / 32; b++) {
        const uint8_t *blk = row + b * 34;
        uint16_t dw;
        memcpy(&dw, blk, 2);
        const int8_t *q = (const int8_t *)(blk + 2);
        int sumi = 0;
        for (int j = 0; j < 32; j++) sumi += q[j] * aq[b * 32 + j];
        sumf += sumi * (mo_fp16_to_f32(dw) * mo_fp16_to_f32(ad[b]));
    }
    return sumf;
}

static void get_scale_min_k4(int j, const uint8_t *q, uint8_t *d, uint8_t *m) {
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

/* per-superblock integer parts (exposed for exactness tests) */
void mo_q4k_superblock_ints(const uint8_t *blk, const int8_t *aq, const int16_t *bsums, int *isum,
                            int *imin) {
    const uint8_t *scales = blk + 4, *qs = blk + 16;
    int s = 0, mn = 0;
    for (int j = 0; j < 8; j++) {
        uint8_t sc, m;
        get_scale_min_k4(j, scales, &sc, &m);
        const int chunk = j / 2, hi = j & 1;
        int dot = 0;
        for (int l = 0; l < 32; l++) {
            const int q = hi ? (qs[32 * chunk + l] >> 4) : (qs[32 * chunk + l] & 0xF);
            dot += q * aq[32 * j + l];
        }
        s += sc * dot;
        mn += m * (bsums[2 * j] + bsums[2 * j + 1]);
    }
    *isum = s;
    *imin = mn;
}

float mo_vec_dot_q4_K(const uint8_t *row, int64_t k, const float *ad, const int8_t *aq,
                      const int16_t *bsums) {
    float sumf = 0;
    for (int64_t b = 0; b < k / 256; b++) {
        const uint8_t *blk = row + b * 144;
        uint16_t dh, dmh;
        memcpy(&dh, blk, 2);
        memcpy(&dmh, blk + 2, 2);
        int isum, imin;
        mo_q4k_superblock_ints(blk, aq + b * 256, bsums + b * 16, &isum, &imin);
        const float d = mo_fp16_to_f32(dh) * ad[b];
        const float dmin = mo_fp16_to_f32(dmh) * ad[b];
        sumf += d * (float)isum;
        sumf -= dmin * (float)imin;
    }
    return sumf;
}

void mo_q6k_superblock_ints(const uint8_t *blk, const int8_t *aq, int *isum) {
    const uint8_t *ql = blk, *qh = blk + 128;
    const int8_t *sc = (const int8_t *)(blk + 192);
    int8_t a[256];
    for (int n = 0; n < 2; n++)
        for (int l = 0; l < 32; l++) {
            const uint8_t *L = ql + 64 * n, *H = qh + 32 * n;
            a[128 * n + l + 0] = (int8_t)((L[l + 0] & 0xF) | (((H[l] >> 0) & 3) << 4)) - 32;
            a[128 * n + l + 32] = (int8_t)((L[l + 32] & 0xF) | (((H[l] >> 2) & 3) << 4)) - 32;
            a[128 * n + l + 64] = (int8_t)((L[l + 0] >> 4) | (((H[l] >> 4) & 3) << 4)) - 32;
            a[128 * n + l + 96] = (int8_t)((L[l + 32] >> 4) | (((H[l] >> 6) & 3) << 4)) - 32;
        }
    int s = 0;
    for (int j = 0; j < 16; j++) {
        int dot = 0;
        for (int l = 0; l < 16; l++) dot += a[16 * j + l] * aq[16 * j + l];
        s += sc[j] * dot;
    }
    *isum = s;
}

float mo_vec_dot_q6_K(const uint8_t *row, int64_t k, const float *ad, const int8_t *aq) {
    float sumf = 0;
    for (int64_t b = 0; b < k / 256; b++) {
        const uint8_t *blk = row + b * 210;
        uint16_t dh;
        memcpy(&dh, blk + 208, 2);
        int isum;
        mo_q6k_superblock_ints(blk, aq + b * 256, &isum);
        const float d = mo_fp16_to_f32(dh) * ad[b];
        sumf += d * (float)isum;
    }
    return sumf;
}

/* dequantize one GGUF row (ggml dequantize_row_*), used for get_rows (embedding) */
int mo_dequantize_row(uint32_t type, const uint8_t *row, int64_t k, float *y) {
    if (type == 0) {
        memcpy(y, row, 4 * k);
    } else if (type == 1) {
        for (int64_t i = 0; i < k; i++) {
            uint16_t h;
            memcpy(&h, row + 2 * i, 2);
            y[i] = mo_fp16_to_f32(h);
        }
    } else if (type == 8) {
        for (int64_t b = 0; b < k / 32; b++) {
            uint16_t dh;
            memcpy(&dh, row + 34 * b, 2);
            const float d = mo_fp16_to_f32(dh);
            const int8_t *q = (const int8_t *)(row + 34 * b + 2);
            for (int j = 0; j < 32; j++) y[b * 32 + j] = q[j] * d;
        }
    } else if (type == 30) {
        for (int64_t i = 0; i < k; i++) {
            uint16_t h;
            memcpy(&h, row + 2 * i, 2);
            y[i] = bf16_to_f32(h);
        }
    } else if (type == 2 || type == 6) {
        const int bb = type == 2 ? 18 : 22;
        for (int64_t b = 0; b < k / 32; b++) {
            uint16_t dh;
            memcpy(&dh, row + bb * b, 2);
            const float d = mo_fp16_to_f32(dh);
            for (int j = 0; j < 16; j++) {
                int x0, x1;
                q45_codes(type, row + bb * b, j, &x0, &x1);
                y[b * 32 + j] = x0 * d;
                y[b * 32 + j + 16] = x1 * d;
            }
        }
    } else if (type == 12) {
        for (int64_t b = 0; b < k / 256; b++) {
            const uint8_t *blk = row + 144 * b;
            uint16_t dh, mh;
            memcpy(&dh, blk, 2);
            memcpy(&mh, blk + 2, 2);
            const float d = mo_fp16_to_f32(dh), min = mo_fp16_to_f32(mh);
            const uint8_t *q = blk + 16;
            float *yy = y + 256 * b;
            for (int j = 0, is = 0; j < 256; j += 64, is += 2) {
                uint8_t sc, m;
                get_scale_min_k4(is + 0, blk + 4, &sc, &m);
                const float d1 = d * sc, m1 = min * m;
                get_scale_min_k4(is + 1, blk + 4, &sc, &m);
                const float d2 = d * sc, m2 = min * m;
                for (int l = 0; l < 32; ++l) *yy++ = d1 * (q[l] & 0xF) - m1;
                for (int l = 0; l < 32; ++l) *yy++ = d2 * (q[l] >> 4) - m2;
                q += 32;
            }
        }
    } else if (type == 14) {
        for (int64_t b = 0; b < k / 256; b++) {
            const uint8_t *blk = row + 210 * b;
            uint16_t dh;
            memcpy(&dh, blk + 208, 2);
            const float d = mo_fp16_to_f32(dh);
            const uint8_t *ql = blk, *qh = blk + 128;
            const int8_t *sc = (const int8_t *)(blk + 192);
            float *yy = y + 256 * b;
            for (int n = 0; n < 256; n += 128) {
                for (int l = 0; l < 32; ++l) {
                    const int is = l / 16;
                    const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                    const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                    const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                    const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                    yy[l + 0] = d * sc[is + 0] * q1;
                    yy[l + 32] = d * sc[is + 2] * q2;
                    yy[l + 64] = d * sc[is + 4] * q3;
                    yy[l + 96] = d * sc[is + 6] * q4;
                }
                yy += 128;
                ql += 64;
                qh += 32;
                sc += 8;
            }
        }
    } else {
        return -1;
    }
    return 0;
}

/* y[r] = vec_dot(row r, x) with x re-quantized per the weight type (test helper) */
int mo_matvec(uint32_t type, const uint8_t *w, int rows, int64_t k, const float *x, float *y) {
    int8_t *qs = (int8_t *)malloc(k);
    float *dk = (float *)malloc(sizeof(float) * (k / 256 + 1));
    int16_t *bs = (int16_t *)malloc(sizeof(int16_t) * (k / 16 + 1));
    uint16_t *d0 = (uint16_t *)malloc(sizeof(uint16_t) * (k / 32 + 1));
    size_t rb;
    if (type == 8) {
        rb = (size_t)k / 32 * 34;
        mo_quantize_q8_0(x, k, d0, qs);
        for (int r = 0; r < rows; r++) y[r] = mo_vec_dot_q8_0(w + r * rb, k, d0, qs);
    } else if (type == 30) {
        rb = (size_t)k * 2;
        uint16_t *xb = (uint16_t *)malloc(sizeof(uint16_t) * k);
        for (int64_t i = 0; i < k; i++) xb[i] = mo_f32_to_bf16(x[i]);
        for (int r = 0; r < rows; r++) y[r] = mo_vec_dot_bf16(w + r * rb, k, xb);
        free(xb);
    } else if (type == 2 || type == 6) {
        rb = (size_t)k / 32 * (type == 2 ? 18 : 22);
        mo_quantize_q8_0(x, k, d0, qs);
        for (int r = 0; r < rows; r++) y[r] = mo_vec_dot_q45_0(type, w + r * rb, k, d0, qs);
    } else if (type == 12 || type == 14) {
        rb = (size_t)k / 256 * (type == 12 ? 144 : 210);
        mo_quantize_q8_K(x, k, dk, qs, bs);
        for (int r = 0; r < rows; r++)
            y[r] = type == 12 ? mo_vec_dot_q4_K(w + r * rb, k, dk, qs, bs) : mo_vec_dot_q6_K(w + r * rb, k, dk, qs);
    } else {
        free(qs), free(dk), free(bs), free(d0);
        return -1;
    }
    free(qs), free(dk), free(bs), free(d0);
    return 0;
}
