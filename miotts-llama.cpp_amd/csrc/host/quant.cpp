// ggml block formats on the host (see quant.h).
#include "quant.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "gguf.h"

namespace mio {

float fp16_to_f32(uint16_t h) {
    _Float16 v;
    std::memcpy(&v, &h, 2);
    return (float)v;
}

// ggml_compute_fp32_to_bf16: round to nearest even, NaN kept quiet
uint16_t f32_to_bf16(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    return (uint16_t)((u + (0x7fffu + ((u >> 16) & 1u))) >> 16);
}

uint16_t f32_to_fp16(float f) {
    _Float16 v = (_Float16)f;
    uint16_t h;
    std::memcpy(&h, &v, 2);
    return h;
}

// ggml nearest_int: round half to even via the 1.5*2^23 trick
static inline int nearest_int(float fval) {
    float val = fval + 12582912.f;
    int i;
    std::memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

void quantize_row_q8_0(const float *x, void *vy, int64_t k) {
    BlockQ8_0 *y = (BlockQ8_0 *)vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        float amax = 0.0f;
        for (int j = 0; j < 32; ++j) amax = std::max(amax, std::fabs(x[i * 32 + j]));
        const float d = amax / 127.0f;
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = f32_to_fp16(d);
        for (int j = 0; j < 32; ++j) y[i].qs[j] = (int8_t)roundf(x[i * 32 + j] * id);
    }
}

// ggml quantize_row_q4_0_ref / quantize_row_q5_0_ref: d = max / -8 (-16) with max the
// signed value of largest magnitude, codes min(15 (31), (int8)(x / d + 8.5 (16.5))); Q5_0's
// fifth bits packed into qh (bit j: element j, bit j + 16: element j + 16)
static int64_t block_signed_max(const float *x, int n, float &amax) {
    amax = 0.0f;
    int64_t at = 0;
    for (int j = 0; j < n; ++j)
        if (std::fabs(x[j]) > amax) amax = std::fabs(x[j]), at = j;
    return at;
}
void quantize_row_q4_0(const float *x, void *vy, int64_t k) {
    BlockQ4_0 *y = (BlockQ4_0 *)vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        const float *xb = x + i * 32;
        float amax;
        const float mx = xb[block_signed_max(xb, 32, amax)];
        const float d = mx / -8.0f, id = d ? 1.0f / d : 0.0f;
        y[i].d = f32_to_fp16(d);
        for (int j = 0; j < 16; ++j) {
            const uint8_t a = (uint8_t)std::min(15, (int)(int8_t)(xb[j] * id + 8.5f));
            const uint8_t b = (uint8_t)std::min(15, (int)(int8_t)(xb[16 + j] * id + 8.5f));
            y[i].qs[j] = a | (uint8_t)(b << 4);
        }
    }
}
void quantize_row_q5_0(const float *x, void *vy, int64_t k) {
    BlockQ5_0 *y = (BlockQ5_0 *)vy;
    for (int64_t i = 0; i < k / 32; ++i) {
        const float *xb = x + i * 32;
        float amax;
        const float mx = xb[block_signed_max(xb, 32, amax)];
        const float d = mx / -16.0f, id = d ? 1.0f / d : 0.0f;
        y[i].d = f32_to_fp16(d);
        uint32_t qh = 0;
        for (int j = 0; j < 16; ++j) {
            const uint8_t a = (uint8_t)std::min(31, (int)(int8_t)(xb[j] * id + 16.5f));
            const uint8_t b = (uint8_t)std::min(31, (int)(int8_t)(xb[16 + j] * id + 16.5f));
            y[i].qs[j] = (uint8_t)((a & 0x0F) | ((b & 0x0F) << 4));
            qh |= ((uint32_t)(a & 0x10) >> 4) << j;
            qh |= ((uint32_t)(b & 0x10) >> 4) << (j + 16);
        }
        std::memcpy(y[i].qh, &qh, 4);
    }
}

// the signed codes of one Q4_0 / Q5_0 block (ggml dequantize_row_q4_0 / _q5_0 before * d)
static void block_codes_4_5(uint32_t type, const uint8_t *blk, int8_t (&q)[32], uint16_t &d) {
    std::memcpy(&d, blk, 2);
    if (type == GGML_Q4_0) {
        const uint8_t *qs = blk + 2;
        for (int j = 0; j < 16; ++j) q[j] = (int8_t)((qs[j] & 0x0F) - 8), q[j + 16] = (int8_t)((qs[j] >> 4) - 8);
    } else {
        uint32_t qh;
        std::memcpy(&qh, blk + 2, 4);
        const uint8_t *qs = blk + 6;
        for (int j = 0; j < 16; ++j) {
            q[j] = (int8_t)(((qs[j] & 0x0F) | (((qh >> j) << 4) & 0x10)) - 16);
            q[j + 16] = (int8_t)(((qs[j] >> 4) | ((qh >> (j + 12)) & 0x10)) - 16);
        }
    }
}

bool repacks_to_q8_0(uint32_t type) { return type == GGML_Q4_0 || type == GGML_Q5_0; }

bool repack_to_q8_0(uint32_t type, const void *src, int64_t R, int64_t K, void *dst) {
    if (!repacks_to_q8_0(type) || K % 32) return false;
    const size_t bb = type == GGML_Q4_0 ? sizeof(BlockQ4_0) : sizeof(BlockQ5_0);
    const uint8_t *s = (const uint8_t *)src;
    BlockQ8_0 *y = (BlockQ8_0 *)dst;
    for (int64_t i = 0; i < R * (K / 32); ++i) {
        int8_t q[32];
        block_codes_4_5(type, s + (size_t)i * bb, q, y[i].d);
        std::memcpy(y[i].qs, q, 32);
    }
    return true;
}

// Simplified K-quant quantizers (one pass, min/max scales). Any byte pattern of the
// right layout is a valid model for the synthetic benchmark; these keep the
// dequantized weights close to the generating N(0, s) values.
void quantize_row_q4_K(const float *x, void *vy, int64_t k) {
    BlockQ4_K *y = (BlockQ4_K *)vy;
    for (int64_t i = 0; i < k / 256; ++i) {
        const float *xb = x + i * 256;
        float scales[8], mins[8];
        float max_scale = 0.0f, max_min = 0.0f;
        for (int j = 0; j < 8; ++j) {
            float mn = 0.0f, mx = xb[32 * j];
            for (int l = 0; l < 32; ++l) {
                mn = std::min(mn, xb[32 * j + l]);
                mx = std::max(mx, xb[32 * j + l]);
            }
            if (mx < 0.0f) mx = 0.0f;
            scales[j] = (mx - mn) / 15.0f;
            mins[j] = -mn;
            max_scale = std::max(max_scale, scales[j]);
            max_min = std::max(max_min, mins[j]);
        }
        const float inv_scale = max_scale > 0 ? 63.0f / max_scale : 0.0f;
        const float inv_min = max_min > 0 ? 63.0f / max_min : 0.0f;
        uint8_t ls[8], lm[8];
        for (int j = 0; j < 8; ++j) {
            ls[j] = (uint8_t)std::min(63, std::max(0, nearest_int(inv_scale * scales[j])));
            lm[j] = (uint8_t)std::min(63, std::max(0, nearest_int(inv_min * mins[j])));
        }
        std::memset(y[i].scales, 0, 12);
        for (int j = 0; j < 8; ++j) {
            if (j < 4) {
                y[i].scales[j] = ls[j];
                y[i].scales[j + 4] = lm[j];
            } else {
                y[i].scales[j + 4] = (ls[j] & 0xF) | ((lm[j] & 0xF) << 4);
                y[i].scales[j - 4] |= ((ls[j] >> 4) << 6);
                y[i].scales[j] |= ((lm[j] >> 4) << 6);
            }
        }
        y[i].d = f32_to_fp16(max_scale / 63.0f);
        y[i].dmin = f32_to_fp16(max_min / 63.0f);
        const float d = fp16_to_f32(y[i].d), dmin = fp16_to_f32(y[i].dmin);
        uint8_t L[256];
        for (int j = 0; j < 8; ++j) {
            const float dd = d * ls[j], dm = dmin * lm[j];
            for (int l = 0; l < 32; ++l) {
                int q = dd > 0 ? nearest_int((xb[32 * j + l] + dm) / dd) : 0;
                L[32 * j + l] = (uint8_t)std::min(15, std::max(0, q));
            }
        }
        uint8_t *q = y[i].qs;
        for (int j = 0; j < 256; j += 64) {
            for (int l = 0; l < 32; ++l) q[l] = L[j + l] | (L[j + l + 32] << 4);
            q += 32;
        }
    }
}

void quantize_row_q6_K(const float *x, void *vy, int64_t k) {
    BlockQ6_K *y = (BlockQ6_K *)vy;
    for (int64_t i = 0; i < k / 256; ++i) {
        const float *xb = x + i * 256;
        float scales[16], max_scale = 0.0f;
        for (int j = 0; j < 16; ++j) {
            float amax = 0.0f;
            for (int l = 0; l < 16; ++l) amax = std::max(amax, std::fabs(xb[16 * j + l]));
            scales[j] = amax / 31.0f;
            max_scale = std::max(max_scale, scales[j]);
        }
        const float d = max_scale / 127.0f;
        y[i].d = f32_to_fp16(d);
        const float dh = fp16_to_f32(y[i].d);
        uint8_t L[256];
        for (int j = 0; j < 16; ++j) {
            const int sc = dh > 0 ? std::min(127, std::max(-128, nearest_int(scales[j] / dh))) : 0;
            y[i].scales[j] = (int8_t)sc;
            const float dd = dh * sc;
            for (int l = 0; l < 16; ++l) {
                int q = dd != 0 ? nearest_int(xb[16 * j + l] / dd) : 0;
                q = std::min(31, std::max(-32, q));
                L[16 * j + l] = (uint8_t)(q + 32);
            }
        }
        uint8_t *ql = y[i].ql, *qh = y[i].qh;
        for (int j = 0; j < 256; j += 128) {
            for (int l = 0; l < 32; ++l) {
                const uint8_t q1 = L[j + l] & 0xF, q2 = L[j + l + 32] & 0xF;
                const uint8_t q3 = L[j + l + 64] & 0xF, q4 = L[j + l + 96] & 0xF;
                ql[l] = q1 | (q3 << 4);
                ql[l + 32] = q2 | (q4 << 4);
                qh[l] = (L[j + l] >> 4) | ((L[j + l + 32] >> 4) << 2) | ((L[j + l + 64] >> 4) << 4) |
                        ((L[j + l + 96] >> 4) << 6);
            }
            ql += 64;
            qh += 32;
        }
    }
}

bool quantize_row(uint32_t type, const float *x, void *y, int64_t k) {
    switch (type) {
        case GGML_F32: std::memcpy(y, x, k * 4); return true;
        case GGML_F16:
            for (int64_t i = 0; i < k; ++i) ((uint16_t *)y)[i] = f32_to_fp16(x[i]);
            return true;
        case GGML_BF16:
            for (int64_t i = 0; i < k; ++i) ((uint16_t *)y)[i] = f32_to_bf16(x[i]);
            return true;
        case GGML_Q8_0: quantize_row_q8_0(x, y, k); return true;
        case GGML_Q4_0: quantize_row_q4_0(x, y, k); return true;
        case GGML_Q5_0: quantize_row_q5_0(x, y, k); return true;
        case GGML_Q4_K: quantize_row_q4_K(x, y, k); return true;
        case GGML_Q6_K: quantize_row_q6_K(x, y, k); return true;
        default: return false;
    }
}

// ggml dequantize_row_* (same float expression order)
bool dequantize_row(uint32_t type, const void *vx, float *y, int64_t k) {
    switch (type) {
        case GGML_F32: std::memcpy(y, vx, k * 4); return true;
        case GGML_F16:
            for (int64_t i = 0; i < k; ++i) y[i] = fp16_to_f32(((const uint16_t *)vx)[i]);
            return true;
        case GGML_Q8_0: {
            const BlockQ8_0 *x = (const BlockQ8_0 *)vx;
            for (int64_t i = 0; i < k / 32; ++i) {
                const float d = fp16_to_f32(x[i].d);
                for (int j = 0; j < 32; ++j) y[i * 32 + j] = x[i].qs[j] * d;
            }
            return true;
        }
        case GGML_BF16:
            for (int64_t i = 0; i < k; ++i) {
                const uint32_t u = (uint32_t)((const uint16_t *)vx)[i] << 16;
                std::memcpy(&y[i], &u, 4);
            }
            return true;
        case GGML_Q4_0:
        case GGML_Q5_0: {
            const size_t bb = type == GGML_Q4_0 ? sizeof(BlockQ4_0) : sizeof(BlockQ5_0);
            for (int64_t i = 0; i < k / 32; ++i) {
                int8_t q[32];
                uint16_t dh;
                block_codes_4_5(type, (const uint8_t *)vx + (size_t)i * bb, q, dh);
                const float d = fp16_to_f32(dh);
                for (int j = 0; j < 32; ++j) y[i * 32 + j] = q[j] * d;
            }
            return true;
        }
        case GGML_Q4_K: {
            const BlockQ4_K *x = (const BlockQ4_K *)vx;
            for (int64_t i = 0; i < k / 256; ++i) {
                const uint8_t *q = x[i].qs;
                const float d = fp16_to_f32(x[i].d), min = fp16_to_f32(x[i].dmin);
                int is = 0;
                for (int j = 0; j < 256; j += 64) {
                    uint8_t sc, m;
                    auto gsm = [&](int jj, uint8_t *dd, uint8_t *mm) {
                        const uint8_t *s = x[i].scales;
                        if (jj < 4) {
                            *dd = s[jj] & 63;
                            *mm = s[jj + 4] & 63;
                        } else {
                            *dd = (s[jj + 4] & 0xF) | ((s[jj - 4] >> 6) << 4);
                            *mm = (s[jj + 4] >> 4) | ((s[jj - 0] >> 6) << 4);
                        }
                    };
                    gsm(is + 0, &sc, &m);
                    const float d1 = d * sc, m1 = min * m;
                    gsm(is + 1, &sc, &m);
                    const float d2 = d * sc, m2 = min * m;
                    for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
                    for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
                    q += 32;
                    is += 2;
                }
            }
            return true;
        }
        case GGML_Q6_K: {
            const BlockQ6_K *x = (const BlockQ6_K *)vx;
            for (int64_t i = 0; i < k / 256; ++i) {
                const float d = fp16_to_f32(x[i].d);
                const uint8_t *ql = x[i].ql, *qh = x[i].qh;
                const int8_t *sc = x[i].scales;
                for (int n = 0; n < 256; n += 128) {
                    for (int l = 0; l < 32; ++l) {
                        const int is = l / 16;
                        const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                        const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                        const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                        const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                        y[l + 0] = d * sc[is + 0] * q1;
                        y[l + 32] = d * sc[is + 2] * q2;
                        y[l + 64] = d * sc[is + 4] * q3;
                        y[l + 96] = d * sc[is + 6] * q4;
                    }
                    y += 128;
                    ql += 64;
                    qh += 32;
                    sc += 8;
                }
            }
            return true;
        }
        default: return false;
    }
}

static size_t a16(size_t x) { return (x + 255) / 256 * 256; }

SplitLayout split_layout(uint32_t type, int64_t R, int64_t K) {
    SplitLayout L;
    L.type = type, L.rows = R, L.k = K;
    size_t o = 0;
    auto take = [&](int i, size_t n) {
        L.off[i] = o;
        o = a16(o + n);
    };
    switch (type) {
        case GGML_Q8_0: take(0, (size_t)R * K), take(1, (size_t)R * (K / 32) * 2); break;
        case GGML_Q4_K: take(0, (size_t)R * K / 2), take(1, (size_t)R * (K / 256) * 16); break;
        case GGML_Q6_K:
            take(0, (size_t)R * K / 2), take(1, (size_t)R * K / 4), take(2, (size_t)R * K / 16),
                take(3, (size_t)R * (K / 256) * 2);
            break;
        case GGML_F32: take(0, (size_t)R * K * 4); break;
        case GGML_F16:
        case GGML_BF16: take(0, (size_t)R * K * 2); break;
        default: return L;
    }
    L.bytes = o;
    return L;
}

bool to_split(uint32_t type, const void *src, int64_t R, int64_t K, uint8_t *dst) {
    const SplitLayout L = split_layout(type, R, K);
    if (!L.bytes) return false;
    if (type == GGML_F32 || type == GGML_F16 || type == GGML_BF16) {
        std::memcpy(dst, src, (size_t)R * K * (type == GGML_F32 ? 4 : 2));
        return true;
    }
    const size_t row_bytes = ggml_row_bytes(type, K);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < R; ++r) {
        const uint8_t *row = (const uint8_t *)src + (size_t)r * row_bytes;
        if (type == GGML_Q8_0) {
            const BlockQ8_0 *b = (const BlockQ8_0 *)row;
            int8_t *qs = (int8_t *)(dst + L.off[0]) + (size_t)r * K;
            uint16_t *d = (uint16_t *)(dst + L.off[1]) + (size_t)r * (K / 32);
            for (int64_t i = 0; i < K / 32; ++i) {
                std::memcpy(qs + 32 * i, b[i].qs, 32);
                d[i] = b[i].d;
            }
        } else if (type == GGML_Q4_K) {
            const BlockQ4_K *b = (const BlockQ4_K *)row;
            uint8_t *qs = dst + L.off[0] + (size_t)r * K / 2;
            uint8_t *hd = dst + L.off[1] + (size_t)r * (K / 256) * 16;
            for (int64_t i = 0; i < K / 256; ++i) {
                std::memcpy(qs + 128 * i, b[i].qs, 128);
                std::memcpy(hd + 16 * i, &b[i].d, 2);
                std::memcpy(hd + 16 * i + 2, &b[i].dmin, 2);
                // scales re-packed (same 96 bits) as 4 x 24-bit pairs {sc(2j), m(2j), sc(2j+1),
                // m(2j+1)} at bit 24j, so a lane extracts its pair with one funnel shift
                for (int j = 0; j < 4; ++j) {
                    uint32_t f = 0;
                    for (int t = 0; t < 2; ++t) {
                        const int sj = 2 * j + t;
                        const uint8_t *sc = b[i].scales;
                        const uint32_t d = sj < 4 ? (sc[sj] & 63) : ((sc[sj + 4] & 0xF) | ((sc[sj - 4] >> 6) << 4));
                        const uint32_t m = sj < 4 ? (sc[sj + 4] & 63) : ((sc[sj + 4] >> 4) | ((sc[sj] >> 6) << 4));
                        f |= (d | (m << 6)) << (12 * t);
                    }
                    hd[16 * i + 4 + 3 * j + 0] = (uint8_t)f;
                    hd[16 * i + 4 + 3 * j + 1] = (uint8_t)(f >> 8);
                    hd[16 * i + 4 + 3 * j + 2] = (uint8_t)(f >> 16);
                }
            }
        } else {  // Q6_K
            const BlockQ6_K *b = (const BlockQ6_K *)row;
            uint8_t *ql = dst + L.off[0] + (size_t)r * K / 2;
            uint8_t *qh = dst + L.off[1] + (size_t)r * K / 4;
            int8_t *sc = (int8_t *)(dst + L.off[2]) + (size_t)r * K / 16;
            uint16_t *d = (uint16_t *)(dst + L.off[3]) + (size_t)r * (K / 256);
            for (int64_t i = 0; i < K / 256; ++i) {
                std::memcpy(ql + 128 * i, b[i].ql, 128);
                std::memcpy(qh + 64 * i, b[i].qh, 64);
                // scales re-ordered in lane pairs: pair p = 4n + r -> {scales[8n + r], scales[8n + r + 4]}
                for (int p = 0; p < 8; ++p) {
                    const int n = p >> 2, r = p & 3;
                    sc[16 * i + 2 * p] = b[i].scales[8 * n + r];
                    sc[16 * i + 2 * p + 1] = b[i].scales[8 * n + r + 4];
                }
                d[i] = b[i].d;
            }
        }
    }
    return true;
}

}  // namespace mio
