// Probe: Q8_0 x Q8_0 multi-token matvec shapes for the batched decode (8 tokens), gate|up of
// the 2.6B shape (2 x 10752 rows, K 2048). Variants of the 16x16x32 int8 MFMA kernel, all with
// the same per-block integer dots, scale products and balanced 64-leaf summation tree, so their
// outputs must be equal bit for bit; each is timed over repeated launches (HIP events).
//   v0  k_mmq16 as in llm_mmq.hip: 16-row tile per workgroup, 8 waves split K by lane slots,
//       activation scales staged first, gate then up, LDS cross-wave tree
//   v1  v0 with both matrices' loads issued before the scale staging
//   v2  one 16-row tile per WAVE over the whole K (no cross-wave reduction), loads of the next
//       8 blocks in flight while the current 8 are reduced; W waves per workgroup
//   rd  plain 16-B streaming read of the same bytes (bandwidth reference)
// build: make -C tools/micro mmq_probe ; run: tools/micro/mmq_probe [rows] [K] [nt]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float h2f(uint32_t b) {
    _Float16 h;
    uint16_t s = (uint16_t)b;
    __builtin_memcpy(&h, &s, 2);
    return (float)h;
}
__device__ __forceinline__ int tok16(int lane, int i) { return 4 * (lane >> 4) + i; }
__device__ __forceinline__ v4i mfma16(long a, long b, v4i c) { return __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0); }

constexpr int ilog2(int x) { return x <= 1 ? 0 : 1 + ilog2(x / 2); }
template <int L>
struct Tree {
    v4f lv[L > 0 ? L : 1];
    v4f result;
    template <int I>
    __device__ __forceinline__ void push(v4f x) {
        if constexpr (L >= 1 && (I & 1)) x = lv[0] + x;
        if constexpr (L >= 2 && (I & 3) == 3) x = lv[1] + x;
        if constexpr (L >= 3 && (I & 7) == 7) x = lv[2] + x;
        if constexpr (L >= 4 && (I & 15) == 15) x = lv[3] + x;
        if constexpr (L >= 5 && (I & 31) == 31) x = lv[4] + x;
        if constexpr (L >= 6 && (I & 63) == 63) x = lv[5] + x;
        constexpr int lvl = (I & 1) == 0 ? 0 : (I & 3) != 3 ? 1 : (I & 7) != 7 ? 2 : (I & 15) != 15 ? 3
                          : (I & 31) != 31 ? 4 : (I & 63) != 63 ? 5 : 6;
        if constexpr (lvl < L) lv[lvl] = x;
        else result = x;
    }
};

struct Args {
    const int8_t *w[2];
    const uint16_t *d[2];
    const char *act;  // per token: K int8 | K/32 f32
    size_t as;
    int K, R, nt;
    float *out[2];  // [nt][R]
};

// ---------------------------------------------------------------- v0 / v1
__device__ __forceinline__ void q80_load16(const Args &a, int m, int row, int k, const int8_t *aq, long *w, long *ac,
                                           float *dw) {
    const int g = (threadIdx.x & 63) >> 4, nb = a.K >> 5;
    const int8_t *qrow = a.w[m] + (size_t)row * a.K;
    const uint16_t *drow = a.d[m] + (size_t)row * nb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int b = min(8 * k + i, nb - 1);
        w[i] = *reinterpret_cast<const long *>(qrow + (size_t)b * 32 + 8 * g);
        ac[i] = *reinterpret_cast<const long *>(aq + b * 32 + 8 * g);
        dw[i] = h2f(drow[b]);
    }
}
__device__ __forceinline__ v4f q80_sum16(const long *w, const long *ac, const float *dw, int nb, int k, const float *da) {
    const int lane = threadIdx.x & 63;
    Tree<3> t;
    auto one = [&]<int i>() {
        const int b = 8 * k + i;
        v4f v = {};
        if (b < nb) {
            const v4i c = mfma16(ac[i], w[i], v4i{});
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (float)c[j] * (dw[i] * da[b * 16 + tok16(lane, j)]);
        }
        t.template push<i>(v4f{} + v);
    };
    one.template operator()<0>();
    one.template operator()<1>();
    one.template operator()<2>();
    one.template operator()<3>();
    one.template operator()<4>();
    one.template operator()<5>();
    one.template operator()<6>();
    one.template operator()<7>();
    return t.result;
}

__device__ __forceinline__ v4f tree8_lds(const float *red, int lane) {
    Tree<3> t;
    auto leaf = [&]<int kk>() { t.template push<kk>(*reinterpret_cast<const v4f *>(&red[(kk * 64 + lane) * 4])); };
    leaf.template operator()<0>();
    leaf.template operator()<1>();
    leaf.template operator()<2>();
    leaf.template operator()<3>();
    leaf.template operator()<4>();
    leaf.template operator()<5>();
    leaf.template operator()<6>();
    leaf.template operator()<7>();
    return t.result;
}

__device__ __forceinline__ void store_out(const Args &a, int m, int row0, v4f y) {
    const int lane = threadIdx.x & 63, orow = row0 + (lane & 15);
    if (orow >= a.R) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int t = tok16(lane, j);
        if (t < a.nt) a.out[m][(size_t)t * a.R + orow] = y[j];
    }
}

template <bool EARLY>
__global__ __launch_bounds__(512) void k_v01(Args a) {
    __shared__ float red[2][512 * 4];
    __shared__ float da[64 * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = blockIdx.x * 16, row = min(row0 + (lane & 15), a.R - 1);
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = a.K >> 5;
    const int8_t *aq = reinterpret_cast<const int8_t *>(a.act + (size_t)min(lane & 15, a.nt - 1) * a.as);
    long w0[8], c0[8], w1[8], c1[8];
    float d0[8], d1[8];
    if constexpr (EARLY) {
        q80_load16(a, 0, row, k, aq, w0, c0, d0);
        q80_load16(a, 1, row, k, aq, w1, c1, d1);
    }
    for (int e = threadIdx.x; e < nb * 16; e += 512) {
        const int b = e / 16, t = min(e % 16, a.nt - 1);
        da[e] = reinterpret_cast<const float *>(a.act + (size_t)t * a.as + a.K)[b];
    }
    __syncthreads();
    if constexpr (!EARLY) q80_load16(a, 0, row, k, aq, w0, c0, d0);
    const v4f y0 = q80_sum16(w0, c0, d0, nb, k, da);
    *reinterpret_cast<v4f *>(&red[0][(wave * 64 + lane) * 4]) = y0;
    if constexpr (!EARLY) q80_load16(a, 1, row, k, aq, w1, c1, d1);
    const v4f y1 = q80_sum16(w1, c1, d1, nb, k, da);
    *reinterpret_cast<v4f *>(&red[1][(wave * 64 + lane) * 4]) = y1;
    __syncthreads();
    if (wave != 0) return;
    store_out(a, 0, row0, tree8_lds(red[0], lane));
    store_out(a, 1, row0, tree8_lds(red[1], lane));
}

// ---------------------------------------------------------------- v2: a 16-row tile per wave
struct Batch {
    long w0[8], w1[8], ac[8];
    float d0[8], d1[8];
};
__device__ __forceinline__ void batch_load(const Args &a, int row, int j, const int8_t *aq, Batch &B) {
    const int g = (threadIdx.x & 63) >> 4, nb = a.K >> 5;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int b = min(8 * j + i, nb - 1);
        B.w0[i] = *reinterpret_cast<const long *>(a.w[0] + (size_t)row * a.K + (size_t)b * 32 + 8 * g);
        B.w1[i] = *reinterpret_cast<const long *>(a.w[1] + (size_t)row * a.K + (size_t)b * 32 + 8 * g);
        B.ac[i] = *reinterpret_cast<const long *>(aq + b * 32 + 8 * g);
        B.d0[i] = h2f(a.d[0][(size_t)row * nb + b]);
        B.d1[i] = h2f(a.d[1][(size_t)row * nb + b]);
    }
}

template <int W>
__global__ __launch_bounds__(64 * W) void k_v2(Args a) {
    __shared__ float da[64 * 16];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int row0 = (blockIdx.x * W + wave) * 16, row = min(row0 + (lane & 15), a.R - 1);
    const int nb = a.K >> 5;
    const int8_t *aq = reinterpret_cast<const int8_t *>(a.act + (size_t)min(lane & 15, a.nt - 1) * a.as);
    Batch B[2];
    batch_load(a, row, 0, aq, B[0]);
    for (int e = threadIdx.x; e < nb * 16; e += 64 * W) {
        const int b = e / 16, t = min(e % 16, a.nt - 1);
        da[e] = reinterpret_cast<const float *>(a.act + (size_t)t * a.as + a.K)[b];
    }
    __syncthreads();
    Tree<6> t0, t1;
    auto batch = [&]<int J>() {
        if constexpr (J + 1 < 8) batch_load(a, row, J + 1, aq, B[(J + 1) & 1]);
        const Batch &c = B[J & 1];
        auto one = [&]<int i>() {
            const int b = 8 * J + i;
            v4f v0 = {}, v1 = {};
            if (b < nb) {
                const v4i s0 = mfma16(c.ac[i], c.w0[i], v4i{});
                const v4i s1 = mfma16(c.ac[i], c.w1[i], v4i{});
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float dd = da[b * 16 + tok16(lane, j)];
                    v0[j] = (float)s0[j] * (c.d0[i] * dd);
                    v1[j] = (float)s1[j] * (c.d1[i] * dd);
                }
            }
            t0.template push<8 * J + i>(v4f{} + v0);
            t1.template push<8 * J + i>(v4f{} + v1);
        };
        one.template operator()<0>();
        one.template operator()<1>();
        one.template operator()<2>();
        one.template operator()<3>();
        one.template operator()<4>();
        one.template operator()<5>();
        one.template operator()<6>();
        one.template operator()<7>();
    };
    batch.template operator()<0>();
    batch.template operator()<1>();
    batch.template operator()<2>();
    batch.template operator()<3>();
    batch.template operator()<4>();
    batch.template operator()<5>();
    batch.template operator()<6>();
    batch.template operator()<7>();
    store_out(a, 0, row0, t0.result);
    store_out(a, 1, row0, t1.result);
}


// ---------------------------------------------------------------- v3: v2's tile walk, ablations
// F bits: 1 no MFMA / VALU (xor the loads), 2 no scale loads, 4 16-B weight loads (timing only),
// 8 no activation loads. Outputs are garbage (timing only).
template <int F>
__global__ __launch_bounds__(64) void k_v3(Args a) {
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int row0 = blockIdx.x * 16, row = min(row0 + (lane & 15), a.R - 1);
    const int nb = a.K >> 5;
    const int8_t *aq = reinterpret_cast<const int8_t *>(a.act + (size_t)min(lane & 15, a.nt - 1) * a.as);
    v4i acc = {};
    v4f facc = {};
    constexpr int NB = (F & 4) ? 4 : 8;  // 16-B loads: half the instructions per 8 blocks
    for (int j = 0; j < 8; ++j) {
        long w0[8], w1[8], ac[8];
        float d0[8], d1[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int b = min(8 * j + i, nb - 1);
            if constexpr (F & 4) {
                if (i < NB) {
                    const v4i x0 = *reinterpret_cast<const v4i *>(a.w[0] + (size_t)row * a.K + (size_t)(8 * j + 2 * i) * 32 + 16 * (g & 1) + 32 * (g >> 1));
                    const v4i x1 = *reinterpret_cast<const v4i *>(a.w[1] + (size_t)row * a.K + (size_t)(8 * j + 2 * i) * 32 + 16 * (g & 1) + 32 * (g >> 1));
                    w0[2 * i] = ((long)x0.x << 32) | (uint32_t)x0.y, w0[2 * i + 1] = ((long)x0.z << 32) | (uint32_t)x0.w;
                    w1[2 * i] = ((long)x1.x << 32) | (uint32_t)x1.y, w1[2 * i + 1] = ((long)x1.z << 32) | (uint32_t)x1.w;
                }
            } else {
                w0[i] = *reinterpret_cast<const long *>(a.w[0] + (size_t)row * a.K + (size_t)b * 32 + 8 * g);
                w1[i] = *reinterpret_cast<const long *>(a.w[1] + (size_t)row * a.K + (size_t)b * 32 + 8 * g);
            }
            ac[i] = (F & 8) ? (long)i : *reinterpret_cast<const long *>(aq + b * 32 + 8 * g);
            d0[i] = (F & 2) ? 1.0f : h2f(a.d[0][(size_t)row * nb + b]);
            d1[i] = (F & 2) ? 1.0f : h2f(a.d[1][(size_t)row * nb + b]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (F & 1) {
                acc.x ^= (int)w0[i] ^ (int)(w1[i] >> 7) ^ (int)ac[i];
                facc.x += d0[i] + d1[i];
            } else {
                const v4i s0 = mfma16(ac[i], w0[i], v4i{});
                const v4i s1 = mfma16(ac[i], w1[i], v4i{});
#pragma unroll
                for (int q = 0; q < 4; ++q) facc[q] += (float)s0[q] * d0[i] + (float)s1[q] * d1[i];
            }
        }
    }
    if (acc.x == 0x7fffffff || facc.x == 1.2345f) a.out[0][row] = facc.x + acc.x;
}

// ---------------------------------------------------------------- v4: v0 with 16-B loads
// Lane (row / token l & 15, group g = l >> 4) loads 16 B at byte 16 g of a 64-B block pair
// (b, b + 1): groups 0, 1 hold block b, groups 2, 3 block b + 1. One v_permlane32_swap per
// dword swaps the high 8 B of lanes 0-31 with the low 8 B of lanes 32-63, after which the low
// halves of the 4 groups are block b's bytes {0-7, 16-23, 8-15, 24-31} and the high halves
// block b + 1's: one 16x16x32 MFMA per block, the same exact integer dot. Weight scales: one
// 16-B load of 8 consecutive f16 per lane.
__device__ __forceinline__ void swap_halves(v4i &x) {
    const auto p = __builtin_amdgcn_permlane32_swap(x.x, x.z, false, false);
    const auto q = __builtin_amdgcn_permlane32_swap(x.y, x.w, false, false);
    x.x = p[0], x.z = p[1], x.y = q[0], x.w = q[1];
}
__device__ __forceinline__ long lo8(const v4i &x) { return (long)(uint32_t)x.x | ((long)(uint32_t)x.y << 32); }
__device__ __forceinline__ long hi8(const v4i &x) { return (long)(uint32_t)x.z | ((long)(uint32_t)x.w << 32); }

struct Q80x {
    v4i w[4], a[4];
    v4i ds;  // 8 f16 scales
};
__device__ __forceinline__ void q80x_load(const int8_t *qrow, const uint16_t *drow, const int8_t *aq, int k, Q80x &q,
                                          bool act) {
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        q.w[i] = *reinterpret_cast<const v4i *>(qrow + (size_t)(8 * k + 2 * i) * 32 + 16 * g);
        if (act) q.a[i] = *reinterpret_cast<const v4i *>(aq + (8 * k + 2 * i) * 32 + 16 * g);
    }
    q.ds = *reinterpret_cast<const v4i *>(drow + 8 * k);
}
__device__ __forceinline__ v4f q80x_sum(Q80x &q, const v4i *av, int k, const float *da) {
    const int lane = threadIdx.x & 63;
    Tree<3> t;
#pragma unroll
    for (int i = 0; i < 4; ++i) swap_halves(q.w[i]);
    auto one = [&]<int i>() {
        const int b = 8 * k + i;
        const v4i &w = q.w[i >> 1], &a = av[i >> 1];
        const v4i c = (i & 1) ? mfma16(hi8(a), hi8(w), v4i{}) : mfma16(lo8(a), lo8(w), v4i{});
        const uint32_t dd = (uint32_t)q.ds[i >> 1];
        const float dw = h2f((i & 1) ? dd >> 16 : dd & 0xFFFF);
        v4f v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (float)c[j] * (dw * da[b * 16 + tok16(lane, j)]);
        t.template push<i>(v4f{} + v);
    };
    one.template operator()<0>();
    one.template operator()<1>();
    one.template operator()<2>();
    one.template operator()<3>();
    one.template operator()<4>();
    one.template operator()<5>();
    one.template operator()<6>();
    one.template operator()<7>();
    return t.result;
}

__global__ __launch_bounds__(512) void k_v4(Args a) {
    __shared__ float red[2][512 * 4];
    __shared__ float da[64 * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row0 = blockIdx.x * 16, row = min(row0 + (lane & 15), a.R - 1);
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = a.K >> 5;
    const int8_t *aq = reinterpret_cast<const int8_t *>(a.act + (size_t)min(lane & 15, a.nt - 1) * a.as);
    Q80x q0, q1;
    q80x_load(a.w[0] + (size_t)row * a.K, a.d[0] + (size_t)row * nb, aq, k, q0, true);
    q80x_load(a.w[1] + (size_t)row * a.K, a.d[1] + (size_t)row * nb, aq, k, q1, false);
    for (int e = threadIdx.x; e < nb * 16; e += 512) {
        const int b = e / 16, t = min(e % 16, a.nt - 1);
        da[e] = reinterpret_cast<const float *>(a.act + (size_t)t * a.as + a.K)[b];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) swap_halves(q0.a[i]);
    const v4f y0 = q80x_sum(q0, q0.a, k, da);
    const v4f y1 = q80x_sum(q1, q0.a, k, da);
    *reinterpret_cast<v4f *>(&red[0][(wave * 64 + lane) * 4]) = y0;
    *reinterpret_cast<v4f *>(&red[1][(wave * 64 + lane) * 4]) = y1;
    __syncthreads();
    if (wave != 0) return;
    store_out(a, 0, row0, tree8_lds(red[0], lane));
    store_out(a, 1, row0, tree8_lds(red[1], lane));
}

// v5: v4 with T 16-row tiles per workgroup (8 waves: slot k of every tile), activation loads
// shared by the tiles
template <int T>
__global__ __launch_bounds__(512) void k_v5(Args a) {
    __shared__ float red[2 * T][512 * 4];
    __shared__ float da[64 * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nb = a.K >> 5;
    const int8_t *aq = reinterpret_cast<const int8_t *>(a.act + (size_t)min(lane & 15, a.nt - 1) * a.as);
    Q80x q[2 * T];
    int rows[T];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) {
        rows[tt] = (blockIdx.x * T + tt) * 16;
        const int row = min(rows[tt] + (lane & 15), a.R - 1);
        q80x_load(a.w[0] + (size_t)row * a.K, a.d[0] + (size_t)row * nb, aq, k, q[2 * tt], tt == 0);
        q80x_load(a.w[1] + (size_t)row * a.K, a.d[1] + (size_t)row * nb, aq, k, q[2 * tt + 1], false);
    }
    for (int e = threadIdx.x; e < nb * 16; e += 512) {
        const int b = e / 16, t = min(e % 16, a.nt - 1);
        da[e] = reinterpret_cast<const float *>(a.act + (size_t)t * a.as + a.K)[b];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) swap_halves(q[0].a[i]);
#pragma unroll
    for (int m = 0; m < 2 * T; ++m) {
        const v4f y = q80x_sum(q[m], q[0].a, k, da);
        *reinterpret_cast<v4f *>(&red[m][(wave * 64 + lane) * 4]) = y;
    }
    __syncthreads();
    if (wave >= T) return;
    store_out(a, 0, rows[wave], tree8_lds(red[2 * wave], lane));
    store_out(a, 1, rows[wave], tree8_lds(red[2 * wave + 1], lane));
}

// ---------------------------------------------------------------- v6: general K, W waves
// W waves per 16-row tile, wave k owns slots [k S, k S + S), S = 64 / W (S / 2 block pairs per
// pass); per slot the passes accumulate in order (0 + v_p0 + v_p1 ...), then the slot tree in
// the wave and the wave tree in wave 0: the decode's balanced 64-leaf tree. The next pass's
// loads are in flight while the current one is reduced. LA: activation codes staged in LDS
// (16-B contiguous loads of the nt real rows) instead of per-wave global loads. NV matrices.
template <int S>
struct PassRegs {
    v4i w[2][S / 2];
    v4i a[S / 2];
    uint32_t ds[2][S / 2];  // S f16 scales = S / 2 words, loaded 16 B (or 8 B) at a time
};
template <int W, bool LA, int NV, bool DB = true>
__global__ __launch_bounds__(64 * W) void k_v6(Args a) {
    constexpr int S = 64 / W, PR = S / 2;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    float *red = reinterpret_cast<float *>(lds);                 // [NV][W][64][4]
    float *da = red + NV * W * 256;                              // [nb][16]
    const int nb = a.K >> 5, NP = (nb + 63) / 64;
    int8_t *al = reinterpret_cast<int8_t *>(da + nb * 16);       // [nt][K] when LA
    const int lane = threadIdx.x & 63, g = lane >> 4;
    const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int row0 = blockIdx.x * 16, row = min(row0 + (lane & 15), a.R - 1);
    const int tk = min(lane & 15, a.nt - 1);
    const int8_t *aq = reinterpret_cast<const int8_t *>(a.act + (size_t)tk * a.as);
    auto load = [&](int p, PassRegs<S> &r) {
#pragma unroll
        for (int i = 0; i < PR; ++i) {
            const int b = min(p * 64 + k * S + 2 * i, nb - 2);
#pragma unroll
            for (int m = 0; m < NV; ++m)
                r.w[m][i] = *reinterpret_cast<const v4i *>(a.w[m] + (size_t)row * a.K + (size_t)b * 32 + 16 * g);
            if constexpr (!LA) r.a[i] = *reinterpret_cast<const v4i *>(aq + b * 32 + 16 * g);
        }
        const int b0 = min(p * 64 + k * S, nb - S);
#pragma unroll
        for (int m = 0; m < NV; ++m) {
            const uint16_t *dp = a.d[m] + (size_t)row * nb + b0;
            if constexpr (S >= 8) {
#pragma unroll
                for (int q = 0; q < S / 8; ++q) {
                    const v4i x = *reinterpret_cast<const v4i *>(dp + 8 * q);
                    r.ds[m][4 * q] = x.x, r.ds[m][4 * q + 1] = x.y, r.ds[m][4 * q + 2] = x.z, r.ds[m][4 * q + 3] = x.w;
                }
            } else if constexpr (S == 4) {
                const uint2 x = *reinterpret_cast<const uint2 *>(dp);
                r.ds[m][0] = x.x, r.ds[m][1] = x.y;
            } else {
                r.ds[m][0] = *reinterpret_cast<const uint32_t *>(dp);
            }
        }
    };
    PassRegs<S> R[DB ? 2 : 1];
    load(0, R[0]);
    if constexpr (LA) {
        const int n16 = a.nt * a.K / 16;
        for (int e = threadIdx.x; e < n16; e += 64 * W) {
            const int t = e / (a.K / 16), c = e - t * (a.K / 16);
            *reinterpret_cast<v4i *>(al + (size_t)t * a.K + 16 * c) =
                *reinterpret_cast<const v4i *>(a.act + (size_t)t * a.as + 16 * c);
        }
    }
    for (int e = threadIdx.x; e < a.nt * nb; e += 64 * W) {
        const int t = e / nb, b = e - t * nb;
        da[b * 16 + t] = reinterpret_cast<const float *>(a.act + (size_t)t * a.as + a.K)[b];
    }
    __syncthreads();
    v4f acc[NV][S];
#pragma unroll
    for (int m = 0; m < NV; ++m)
#pragma unroll
        for (int s = 0; s < S; ++s) acc[m][s] = v4f{};
    auto compute = [&](int p, PassRegs<S> &c) {
#pragma unroll
        for (int i = 0; i < PR; ++i) {
            const int b = p * 64 + k * S + 2 * i;
            v4i av;
            if constexpr (LA) av = *reinterpret_cast<const v4i *>(al + (size_t)tk * a.K + (size_t)min(b, nb - 2) * 32 + 16 * g);
            else av = c.a[i];
            swap_halves(av);
#pragma unroll
            for (int m = 0; m < NV; ++m) {
                v4i w = c.w[m][i];
                swap_halves(w);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    v4f v = {};
                    if (b + h < nb) {
                        const v4i cc = h ? mfma16(hi8(av), hi8(w), v4i{}) : mfma16(lo8(av), lo8(w), v4i{});
                        const float dw = h2f(h ? c.ds[m][i] >> 16 : c.ds[m][i] & 0xFFFF);
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = (float)cc[j] * (dw * da[(b + h) * 16 + tok16(lane, j)]);
                    }
                    acc[m][2 * i + h] = acc[m][2 * i + h] + v;
                }
            }
        }
    };
    if constexpr (DB) {
        for (int p = 0; p < NP; p += 2) {
            if (p + 1 < NP) load(p + 1, R[DB ? 1 : 0]);
            compute(p, R[0]);
            if (p + 1 < NP) {
                if (p + 2 < NP) load(p + 2, R[0]);
                compute(p + 1, R[DB ? 1 : 0]);
            }
        }
    } else {
        for (int p = 0; p < NP; ++p) {
            if (p > 0) load(p, R[0]);
            compute(p, R[0]);
        }
    }
#pragma unroll
    for (int m = 0; m < NV; ++m) {
        Tree<ilog2(S)> t;
        auto leaf = [&]<int s>() { if constexpr (s < S) t.template push<s>(acc[m][s]); };
        leaf.template operator()<0>(); leaf.template operator()<1>(); leaf.template operator()<2>();
        leaf.template operator()<3>(); leaf.template operator()<4>(); leaf.template operator()<5>();
        leaf.template operator()<6>(); leaf.template operator()<7>(); leaf.template operator()<8>();
        leaf.template operator()<9>(); leaf.template operator()<10>(); leaf.template operator()<11>();
        leaf.template operator()<12>(); leaf.template operator()<13>(); leaf.template operator()<14>();
        leaf.template operator()<15>();
        *reinterpret_cast<v4f *>(&red[((m * W + k) * 64 + lane) * 4]) = t.result;
    }
    __syncthreads();
    if (k != 0) return;
#pragma unroll
    for (int m = 0; m < NV; ++m) {
        Tree<ilog2(W)> t;
        auto leaf = [&]<int w>() {
            if constexpr (w < W) t.template push<w>(*reinterpret_cast<const v4f *>(&red[((m * W + w) * 64 + lane) * 4]));
        };
        leaf.template operator()<0>(); leaf.template operator()<1>(); leaf.template operator()<2>();
        leaf.template operator()<3>(); leaf.template operator()<4>(); leaf.template operator()<5>();
        leaf.template operator()<6>(); leaf.template operator()<7>(); leaf.template operator()<8>();
        leaf.template operator()<9>(); leaf.template operator()<10>(); leaf.template operator()<11>();
        leaf.template operator()<12>(); leaf.template operator()<13>(); leaf.template operator()<14>();
        leaf.template operator()<15>();
        store_out(a, m, row0, t.result);
    }
}
// ---------------------------------------------------------------- read reference
__global__ __launch_bounds__(256) void k_rd(const uint4 *p, size_t n16, const uint4 *q, size_t m16, uint32_t *sink) {
    int x = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const v4i v = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(p) + i);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < m16; i += stride) {
        const v4i v = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(q) + i);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678) sink[0] = x;
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 10752, K = argc > 2 ? atoi(argv[2]) : 2048, nt = argc > 3 ? atoi(argv[3]) : 8;
    const int NV = argc > 4 ? atoi(argv[4]) : 2;
    if (K % 64 || nt > 16 || R % 16 || K % 256) {
        fprintf(stderr, "need K %% 256 == 0, nt <= 16, R %% 16 == 0\n");
        return 1;
    }
    const int nb = K / 32;
    const size_t as = ((size_t)K + nb * 4 + 15) & ~(size_t)15;
    std::vector<int8_t> hw((size_t)R * K);
    std::vector<uint16_t> hd((size_t)R * nb);
    std::vector<char> hact(as * 16, 0);
    const bool small = K <= 2048;
    uint64_t st = 12345;
    auto rnd = [&]() { st = st * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(st >> 33); };
    Args a{};
    a.K = K, a.R = R, a.nt = nt, a.as = as;
    // NC copies of the weights (> the 256 MB Infinity Cache together): launch i reads copy
    // i % NC, so every launch streams cold HBM as the decode step does
    const size_t wb = (size_t)R * K + (size_t)R * nb * 2;
    const int NC = (int)std::max<size_t>(1, (size_t)(1024ull << 20) / (2 * wb));
    std::vector<Args> copies;
    for (int m = 0; m < 2; ++m) {
        for (auto &v : hw) v = (int8_t)(rnd() & 0xFF);
        for (auto &v : hd) {
            _Float16 h = (_Float16)(0.001f + (rnd() % 1000) * 1e-5f);
            __builtin_memcpy(&v, &h, 2);
        }
        int8_t *dw;
        uint16_t *dd;
        CK(hipMalloc(&dw, hw.size()));
        CK(hipMalloc(&dd, hd.size() * 2));
        CK(hipMemcpy(dw, hw.data(), hw.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dd, hd.data(), hd.size() * 2, hipMemcpyHostToDevice));
        a.w[m] = dw, a.d[m] = dd;
        float *o;
        CK(hipMalloc(&o, (size_t)16 * R * 4));
        a.out[m] = o;
    }
    for (int c = 0; c < NC; ++c) {
        Args ac = a;
        if (c > 0)
            for (int m = 0; m < 2; ++m) {
                int8_t *dw;
                uint16_t *dd;
                CK(hipMalloc(&dw, (size_t)R * K));
                CK(hipMalloc(&dd, (size_t)R * nb * 2));
                CK(hipMemcpy(dw, a.w[m], (size_t)R * K, hipMemcpyDeviceToDevice));
                CK(hipMemcpy(dd, a.d[m], (size_t)R * nb * 2, hipMemcpyDeviceToDevice));
                ac.w[m] = dw, ac.d[m] = dd;
            }
        copies.push_back(ac);
    }
    for (int t = 0; t < 16; ++t) {
        for (int e = 0; e < K; ++e) hact[t * as + e] = (char)(rnd() & 0xFF);
        for (int b = 0; b < nb; ++b) {
            const float f = 0.01f + (rnd() % 1000) * 1e-4f;
            memcpy(&hact[t * as + K + 4 * b], &f, 4);
        }
    }
    char *dact;
    CK(hipMalloc(&dact, hact.size()));
    CK(hipMemcpy(dact, hact.data(), hact.size(), hipMemcpyHostToDevice));
    a.act = dact;
    for (auto &c : copies) c.act = dact;
    uint32_t *sink;
    CK(hipMalloc(&sink, 4));
    const double bytes = NV * ((double)R * K + (double)R * nb * 2);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ref[2];
    auto run = [&](const char *name, auto launch, bool check) {
        for (int m = 0; m < 2; ++m) CK(hipMemset(a.out[m], 0, (size_t)16 * R * 4));
        for (int i = 0; i < NC; ++i) launch(i % NC);
        CK(hipDeviceSynchronize());
        const int it = 20 * NC;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; ++i) launch(i % NC);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        int bad = -1;
        if (check) {
            bad = 0;
            for (int m = 0; m < 2; ++m) {
                std::vector<float> h((size_t)nt * R);
                CK(hipMemcpy(h.data(), a.out[m], h.size() * 4, hipMemcpyDeviceToHost));
                if (ref[m].empty()) ref[m] = h;
                else bad += memcmp(h.data(), ref[m].data(), h.size() * 4) != 0;
            }
        }
        printf("%-14s %8.2f us  %7.1f GB/s  %s\n", name, us, bytes / us * 1e-3,
               bad < 0 ? "" : bad ? "MISMATCH" : "bit-equal");
        fflush(stdout);
    };
    const int tiles = R / 16;
    auto v6 = [&](const char *name, auto kern, int W, bool la) {
        const size_t lds = (size_t)NV * W * 256 * 4 + (size_t)nb * 16 * 4 + (la ? (size_t)nt * K : 0);
        if (lds > 160 * 1024) return;
        if (lds > 64 * 1024) CK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        run(name, [&](int ci) { hipLaunchKernelGGL(kern, dim3(tiles), dim3(64 * W), lds, 0, copies[ci]); }, true);
    };
    if (small && NV == 2) {
        run("v0", [&](int ci) { hipLaunchKernelGGL(k_v01<false>, dim3(tiles), dim3(512), 0, 0, copies[ci]); }, true);
        run("v4", [&](int ci) { hipLaunchKernelGGL(k_v4, dim3(tiles), dim3(512), 0, 0, copies[ci]); }, true);
    }
    if (NV == 2) {
        v6("v6 W8 LA", k_v6<8, true, 2>, 8, true);
        v6("v6 W16 LA", k_v6<16, true, 2>, 16, true);
        v6("s6 W8", k_v6<8, false, 2, false>, 8, false);
        v6("s6 W8 LA", k_v6<8, true, 2, false>, 8, true);
        v6("s6 W16", k_v6<16, false, 2, false>, 16, false);
        v6("s6 W16 LA", k_v6<16, true, 2, false>, 16, true);
    } else {
        v6("v6 W8 LA", k_v6<8, true, 1>, 8, true);
        v6("v6 W16 LA", k_v6<16, true, 1>, 16, true);
        v6("s6 W8", k_v6<8, false, 1, false>, 8, false);
        v6("s6 W8 LA", k_v6<8, true, 1, false>, 8, true);
        v6("s6 W16", k_v6<16, false, 1, false>, 16, false);
        v6("s6 W16 LA", k_v6<16, true, 1, false>, 16, true);
    }
    run("rd", [&](int ci) {
        hipLaunchKernelGGL(k_rd, dim3(1024), dim3(256), 0, 0, (const uint4 *)copies[ci].w[0], (size_t)R * K / 16,
                           (const uint4 *)copies[ci].w[1], NV == 2 ? (size_t)R * K / 16 : 0, sink);
    }, false);
    return 0;
}
