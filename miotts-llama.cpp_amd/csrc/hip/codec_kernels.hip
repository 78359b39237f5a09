// MioCodec decoder kernels for gfx950 (CDNA4), f32 numerics matching the reference's
// ggml CPU graph (miocodec.cpp:204-420, 599-737) up to summation order.
//
//  * gemm_f32_kernel   : C = A * B^T on v_mfma_f32_32x32x2_f32 (exact f32 fma chains, one
//                        per K-group, added once), 64 x 64 tiles, LDS double-buffered with
//                        loads two stages ahead, fused epilogues
//                        (bias / residual / AdaLN gate / SwiGLU / ConvT remap + Snake /
//                        Snake / iSTFT-head polar->complex). The A operand may be a
//                        sliding tap window over consecutive rows (implicit im2col for
//                        ConvTranspose with kernel > stride).
//  * conv_f16_kernel   : Conv1d as implicit GEMM on v_mfma_f32_32x32x16_f16 over the f16
//                        GroupNorm+SiLU activation — exactly ggml's conv_1d (f16 kernel,
//                        f16 im2col, f32 sums).
//  * rownorm_kernel    : ggml_norm (+affine / AdaLN modulate), one wave per row.
//  * gn_partial/apply  : ggml_group_norm statistics (double accumulation) over 64 row
//                        slices, then affine + SiLU -> f16 conv operand.
//  * band_attention    : softmax(QK^T/8 + local mask) V restricted to the |i-j|<=w/2
//                        band (masked entries are exp(-inf)=0 in the reference, so this
//                        is the same function without the S x S work), RoPE applied on load.
#include "codec_kernels.h"

#include <cmath>
#include <cstdlib>
#include <string>
#include <type_traits>

#pragma clang fp contract(off)

namespace mio {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

__device__ __forceinline__ float snake_f(float v, float a, float b) {
    const float ax = v * a;
    const float s = sinf(ax);
    const float s2 = s * s;
    return v + s2 / b;
}

// ---------------------------------------------------------------- f32 GEMM
// (64 WTM) x (64 WTN) output tile per block, 2 x 2 waves of (32 WTM) x (32 WTN) (WTM x WTN
// independent 32 x 32 accumulators per wave), times KG K-groups (256*KG threads).
// A stage is BK = 32*KG deep; K-group kg owns k in [32kg, 32kg + 32) of every stage, so each
// wave runs one exact f32 fma chain (16 v_mfma_f32_32x32x2_f32 per stage) and the KG chains
// are added once, in K-group order, in the epilogue. KG grows as the tile count shrinks so
// that small GEMMs still put 16 waves on every CU. Operands go global -> VGPR -> LDS (float4)
// two stages ahead of the MFMAs; the MFMA reads ds_read_b128 = 4 consecutive k of one row,
// so an octet of k feeds four MFMAs whose lane-half h supplies k = 8o + 4h + q in A and B.
constexpr int GF_T = 64, GF_KD = 32;

// Epilogue of one 32 x 32 accumulator tile (C layout: col = lane&31, row = (r&3) + 8(r>>2) +
// 4(lane>>5)) at rows [rowbase, +32), columns [colbase, +32).
// Residual epilogues (RESID / GATED) read C and the per-column bias / gate: gemm_f32_kernel
// loads them before its K loop (gemm_prefetch), so the epilogue does not open with a global
// round trip after the last MFMA. pre == nullptr: read them here.
struct EpiPre {
    float c[16];
    float col;  // bias[col] (RESID, 0 without bias) or gate[col] (GATED)
};

template <int EPI>
__device__ __forceinline__ void gemm_prefetch(const GemmArgs &g, int rowbase, int colbase, int lane, EpiPre &p) {
    const int col = min(colbase + (lane & 31), g.N - 1);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = min(rowbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), g.M - 1);
        p.c[r] = g.C[(long)row * g.ldc + col];
    }
    if constexpr (EPI == EPI_GATED) {
        p.col = g.aux[col];
    } else {
        const float b = (g.bias ? g.bias : g.C)[col];
        p.col = g.bias ? b : 0.0f;
    }
}

template <int EPI>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs &g, const f32x16 &acc, int rowbase, int colbase,
                                              int lane, const EpiPre *pre = nullptr) {
    const int col = colbase + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = rowbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        float v = acc[r];
        if constexpr (EPI == EPI_SWIGLU || EPI == EPI_HEAD) {
            if constexpr (EPI == EPI_HEAD) v = (col < g.N) ? v + g.bias[col] : 0.0f;
            const float p = __shfl_xor(v, 16);
            if ((lane & 16) == 0 && row < g.M) {
                const int oc = colbase / 2 + (lane & 15);
                if constexpr (EPI == EPI_SWIGLU) {
                    if (oc < g.N / 2) g.C[(long)row * g.ldc + oc] = silu_f(v) * p;
                } else {
                    if (oc < g.cout) {
                        float mag = expf(v);
                        mag = fminf(fmaxf(mag, 0.0f), 100.0f);
                        float *o = g.C + (long)row * g.ldc + 2 * oc;
                        o[0] = mag * cosf(p);
                        o[1] = mag * sinf(p);
                    }
                }
            }
        } else if constexpr (EPI == EPI_CONVT || EPI == EPI_CONVT_SNAKE) {
            if (row < g.M && col < g.N) {
                const int rr = col / g.cout, co = col - rr * g.cout;
                const int orow = g.f * row + rr - g.trim;
                if (orow >= 0 && orow < g.rows_out) {
                    v = v + g.bias[co];
                    if constexpr (EPI == EPI_CONVT_SNAKE) v = snake_f(v, g.aux[co], g.aux2[co]);
                    g.C[(long)orow * g.ldc + co] = v;
                }
            }
        } else {
            if (row < g.M && col < g.N) {
                float *o = g.C + (long)row * g.ldc + col;
                if constexpr (EPI == EPI_STORE) {
                    *o = g.bias ? v + g.bias[col] : v;
                } else if constexpr (EPI == EPI_RESID) {
                    if (pre) {
                        if (g.bias) v = v + pre->col;
                        *o = pre->c[r] + v;
                    } else {
                        if (g.bias) v = v + g.bias[col];
                        *o = *o + v;
                    }
                } else if constexpr (EPI == EPI_GATED) {
                    const float gh = v * (pre ? pre->col : g.aux[col]);
                    *o = (pre ? pre->c[r] : *o) + gh;
                } else if constexpr (EPI == EPI_SNAKE) {
                    v = v + g.bias[col];
                    *o = snake_f(v, g.aux[col], g.aux2[col]);
                }
            }
        }
    }
}


template <int KG, int EPI, int WTM, int WTN>
__global__ __launch_bounds__(256 * KG) void gemm_f32_kernel(GemmArgs g) {
    constexpr int BM = GF_T * WTM, BN = GF_T * WTN, BK = GF_KD * KG, LDK = BK + 4, NT = 256 * KG;
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
    constexpr int AV = BM * BK / 4 / NT, BV = BN * BK / 4 / NT;
    static_assert(AV >= 1 && BV >= 1, "tile");
    static_assert(2 * (BM + BN) * LDK >= (KG - 1) * BM * BN, "reduction area");
    __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDK];
    float *const As = smem, *const Bs = smem + 2 * BM * LDK;

    // XCD-aware tile order: block b runs on XCD b % 8 (round-robin dispatch), so block b takes
    // logical tile (b % 8) * per + b / 8 and each XCD owns one contiguous run of tiles. Tiles
    // are numbered along M first (g.m_major == 0: each XCD gets a slab of N columns, all of A
    // plus 1/8 of B in its L2) or along N first (m_major: a slab of rows, for tall A).
    const int nM = (g.M + BM - 1) / BM, nN = (g.N + BN - 1) / BN, nb = nM * nN, per = (nb + 7) / 8;
    const int t = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (t >= nb) return;
    const int mt = g.m_major ? t / nN : t % nM, nt = g.m_major ? t % nN : t / nM;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave >> 2, wm = (wave >> 1) & 1, wn = wave & 1;
    const int m0 = mt * BM, n0 = nt * BN;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    float4 ra0[AV], rb0[BV], ra1[AV], rb1[BV];
    // Operands through buffer descriptors: an out-of-range load returns zeros in hardware, so
    // a masked element (row past the operand, tap-window row outside [0, a_rows), k past K:
    // its offset is pushed out of range by a select) needs no branch. Every load then issues
    // unconditionally and in order, and the compiler's vmcnt waits for exactly the stage a
    // store consumes instead of draining the stage issued just before (exec-masked loads).
    const auto ra_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(g.A), 0,
                                                          (int)((long)g.a_rows * g.a_seg * 4), 0x00020000);
    const auto rb_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(g.B), 0,
                                                          (int)((long)g.N * g.K * 4), 0x00020000);
    int a_off[AV], a_c[AV], b_off[BV], b_c[BV];
#pragma unroll
    for (int i = 0; i < AV; ++i) {
        const int e = tid + i * NT, m = m0 + e / (BK / 4);
        a_c[i] = (e % (BK / 4)) * 4;
        a_off[i] = ((m + g.a_row_off) * g.a_seg + a_c[i]) * 4;  // negative: out of range
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) {
        const int e = tid + i * NT, n = n0 + e / (BK / 4);
        b_c[i] = (e % (BK / 4)) * 4;
        b_off[i] = (n * g.K + b_c[i]) * 4;
    }
    auto load = [&](int k0, float4 (&ra)[AV], float4 (&rb)[BV]) {
#pragma unroll
        for (int i = 0; i < AV; ++i) {
            const int off = k0 + a_c[i] < g.K ? a_off[i] + k0 * 4 : (int)0x80000000;
            ra[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra_src, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < BV; ++i) {
            const int off = k0 + b_c[i] < g.K ? b_off[i] + k0 * 4 : (int)0x80000000;
            rb[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rb_src, off, 0, 0));
        }
    };
    auto store = [&](int buf, const float4 (&ra)[AV], const float4 (&rb)[BV]) {
#pragma unroll
        for (int i = 0; i < AV; ++i) {
            const int e = tid + i * NT, r = e / (BK / 4), c4 = e % (BK / 4);
            float4 v = ra[i];
            if (g.a_f16) {  // F16 weight: ggml rounds the activation to f16 (exact f32 products)
                v.x = (float)(_Float16)v.x, v.y = (float)(_Float16)v.y;
                v.z = (float)(_Float16)v.z, v.w = (float)(_Float16)v.w;
            }
            *reinterpret_cast<float4 *>(&As[buf * BM * LDK + r * LDK + c4 * 4]) = v;
        }
#pragma unroll
        for (int i = 0; i < BV; ++i) {
            const int e = tid + i * NT, r = e / (BK / 4), c4 = e % (BK / 4);
            *reinterpret_cast<float4 *>(&Bs[buf * BN * LDK + r * LDK + c4 * 4]) = rb[i];
        }
    };
    auto compute = [&](int buf) {
        const float *Ab = As + buf * BM * LDK, *Bb = Bs + buf * BN * LDK;
#pragma unroll
        for (int o = 0; o < GF_KD / 8; ++o) {
            const int kc = kg * GF_KD + o * 8 + 4 * (lane >> 5);
            float4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                a[i] = *reinterpret_cast<const float4 *>(&Ab[(wm * WM + i * 32 + (lane & 31)) * LDK + kc]);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = *reinterpret_cast<const float4 *>(&Bb[(wn * WN + j * 32 + (lane & 31)) * LDK + kc]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
                }
        }
    };

    constexpr bool PRE = EPI == EPI_RESID || EPI == EPI_GATED;
    EpiPre pre[PRE ? TM : 1][PRE ? TN : 1];
    if constexpr (PRE) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) gemm_prefetch<EPI>(g, m0 + wm * WM + i * 32, n0 + wn * WN + j * 32, lane, pre[i][j]);
    }

    // stages past K load zeros (unconditional loads keep the vmcnt ring exact, see load)
    const int nk = (g.K + BK - 1) / BK;
    load(0, ra0, rb0);
    load(BK, ra1, rb1);
    store(0, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
        // even stage: LDS buffer 0; registers 1 hold stage kt+1, registers 0 refill with kt+2
        load((kt + 2) * BK, ra0, rb0);
        compute(0);
        store(1, ra1, rb1);
        __syncthreads();
        if (kt + 1 >= nk) break;
        // odd stage: LDS buffer 1
        load((kt + 3) * BK, ra1, rb1);
        compute(1);
        store(0, ra0, rb0);
        __syncthreads();
    }

    // ---- K-groups 1.. hand their chains to K-group 0 through LDS (same lane, same slot)
    if constexpr (KG > 1) {
        constexpr int SLOT = TM * TN * 16 * 64;
        const int sp = wave & 3;
        if (kg > 0) {
            float *red = smem + ((kg - 1) * 4 + sp) * SLOT;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) red[((i * TN + j) * 16 + r) * 64 + lane] = acc[i][j][r];
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int q = 1; q < KG; ++q) {
            const float *red = smem + ((q - 1) * 4 + sp) * SLOT;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        acc[i][j][r] = acc[i][j][r] + red[((i * TN + j) * 16 + r) * 64 + lane];
        }
    }

    // ---- epilogue (C layout: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
            gemm_epilogue<EPI>(g, acc[i][j], m0 + wm * WM + i * 32, n0 + wn * WN + j * 32, lane,
                               PRE ? &pre[PRE ? i : 0][PRE ? j : 0] : nullptr);
}

// ---------------------------------------------------------------- conv1d f16
// The A operand is the GroupNorm+SiLU activation already rounded to f16 by gn_apply_kernel
// ([L][Cin], one pass instead of once per tap and per column tile), so staging is a plain
// 16 B copy with the tap shift and zero padding. 64 x 64 tile, 128-deep K stages, 4 waves
// of 32 x 32; k runs in ascending 16-chunks per output like ggml's f16 im2col GEMM row.
constexpr int CV_BM = 64, CV_BN = 64, CV_BK = 128, CV_LD = CV_BK + 8;

__global__ __launch_bounds__(256) void conv_f16_kernel(ConvArgs c) {
    __shared__ __attribute__((aligned(16))) _Float16 As[2][CV_BM * CV_LD];
    __shared__ __attribute__((aligned(16))) _Float16 Bs[2][CV_BN * CV_LD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.y * CV_BM, n0 = blockIdx.x * CV_BN;
    const int K = c.taps * c.Cin;
    constexpr int NV = CV_BM * CV_BK / 8 / 256;  // 16 B chunks per thread per operand

    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;

    uint4 ra0[NV], rb0[NV], ra1[NV], rb1[NV];
    // Buffer-descriptor loads as in gemm_f32_kernel: element (m, k = tap Cin + ci) of the tap
    // window sits at Xa[(m - pad) Cin + k], valid exactly when that index is inside [0, L Cin)
    // (the hardware returns zeros outside, the "same" padding); k past K is pushed out of
    // range by a select. No branches around the loads: the vmcnt ring stays exact.
    const auto xa_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(c.Xa), 0,
                                                          (int)((long)c.L * c.Cin * 2), 0x00020000);
    const auto w_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16 *>(c.B), 0,
                                                         (int)((long)c.Cout * K * 2), 0x00020000);
    auto load = [&](int k0, uint4 (&ra)[NV], uint4 (&rb)[NV]) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = tid + i * 256, r = e / (CV_BK / 8), c8 = (e % (CV_BK / 8)) * 8;
            const int k = k0 + c8;
            const int off = k < K ? ((m0 + r - c.pad) * c.Cin + k) * 2 : (int)0x80000000;
            ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xa_src, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = tid + i * 256, r = e / (CV_BK / 8), c8 = (e % (CV_BK / 8)) * 8;
            const int k = k0 + c8;
            const int off = k < K ? ((n0 + r) * K + k) * 2 : (int)0x80000000;
            rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(w_src, off, 0, 0));
        }
    };
    auto store = [&](int buf, const uint4 (&ra)[NV], const uint4 (&rb)[NV]) {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int e = tid + i * 256, r = e / (CV_BK / 8), c8 = (e % (CV_BK / 8)) * 8;
            *reinterpret_cast<uint4 *>(&As[buf][r * CV_LD + c8]) = ra[i];
            *reinterpret_cast<uint4 *>(&Bs[buf][r * CV_LD + c8]) = rb[i];
        }
    };
    auto compute = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < CV_BK; ks += 16) {
            const f16x8 a = *reinterpret_cast<const f16x8 *>(
                &As[buf][(wm * 32 + (lane & 31)) * CV_LD + ks + 8 * (lane >> 5)]);
            const f16x8 b = *reinterpret_cast<const f16x8 *>(
                &Bs[buf][(wn * 32 + (lane & 31)) * CV_LD + ks + 8 * (lane >> 5)]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
        }
    };

    // epilogue operands (bias, residual) loaded before the K loop, off its critical path
    const int col = n0 + wn * 32 + (lane & 31), colc = min(col, c.Cout - 1);
    const float bias = c.bias[colc];
    float res[16];
    const float *rsrc = c.resid ? c.resid : c.bias;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = min(m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), c.L - 1);
        res[r] = rsrc[c.resid ? (long)row * c.Cout + colc : colc];
    }

    const int nk = (K + CV_BK - 1) / CV_BK;
    load(0, ra0, rb0);
    load(CV_BK, ra1, rb1);
    store(0, ra0, rb0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {  // same two-stage register ring as gemm_f32_kernel
        load((kt + 2) * CV_BK, ra0, rb0);
        compute(0);
        store(1, ra1, rb1);
        __syncthreads();
        if (kt + 1 >= nk) break;
        load((kt + 3) * CV_BK, ra1, rb1);
        compute(1);
        store(0, ra0, rb0);
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < c.L && col < c.Cout) {
            float v = acc[r] + bias;
            if (c.resid) v = v + res[r];
            c.Y[(long)row * c.Cout + col] = v;
        }
    }
}

// ---------------------------------------------------------------- row norms
constexpr int RN_MAXPL = 16;  // D <= 1024

// Sum over the 64 lanes of a wave in double, the total in every lane: DPP steps within rows
// (quad xor 1, 2, half-row and row mirrors), row broadcasts 15 / 31 into lane 63, one read.
// ~6 VALU latencies instead of six ds_bpermute round trips per 32-bit half.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ double dpp_f64(double x) {
    const int2 v = __builtin_bit_cast(int2, x);
    const int lo = __builtin_amdgcn_update_dpp(0, v.x, CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, v.y, CTRL, ROWS, 0xF, false);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double wave_sum_f64(double s) {
    s += dpp_f64<0xB1>(s);        // quad_perm [1,0,3,2]
    s += dpp_f64<0x4E>(s);        // quad_perm [2,3,0,1]
    s += dpp_f64<0x141>(s);       // row_half_mirror
    s += dpp_f64<0x140>(s);       // row_mirror
    s += dpp_f64<0x142, 0xA>(s);  // row_bcast:15 -> rows 1, 3
    s += dpp_f64<0x143, 0xC>(s);  // row_bcast:31 -> rows 2, 3
    const int2 v = __builtin_bit_cast(int2, s);
    return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(v.x, 63), __builtin_amdgcn_readlane(v.y, 63)));
}

// One wave per row; NPL = D / 64 values per lane, fixed at compile time so that every load
// is unconditional (a runtime bound put each load behind a branch and a vmcnt(0) drain).
template <int NPL>
__global__ __launch_bounds__(256) void rownorm_kernel(const float *x, float *y, int M, float eps, int mode,
                                                      const float *p0, const float *p1) {
    constexpr int D = NPL * 64;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float *xr = x + (long)row * D;
    float v[NPL], pa[NPL], pb[NPL];
    // the affine / AdaLN parameters are loaded with the row (not after the two reductions:
    // one memory round trip less on the kernel's critical path)
    const float *q0 = mode != 0 ? p0 : xr, *q1 = (mode != 0 && p1) ? p1 : xr;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        v[i] = xr[i * 64 + lane];
        pa[i] = q0[i * 64 + lane];
        pb[i] = q1[i * 64 + lane];
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NPL; ++i) s += (double)v[i];
    s = wave_sum_f64(s);
    const float mean = (float)(s / D);
    double s2 = 0.0;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        v[i] = v[i] - mean;
        s2 += (double)(v[i] * v[i]);
    }
    s2 = wave_sum_f64(s2);
    const float variance = (float)(s2 / D);
    const float scale = 1.0f / sqrtf(variance + eps);
    float *yr = y + (long)row * D;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int d = i * 64 + lane;
        float t = v[i] * scale;
        if (mode == 1) {
            t = t * pa[i];
            if (p1) t = t + pb[i];
        } else if (mode == 2) {
            const float sc = 1.0f + pb[i];
            t = t * sc;
            t = t + pa[i];
        }
        yr[d] = t;
    }
}

// ---------------------------------------------------------------- group norm
// ggml_group_norm (miocodec.cpp GroupNorm -> ggml.c group_norm_f32): mean = (float)(sum x / n)
// in double, variance = (float)(sum (double)fl(fl(x - mean)^2) / n). Rows are cut into P <= 256
// slices (one block each): pass 1 writes per-slice double sums of x, gn_final reduces the P
// partials of every group (fixed order, see gn_final_kernel) into the means; pass 2 and a second gn_final do the same for the squared
// deviations and write rstd; gn_apply writes the f16 conv operand. Kernel boundaries order
// the passes (no grid-wide fences: on 8 XCDs a device-scope release flushes the L2).
// Requires C % 8 == 0, C <= 1024, G <= 64 and cpg | 64 (groups never straddle 64 lanes).
constexpr int GN_PMAX = 256;

// NJ = ceil(C / 64) channel chunks per lane, fixed at compile time: the loads of a row issue
// unconditionally (a runtime bound put every load behind a branch and a vmcnt(0) drain);
// channels past C read an in-range address and are zeroed by a select.
template <int PASS, int NJ>
__global__ __launch_bounds__(256) void gn_partial_kernel(const float *x, int L, int C, int G, int cpg,
                                                         int rows, const float2 *stat, double *part) {
    __shared__ double wsum[4][64];
    const int p = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r0 = p * rows, r1 = min(L, r0 + rows);
    double acc[NJ];
    float mean[NJ];
    bool ok[NJ];
    int ch[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        ok[j] = j * 64 + lane < C;
        ch[j] = ok[j] ? j * 64 + lane : 0;
        acc[j] = 0.0;
        mean[j] = PASS == 2 ? stat[ch[j] / cpg].x : 0.0f;
    }
#pragma unroll 2
    for (int r = r0 + wave; r < r1; r += 4) {
        const float *xr = x + (long)r * C;
        float v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) v[j] = xr[ch[j]];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            if constexpr (PASS == 1) {
                acc[j] += ok[j] ? (double)v[j] : 0.0;
            } else {
                const float d = v[j] - mean[j];
                acc[j] += ok[j] ? (double)(d * d) : 0.0;
            }
        }
    }
    // a group is cpg consecutive lanes of one 64-channel chunk
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        double s = acc[j];
        for (int o = 1; o < cpg; o <<= 1) s += __shfl_xor(s, o);
        if (lane % cpg == 0 && ok[j]) wsum[wave][(j * 64 + lane) / cpg] = s;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += 256)
        part[(long)p * G + g] = ((wsum[0][g] + wsum[1][g]) + wsum[2][g]) + wsum[3][g];
}

// One block: stat[g].x = mean (PASS 1) or stat[g].y = rstd (PASS 2) from the P slice sums;
// 32 lanes per group, lane s takes slices p = s mod 32, then a 5-level xor tree. The slice
// loads issue unconditionally (clamped index, zeroed by a select).
template <int PASS>
__global__ __launch_bounds__(1024) void gn_final_kernel(const double *part, int P, int G, long n,
                                                        float eps, float2 *stat) {
    const int t = threadIdx.x, s32 = t & 31;
    for (int g0 = 0; g0 < G; g0 += 32) {
        const int g = g0 + (t >> 5), gg = g < G ? g : 0;
        double v[GN_PMAX / 32];
#pragma unroll
        for (int i = 0; i < GN_PMAX / 32; ++i) {
            const int q = s32 + 32 * i;
            v[i] = part[(long)(q < P ? q : 0) * G + gg];
        }
        double sum = 0.0;
#pragma unroll
        for (int i = 0; i < GN_PMAX / 32; ++i)
            if (s32 + 32 * i < P) sum += v[i];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sum += __shfl_xor(sum, o);
        if (s32 == 0 && g < G) {
            if constexpr (PASS == 1) {
                stat[g].x = (float)(sum / (double)n);
            } else {
                const float variance = (float)(sum / (double)n);
                stat[g].y = 1.0f / sqrtf(variance + eps);
            }
        }
    }
}

// GroupNorm + SiLU in ONE launch: one 1024-thread workgroup per group (its L x cpg values,
// 4 channels per float4), three passes over them — the double sum and the mean, the double
// sum of fl(fl(x - mean)^2) and rstd (ggml's two-pass formula), then the f16 conv operand —
// the second and third re-reading the group from L2. Replaces the sliced five-launch path
// (partials, final, partials, final, apply) when cpg % 4 == 0: the re-decodes of the
// streaming path are launch-bound, and their GroupNorms were 60 of ~220 launches.
__device__ __forceinline__ double block_sum_f64_1024(double v, double *red) {
    v = wave_sum_f64(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += red[w];
    __syncthreads();  // red is reused by the next reduction
    return t;
}

__global__ __launch_bounds__(1024) void gn_fused_kernel(const float *x, int L, int C, int cpg, int qsh, float eps,
                                                        const float *gamma, const float *beta, _Float16 *xa) {
    __shared__ double red[16];
    constexpr int U = 8;  // quads in flight per thread
    const int g = blockIdx.x, tid = threadIdx.x;
    const int qm = (1 << qsh) - 1;             // quads per row - 1 (cpg / 4 is a power of two)
    const int nq = L << qsh;                   // quads of the group
    const long n = (long)L * cpg;
    const float *xg = x + (long)g * cpg;
    auto at = [&](int e) { return (long)(e >> qsh) * C + 4 * (e & qm); };
    // pass 1: mean
    double s = 0.0;
    for (int base = 0; base < nq; base += 1024 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4 *>(xg + at(min(base + tid + 1024 * u, nq - 1)));
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + tid + 1024 * u < nq) s += ((((double)v[u].x + (double)v[u].y) + (double)v[u].z) + (double)v[u].w);
    }
    const float mean = (float)(block_sum_f64_1024(s, red) / (double)n);
    // pass 2: rstd
    double s2 = 0.0;
    for (int base = 0; base < nq; base += 1024 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4 *>(xg + at(min(base + tid + 1024 * u, nq - 1)));
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + tid + 1024 * u < nq) {
                const float dx = v[u].x - mean, dy = v[u].y - mean, dz = v[u].z - mean, dw = v[u].w - mean;
                s2 += ((((double)(dx * dx) + (double)(dy * dy)) + (double)(dz * dz)) + (double)(dw * dw));
            }
    }
    const float variance = (float)(block_sum_f64_1024(s2, red) / (double)n);
    const float rstd = 1.0f / sqrtf(variance + eps);
    // pass 3: f16(silu((x - mean) * rstd * gamma + beta)), the op order of gn_apply_kernel
    for (int base = 0; base < nq; base += 1024 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4 *>(xg + at(min(base + tid + 1024 * u, nq - 1)));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = base + tid + 1024 * u;
            if (e >= nq) continue;
            const int c = g * cpg + 4 * (e & qm);
            const float t[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            _Float16 o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float y = t[q] - mean;
                y = y * rstd;
                y = y * gamma[c + q];
                y = y + beta[c + q];
                o[q] = (_Float16)silu_f(y);
            }
            uint2 pk;
            __builtin_memcpy(&pk, o, 8);
            *reinterpret_cast<uint2 *>(xa + (long)(e >> qsh) * C + c) = pk;
        }
    }
}

// ---------------------------------------------------------------- group norm, three launches
// The sliced statistics without the two single-workgroup finals: every workgroup of the
// launch after a partial pass reduces the P <= 128 slice sums itself (the same fixed order as
// gn_final_kernel: 32 lanes per group, lane s takes slices s, s + 32, .., then a 5-level xor
// tree), so the redundant copies agree bit for bit. gn_stat2 = means + pass-2 partials (its
// workgroup 0 also stores the means); gn_apply3 = rstd + the f16 operand, 16 channels per
// thread. Both issue their x loads before the reduction. 3 launches per GroupNorm instead of
// 5 (sliced), ~128-256 workgroups each instead of gn_fused's one per group (32 on 256 CUs,
// three dependent passes over a group strided through memory).
constexpr int GN3_PMAX = 128;

// out[g] (LDS) = sum over the P slice partials of group g, g < G (GI * 8 >= G, 256 threads)
template <int GI>
__device__ __forceinline__ void gn_reduce(const double *part, int P, int G, double *out) {
    const int t = threadIdx.x, s32 = t & 31;
    double v[GI][GN3_PMAX / 32];
#pragma unroll
    for (int k = 0; k < GI; ++k) {
        const int g = k * 8 + (t >> 5), gg = g < G ? g : 0;
#pragma unroll
        for (int i = 0; i < GN3_PMAX / 32; ++i) {
            const int q = s32 + 32 * i;
            v[k][i] = part[(long)(q < P ? q : 0) * G + gg];
        }
    }
#pragma unroll
    for (int k = 0; k < GI; ++k) {
        const int g = k * 8 + (t >> 5);
        double sum = 0.0;
#pragma unroll
        for (int i = 0; i < GN3_PMAX / 32; ++i)
            if (s32 + 32 * i < P) sum += v[k][i];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sum += __shfl_xor(sum, o);
        if (s32 == 0 && g < G) out[g] = sum;
    }
    __syncthreads();
}

template <int NJ, int GI>
__global__ __launch_bounds__(256) void gn_stat2_kernel(const float *x, int L, int C, int G, int cpg, int rows, long n,
                                                       const double *part1, double *part2, float2 *stat) {
    __shared__ double red[64];
    __shared__ double wsum[4][64];
    const int p = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r0 = p * rows, r1 = min(L, r0 + rows);
    double acc[NJ];
    float mean[NJ];
    bool ok[NJ];
    int ch[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        ok[j] = j * 64 + lane < C;
        ch[j] = ok[j] ? j * 64 + lane : 0;
        acc[j] = 0.0;
    }
    // the wave's first two rows are in flight while the slice sums are reduced (a row past
    // r1 reads row r0, in range, and is not added)
    float pre[2][NJ];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int r = r0 + wave + 4 * k;
        const float *xr = x + (long)(r < r1 ? r : r0) * C;
#pragma unroll
        for (int j = 0; j < NJ; ++j) pre[k][j] = xr[ch[j]];
    }
    gn_reduce<GI>(part1, gridDim.x, G, red);
    if (p == 0 && threadIdx.x < G) stat[threadIdx.x].x = (float)(red[threadIdx.x] / (double)n);
#pragma unroll
    for (int j = 0; j < NJ; ++j) mean[j] = (float)(red[ch[j] / cpg] / (double)n);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (r0 + wave + 4 * k >= r1) break;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const float d = pre[k][j] - mean[j];
            acc[j] += ok[j] ? (double)(d * d) : 0.0;
        }
    }
#pragma unroll 2
    for (int r = r0 + wave + 8; r < r1; r += 4) {
        const float *xr = x + (long)r * C;
        float v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) v[j] = xr[ch[j]];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const float d = v[j] - mean[j];
            acc[j] += ok[j] ? (double)(d * d) : 0.0;
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        double sm = acc[j];
        for (int o = 1; o < cpg; o <<= 1) sm += __shfl_xor(sm, o);
        if (lane % cpg == 0 && ok[j]) wsum[wave][(j * 64 + lane) / cpg] = sm;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += 256)
        part2[(long)p * G + g] = ((wsum[0][g] + wsum[1][g]) + wsum[2][g]) + wsum[3][g];
}

template <int GI>
__global__ __launch_bounds__(256) void gn_apply3_kernel(const float *x, int L, int C, int G, int cpg, int P, long n,
                                                        float eps, const double *part2, const float2 *stat,
                                                        const float *gamma, const float *beta, _Float16 *xa) {
    __shared__ double red[64];
    __shared__ float2 st[64];
    // two 8-channel vectors per thread (grid = ceil(n8 / 512)); their x, gamma and beta are
    // in flight while the pass-2 sums are reduced (an index past the end reads vector 0)
    const long n8 = (long)L * C / 8;
    long e8[2];
    float4 u[2][2], gm[2][2], bt[2][2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        e8[k] = (long)blockIdx.x * 512 + 256 * k + threadIdx.x;
        const long e = e8[k] < n8 ? e8[k] : 0;
        const int c0 = (int)((e * 8) % C);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            u[k][h] = *reinterpret_cast<const float4 *>(x + e * 8 + 4 * h);
            gm[k][h] = *reinterpret_cast<const float4 *>(gamma + c0 + 4 * h);
            bt[k][h] = *reinterpret_cast<const float4 *>(beta + c0 + 4 * h);
        }
    }
    gn_reduce<GI>(part2, P, G, red);
    if (threadIdx.x < G) {
        const float variance = (float)(red[threadIdx.x] / (double)n);
        st[threadIdx.x] = make_float2(stat[threadIdx.x].x, 1.0f / sqrtf(variance + eps));
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (e8[k] >= n8) break;
        const int c0 = (int)((e8[k] * 8) % C);
        const float t[8] = {u[k][0].x, u[k][0].y, u[k][0].z, u[k][0].w, u[k][1].x, u[k][1].y, u[k][1].z, u[k][1].w};
        const float ga[8] = {gm[k][0].x, gm[k][0].y, gm[k][0].z, gm[k][0].w,
                             gm[k][1].x, gm[k][1].y, gm[k][1].z, gm[k][1].w};
        const float be[8] = {bt[k][0].x, bt[k][0].y, bt[k][0].z, bt[k][0].w,
                             bt[k][1].x, bt[k][1].y, bt[k][1].z, bt[k][1].w};
        f16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float2 ms = st[(c0 + q) / cpg];
            float y = t[q] - ms.x;
            y = y * ms.y;
            y = y * ga[q];
            y = y + be[q];
            o[q] = (_Float16)silu_f(y);
        }
        *reinterpret_cast<f16x8 *>(xa + e8[k] * 8) = o;
    }
}

// xa[l][c] = f16(silu((x - mean) * rstd * gamma + beta)), 8 channels per thread.
__global__ __launch_bounds__(256) void gn_apply_kernel(const float *x, int L, int C, int G, int cpg,
                                                       const float2 *stat, const float *gamma,
                                                       const float *beta, _Float16 *xa) {
    __shared__ float2 st[64];
    if (threadIdx.x < G) st[threadIdx.x] = stat[threadIdx.x];
    __syncthreads();
    const long e8 = (long)blockIdx.x * 256 + threadIdx.x;
    if (e8 * 8 >= (long)L * C) return;
    const int c0 = (int)((e8 * 8) % C);
    const float4 u0 = *reinterpret_cast<const float4 *>(x + e8 * 8);
    const float4 u1 = *reinterpret_cast<const float4 *>(x + e8 * 8 + 4);
    const float t[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
    f16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int ch = c0 + q;
        const float2 ms = st[ch / cpg];
        float y = t[q] - ms.x;
        y = y * ms.y;
        y = y * gamma[ch];
        y = y + beta[ch];
        o[q] = (_Float16)silu_f(y);
    }
    *reinterpret_cast<f16x8 *>(xa + e8 * 8) = o;
}

// ---------------------------------------------------------------- banded attention
// 16 queries per block, 16 threads per query (thread t scores keys j0 + t + 16 n, then owns
// output dims [4t, 4t + 4)): 4x the blocks of a 4-threads-per-query layout, so that the
// 700 / 1400-row attentions spread over every CU instead of ~150 of them. K (roped) and V
// rows of the block's key range and its roped queries are staged in LDS with float4 loads.
// Each score is the same ascending-d fmaf chain as before; P V runs over ascending j.
constexpr int BA_QB = 16;   // queries per block
constexpr int BA_TQ = 16;   // threads per query
constexpr int BA_HD = 64;   // head dim
constexpr int BA_MAXHW = 32;
constexpr int BA_KB = BA_QB + 2 * BA_MAXHW;
constexpr int BA_LD = BA_HD + 4;  // K / Q row stride (floats): 16 B aligned, rows 4 banks apart
constexpr int BA_NS = (2 * BA_MAXHW + 1 + BA_TQ - 1) / BA_TQ;  // scores per thread

__global__ __launch_bounds__(256) void band_attention_kernel(const float *qkv, float *out, int S,
                                                             int H, int hw, const float2 *rope) {
    __shared__ __attribute__((aligned(16))) float Ks[BA_KB][BA_LD];
    __shared__ __attribute__((aligned(16))) float Vs[BA_KB][BA_HD];
    __shared__ __attribute__((aligned(16))) float Qs[BA_QB][BA_LD];
    __shared__ float Ps[BA_QB][2 * BA_MAXHW + 2];
    const int h = blockIdx.y, i0 = blockIdx.x * BA_QB, tid = threadIdx.x;
    const int D = H * BA_HD, ld = 3 * D;
    const int kbeg = i0 - hw < 0 ? 0 : i0 - hw;
    int kend = i0 + BA_QB - 1 + hw;
    if (kend > S - 1) kend = S - 1;
    const int nk = kend - kbeg + 1;

    // K (roped) and V rows, then the block's queries (roped): float4 = two rotation pairs
    for (int e = tid; e < nk * (BA_HD / 4); e += 256) {
        const int r = e / (BA_HD / 4), c = (e - r * (BA_HD / 4)) * 4;
        const long p = kbeg + r;
        const float4 k = *reinterpret_cast<const float4 *>(qkv + p * ld + D + h * BA_HD + c);
        const float4 cs = *reinterpret_cast<const float4 *>(rope + p * (BA_HD / 2) + c / 2);
        const float4 v = *reinterpret_cast<const float4 *>(qkv + p * ld + 2 * D + h * BA_HD + c);
        *reinterpret_cast<float4 *>(&Ks[r][c]) =
            make_float4(k.x * cs.x - k.y * cs.y, k.x * cs.y + k.y * cs.x, k.z * cs.z - k.w * cs.w, k.z * cs.w + k.w * cs.z);
        *reinterpret_cast<float4 *>(&Vs[r][c]) = v;
    }
    for (int e = tid; e < BA_QB * (BA_HD / 4); e += 256) {
        const int r = e / (BA_HD / 4), c = (e - r * (BA_HD / 4)) * 4;
        const long p = i0 + r < S ? i0 + r : S - 1;
        const float4 q = *reinterpret_cast<const float4 *>(qkv + p * ld + h * BA_HD + c);
        const float4 cs = *reinterpret_cast<const float4 *>(rope + p * (BA_HD / 2) + c / 2);
        *reinterpret_cast<float4 *>(&Qs[r][c]) =
            make_float4(q.x * cs.x - q.y * cs.y, q.x * cs.y + q.y * cs.x, q.z * cs.z - q.w * cs.w, q.z * cs.w + q.w * cs.z);
    }
    __syncthreads();

    const int ql = tid / BA_TQ, t = tid % BA_TQ;
    const int i = i0 + ql;
    const bool active = i < S;
    const int j0 = active ? (i - hw < 0 ? 0 : i - hw) : 0;
    const int j1 = active ? (i + hw > S - 1 ? S - 1 : i + hw) : -1;
    const float scale = 0.125f;  // 1/sqrt(64), exact
    float q[BA_HD];
#pragma unroll
    for (int d = 0; d < BA_HD; d += 4) {
        const float4 v = *reinterpret_cast<const float4 *>(&Qs[ql][d]);
        q[d] = v.x, q[d + 1] = v.y, q[d + 2] = v.z, q[d + 3] = v.w;
    }
    float mx = -INFINITY;
    float sc[BA_NS];
#pragma unroll
    for (int n = 0; n < BA_NS; ++n) {
        const int j = j0 + t + BA_TQ * n;
        float s = -INFINITY;
        if (j <= j1) {
            const float *kr = Ks[j - kbeg];
            float a = 0.0f;
#pragma unroll
            for (int d = 0; d < BA_HD; d += 4) {
                const float4 k = *reinterpret_cast<const float4 *>(kr + d);
                a = fmaf(k.x, q[d], a);
                a = fmaf(k.y, q[d + 1], a);
                a = fmaf(k.z, q[d + 2], a);
                a = fmaf(k.w, q[d + 3], a);
            }
            s = a * scale;
        }
        sc[n] = s;
        mx = fmaxf(mx, s);
    }
#pragma unroll
    for (int o = 1; o < BA_TQ; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.0f;
#pragma unroll
    for (int n = 0; n < BA_NS; ++n) {
        const int j = j0 + t + BA_TQ * n;
        const float e = (j <= j1) ? expf(sc[n] - mx) : 0.0f;
        sc[n] = e;
        sum += e;
    }
#pragma unroll
    for (int o = 1; o < BA_TQ; o <<= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int n = 0; n < BA_NS; ++n) {
        const int j = j0 + t + BA_TQ * n;
        if (j <= j1) Ps[ql][j - j0] = sc[n] * inv;
    }
    __syncthreads();
    if (!active) return;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = j0; j <= j1; ++j) {
        const float p = Ps[ql][j - j0];
        const float4 v = *reinterpret_cast<const float4 *>(&Vs[j - kbeg][4 * t]);
        o.x = fmaf(p, v.x, o.x);
        o.y = fmaf(p, v.y, o.y);
        o.z = fmaf(p, v.z, o.z);
        o.w = fmaf(p, v.w, o.w);
    }
    *reinterpret_cast<float4 *>(out + (long)i * D + h * BA_HD + 4 * t) = o;
}

// ---------------------------------------------------------------- small kernels
__global__ void embed_kernel(const float *table, const int *codes, int T, int D, float *x) {
    const int t = blockIdx.x;
    const float4 *src = reinterpret_cast<const float4 *>(table + (long)codes[t] * D);
    float4 *dst = reinterpret_cast<float4 *>(x + (long)t * D);
    for (int i = threadIdx.x; i < D / 4; i += blockDim.x) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void cond_gemv_kernel(const float *W, const float *b, const float *e,
                                                        int R, int A, float *y, int e_f16) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    float a = 0.0f;
    for (int k = lane; k < A; k += 64) {
        float se = silu_f(e[k]);
        if (e_f16) se = (float)(_Float16)se;
        a = fmaf(W[(long)r * A + k], se, a);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o);
    if (lane == 0) y[r] = a + b[r];
}

template <int KG, int WTM = 1, int WTN = 1>
void launch_gemm_kg(const GemmArgs &a, int epi, hipStream_t s) {
    const int bm = GF_T * WTM, bn = GF_T * WTN;
    const long nb = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    dim3 grid((unsigned)(8 * ((nb + 7) / 8)));
    switch (epi) {
#define CASE(E)                                                                                  \
    case E:                                                                                      \
        hipLaunchKernelGGL((gemm_f32_kernel<KG, E, WTM, WTN>), grid, dim3(256 * KG), 0, s, a);   \
        break;
        CASE(EPI_STORE)
        CASE(EPI_RESID)
        CASE(EPI_GATED)
        CASE(EPI_SWIGLU)
        CASE(EPI_CONVT)
        CASE(EPI_CONVT_SNAKE)
        CASE(EPI_SNAKE)
        CASE(EPI_HEAD)
#undef CASE
    }
}

}  // namespace

// K-groups per block: enough blocks x waves to give every CU 16 waves (MIO_CODEC_KG forces).
int gemm_kgroups(long tiles) {
    static const int forced = [] {
        const char *e = getenv("MIO_CODEC_KG");
        return e ? atoi(e) : 0;
    }();
    if (forced == 1 || forced == 2 || forced == 4) return forced;
    return tiles >= 512 ? 1 : tiles >= 256 ? 2 : 4;
}

void launch_gemm_f32(const GemmArgs &a0, int epi, hipStream_t s) {
    GemmArgs a = a0;
    a.m_major = (long)a.M * a.K > (long)a.N * a.K * 2 ? 1 : 0;  // slab the larger operand
    const long tiles = (long)((a.M + GF_T - 1) / GF_T) * ((a.N + GF_T - 1) / GF_T);
    const int kgs = gemm_kgroups(tiles);
    switch (kgs) {
        case 1: launch_gemm_kg<1>(a, epi, s); break;
        case 2: launch_gemm_kg<2>(a, epi, s); break;
        default: launch_gemm_kg<4>(a, epi, s); break;
    }
}

// One tile configuration, forced (tools/micro/gemm_probe): kg K-groups, wt = 10 WTM + WTN.
// Larger wave tiles (21, 12, 22) measured no faster on any codec shape and are not built
// (profiles/r03_codec_gemm_configs_bufload.txt).
int launch_gemm_f32_cfg(const GemmArgs &a0, int epi, int kg, int wt, hipStream_t s) {
    GemmArgs a = a0;
    a.m_major = (long)a.M * a.K > (long)a.N * a.K * 2 ? 1 : 0;
    switch (wt * 10 + kg) {
        case 111: launch_gemm_kg<1, 1, 1>(a, epi, s); break;
        case 112: launch_gemm_kg<2, 1, 1>(a, epi, s); break;
        case 114: launch_gemm_kg<4, 1, 1>(a, epi, s); break;
        default: return -1;
    }
    return 0;
}

void launch_conv_f16(const ConvArgs &a, hipStream_t s) {
    dim3 grid((a.Cout + CV_BN - 1) / CV_BN, (a.L + CV_BM - 1) / CV_BM);
    hipLaunchKernelGGL(conv_f16_kernel, grid, dim3(256), 0, s, a);
}

void launch_rownorm(const float *x, float *y, int M, int D, float eps, int mode, const float *p0,
                    const float *p1, hipStream_t s) {
    const dim3 grid((M + 3) / 4);
    switch (D / 64) {
#define RN(P)                                                                                             \
    case P: hipLaunchKernelGGL(rownorm_kernel<P>, grid, dim3(256), 0, s, x, y, M, eps, mode, p0, p1); break;
        RN(1) RN(2) RN(3) RN(4) RN(5) RN(6) RN(7) RN(8) RN(9) RN(10) RN(11) RN(12) RN(13) RN(14) RN(15) RN(16)
#undef RN
        default: break;  // refused at load (codec.cpp: D % 64 == 0, D <= 1024)
    }
}

void launch_groupnorm_apply(const float *x, int L, int C, int G, float eps, const float *gamma,
                            const float *beta, GnScratch gs, _Float16 *xa, hipStream_t s) {
    const int cpg = C / G;
    // MIO_GN=3 (default): three launches, every workgroup reducing the slice sums itself;
    // MIO_GN=1: one workgroup per group (gn_fused_kernel) when the group is whole float4 quads
    // (cpg = 4, 8, 16, 32, 64: cpg | 64); MIO_GN=5 (or 1 otherwise): the sliced five launches
    static const int mode = getenv("MIO_GN") ? atoi(getenv("MIO_GN")) : 3;
    const long n = (long)L * cpg;
    if (mode == 3) {
        int rows = 4;
        if ((L + rows - 1) / rows > GN3_PMAX) rows = (L + GN3_PMAX - 1) / GN3_PMAX;
        const int P = (L + rows - 1) / rows;
        double *part1 = gs.part, *part2 = gs.part + GN_PMAX * 64;
        const int nj = (C + 63) / 64;
        const long n8 = (long)L * C / 8;
        const unsigned ga = (unsigned)((n8 + 511) / 512);
        auto go = [&](auto gi) {
            constexpr int GI = decltype(gi)::value;
            switch (nj) {
#define G3(J)                                                                                                      \
    case J:                                                                                                        \
        hipLaunchKernelGGL((gn_partial_kernel<1, J>), dim3(P), dim3(256), 0, s, x, L, C, G, cpg, rows,             \
                           (const float2 *)gs.stat, part1);                                                        \
        hipLaunchKernelGGL((gn_stat2_kernel<J, GI>), dim3(P), dim3(256), 0, s, x, L, C, G, cpg, rows, n, part1,     \
                           part2, gs.stat);                                                                        \
        break;
                G3(1) G3(2) G3(3) G3(4) G3(5) G3(6) G3(7) G3(8) G3(9) G3(10) G3(11) G3(12) G3(13) G3(14) G3(15) G3(16)
#undef G3
                default: return;  // C <= 1024 (codec.cpp refuses larger)
            }
            hipLaunchKernelGGL((gn_apply3_kernel<GI>), dim3(ga), dim3(256), 0, s, x, L, C, G, cpg, P, n, eps, part2,
                               (const float2 *)gs.stat, gamma, beta, xa);
        };
        if (G <= 32)
            go(std::integral_constant<int, 4>{});
        else
            go(std::integral_constant<int, 8>{});
        return;
    }
    if (mode == 1 && cpg % 4 == 0 && (cpg & (cpg - 1)) == 0 && (long)L * (cpg / 4) < (1L << 30)) {
        int qsh = 0;
        while ((4 << qsh) < cpg) ++qsh;
        hipLaunchKernelGGL(gn_fused_kernel, dim3(G), dim3(1024), 0, s, x, L, C, cpg, qsh, eps, gamma, beta, xa);
        return;
    }
    int rows = 4;
    if ((L + rows - 1) / rows > GN_PMAX) rows = (L + GN_PMAX - 1) / GN_PMAX;
    const int P = (L + rows - 1) / rows;
    auto partial = [&](auto pass) {
        constexpr int PS = decltype(pass)::value;
        switch ((C + 63) / 64) {
#define GP(J)                                                                                                  \
    case J:                                                                                                    \
        hipLaunchKernelGGL((gn_partial_kernel<PS, J>), dim3(P), dim3(256), 0, s, x, L, C, G, cpg, rows,        \
                           (const float2 *)gs.stat, gs.part);                                                  \
        break;
            GP(1) GP(2) GP(3) GP(4) GP(5) GP(6) GP(7) GP(8) GP(9) GP(10) GP(11) GP(12) GP(13) GP(14) GP(15) GP(16)
#undef GP
            default: break;  // C <= 1024 (codec.cpp refuses larger)
        }
    };
    partial(std::integral_constant<int, 1>{});
    hipLaunchKernelGGL(gn_final_kernel<1>, dim3(1), dim3(1024), 0, s, (const double *)gs.part, P, G, n, eps,
                       gs.stat);
    partial(std::integral_constant<int, 2>{});
    hipLaunchKernelGGL(gn_final_kernel<2>, dim3(1), dim3(1024), 0, s, (const double *)gs.part, P, G, n, eps,
                       gs.stat);
    const long n8 = (long)L * C / 8;
    hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, x, L, C, G,
                       cpg, (const float2 *)gs.stat, gamma, beta, xa);
}

void launch_band_attention(const float *qkv, float *out, int S, int H, int window,
                           const float2 *rope, hipStream_t s) {
    dim3 grid((S + BA_QB - 1) / BA_QB, H);
    hipLaunchKernelGGL(band_attention_kernel, grid, dim3(256), 0, s, qkv, out, S, H, window / 2, rope);
}

void launch_embed(const float *table, const int *codes, int T, int D, float *x, hipStream_t s) {
    hipLaunchKernelGGL(embed_kernel, dim3(T), dim3(256), 0, s, table, codes, T, D, x);
}

void launch_cond_gemv(const float *W, const float *b, const float *e, int R, int A, float *y, int e_f16,
                      hipStream_t s) {
    hipLaunchKernelGGL(cond_gemv_kernel, dim3((R + 3) / 4), dim3(256), 0, s, W, b, e, R, A, y, e_f16);
}

}  // namespace mio
