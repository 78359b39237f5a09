// Launch interface of the MioCodec decoder kernels (csrc/hip/codec_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace mio {

// Epilogues of the f32 GEMM C[M][N] = A[M][K] * B[N][K]^T (all on v_mfma_f32_32x32x2_f32).
enum GemmEpi : int {
    EPI_STORE = 0,      // C = acc (+bias[n])
    EPI_RESID = 1,      // C += acc (+bias[n])                      (ggml_add residual)
    EPI_GATED = 2,      // C += gate[n] * acc                        (AdaLN-Zero gated residual)
    EPI_SWIGLU = 3,     // B rows interleaved per 32 (gate|up): C[m][n/2] = silu(g)*u
    EPI_CONVT = 4,      // ConvTranspose remap: out[f*m + n/Cout - trim][n%Cout] = acc + bias
    EPI_CONVT_SNAKE = 5,// CONVT then snake(alpha_e, beta_e)
    EPI_SNAKE = 6,      // C = snake(acc + bias)
    EPI_HEAD = 7,       // B rows interleaved per 32 (logmag|phase): spec[m][k] = polar
};

struct GemmArgs {
    const float *A;   // element (m,k) at A[(m + a_row_off) * a_seg + k]
    int a_seg;        // floats per source row (Cin); K = taps * a_seg
    int a_row_off;    // first source row of output row 0 (tap window start)
    int a_rows;       // valid source rows [0, a_rows); others read as zero
    const float *B;   // [N][K]
    int M, N, K;
    float *C;
    int ldc;
    const float *bias;
    const float *aux;   // gate (EPI_GATED), exp(alpha) (snake)
    const float *aux2;  // exp(beta) (snake)
    int f, trim, cout, rows_out;  // CONVT remap; HEAD: cout = n_freq
    int m_major;      // tile order (set by launch_gemm_f32)
    int a_f16;        // B came from an F16 GGUF tensor: A is rounded to f16 (ggml mul_mat /
                      // conv_transpose_1d convert src1 to the F16 vec_dot_type), f32 sums
};

// Conv1d k=taps, stride 1, "same" zero padding, as an implicit GEMM on f16 MFMA over the
// f16 activation written by launch_groupnorm_apply (ggml conv_1d rounds both the kernel and
// the im2col input to f16; miocodec.cpp:382-386). Cin % 8 == 0.
struct ConvArgs {
    const _Float16 *Xa;    // [L][Cin] silu(GroupNorm(x)) rounded to f16
    int L, Cin;
    int taps, pad;
    const _Float16 *B;     // [Cout][taps*Cin] f16 kernel, k-index = tap*Cin + ci
    int Cout;
    const float *bias;     // [Cout]
    float *Y;              // [L][Cout]
    const float *resid;    // optional [L][Cout] added after bias (may alias Y)
};

void launch_gemm_f32(const GemmArgs &a, int epi, hipStream_t s);
// One forced tile configuration (micro-benchmark): kg K-groups (1, 2, 4), wt = 10 WTM + WTN
// (11, 21, 12, 22; WTM x WTN 32 x 32 accumulators per wave). Returns -1 for an unbuilt pair.
int launch_gemm_f32_cfg(const GemmArgs &a, int epi, int kg, int wt, hipStream_t s);
void launch_conv_f16(const ConvArgs &a, hipStream_t s);

// Row norms, one wave per row (D % 64 == 0, D <= 1024). mode 0: plain, 1: affine (w,b; b may be null),
// 2: AdaLN (shift = p0, scale = p1: y*(1+scale)+shift). In-place (y == x) allowed.
void launch_rownorm(const float *x, float *y, int M, int D, float eps, int mode, const float *p0,
                    const float *p1, hipStream_t s);
// xa = f16(silu(GroupNorm(x) * gamma + beta)) over [L][C], G groups of C/G channels
// (C % 8 == 0, C <= 1024, G <= 64, 64 % (C/G) == 0). Five launches on stream s.
struct GnScratch {
    double *part;        // kGnPartDoubles: [2][P <= 256][64] slice sums (pass 1, pass 2)
    float2 *stat;        // [64] (mean, rstd)
};
constexpr int kGnPartDoubles = 2 * 256 * 64;
void launch_groupnorm_apply(const float *x, int L, int C, int G, float eps, const float *gamma,
                            const float *beta, GnScratch gs, _Float16 *xa, hipStream_t s);
// Banded (|i-j| <= window/2) RoPE attention, head_dim 64, q|k|v packed per row (ld = 3*D).
void launch_band_attention(const float *qkv, float *out, int S, int H, int window,
                           const float2 *rope /*[S][32] (cos,sin)*/, hipStream_t s);
void launch_embed(const float *table, const int *codes, int T, int D, float *x, hipStream_t s);
// y[r] = W[r][:] . silu(e) + b[r], W [R][A]; e_f16: W was F16, silu(e) is rounded to f16
void launch_cond_gemv(const float *W, const float *b, const float *e, int R, int A, float *y, int e_f16,
                      hipStream_t s);

}  // namespace mio
