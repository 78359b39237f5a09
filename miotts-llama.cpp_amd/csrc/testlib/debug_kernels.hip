// Test-support kernel (libmiotts_test.so): y = W x with x re-quantized to the vec_dot_type
// in the decode prologue's way, on the decode step's streaming matvec engine (llm_device.h),
// for mio_hip_debug_matvec's parity tests of every weight type.
#include "llm_device.h"

#pragma clang fp contract(off)

namespace mio {
namespace {
template <int NP, int T>
__global__ __launch_bounds__(MT) void k_debug_matvec(QMat W, const float *x, float *y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int K = W.k;
    const Smem s = carve(smem, K);
    XRegs<NP> xr;
    load_x(x, nullptr, K, xr);
    int lo, hi;
    wave_range(W.rows, lo, hi, blockIdx.x, gridDim.x);
    Frag ga[Cfg<NP>::U], gb[Cfg<NP>::U];
    load_first<T, NP, 1>(W, W, lo, hi, ga, gb);
    plain_quant(xr, K, akind(T), s);
    stream_rows<T, NP, 1>(W, W, lo, hi, ga, gb, s.a, [&](int row, float v, float) {
        if ((threadIdx.x & 63) == 0) y[row] = v;
    });
}
}  // namespace

void launch_debug_matvec(const QMat &W, const float *x, float *y, int n_wg, hipStream_t s) {
    LlmDims d{};
    d.n_wg = n_wg;
    dispatch_nt(W.k, W.type, [&]<int NP, int T>() {
        hipLaunchKernelGGL((k_debug_matvec<NP, T>), dim3(matvec_grid(d, W.rows)), dim3(MT), matvec_lds(W.k), s, W, x,
                           y);
    });
}

}  // namespace mio
