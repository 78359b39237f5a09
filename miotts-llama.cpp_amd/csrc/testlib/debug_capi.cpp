// Test-support C-ABI (libmiotts_test.so, include/mio_hip_test.h): parity entry points of the
// matvec / batched-matmul kernels on raw GGUF rows, and the host quantizer the synthetic
// models are built with. Not part of the product library.
#include <vector>

#include "common.h"
#include "gguf.h"
#include "llm_kernels.h"
#include "mio_hip_test.h"
#include "quant.h"

extern "C" int mio_hip_debug_matvec(mio_hip_device *d, uint32_t type, const void *gguf_rows, int rows, int k,
                                    const float *x, float *y) {
    MIO_REQUIRE(d && gguf_rows && x && y && rows > 0 && k > 0, MIO_ERR_INVALID, "debug_matvec: bad args");
    MIO_REQUIRE(type == mio::GGML_Q8_0 || type == mio::GGML_Q4_K || type == mio::GGML_Q6_K ||
                    type == mio::GGML_BF16 || mio::repacks_to_q8_0(type),
                MIO_ERR_UNSUPPORTED, "debug_matvec: type %u", type);
    const bool k32 = type == mio::GGML_Q8_0 || type == mio::GGML_BF16 || mio::repacks_to_q8_0(type);
    MIO_REQUIRE(k % (k32 ? 32 : 256) == 0, MIO_ERR_INVALID, "debug_matvec: k %d", k);
    int rc = mio::bind(d);
    if (rc) return rc;
    // Q4_0 / Q5_0 run as the Q8_0 rows they equal (llm_load does the same)
    std::vector<uint8_t> q80;
    if (mio::repacks_to_q8_0(type)) {
        q80.resize((size_t)rows * (k / 32) * sizeof(mio::BlockQ8_0));
        mio::repack_to_q8_0(type, gguf_rows, rows, k, q80.data());
        gguf_rows = q80.data();
        type = mio::GGML_Q8_0;
    }
    const mio::SplitLayout L = mio::split_layout(type, rows, k);
    std::vector<uint8_t> host(L.bytes);
    mio::to_split(type, gguf_rows, rows, k, host.data());
    uint8_t *dw = nullptr;
    float *dx = nullptr, *dy = nullptr;
    MIO_HIP_CHECK(hipMalloc(&dw, L.bytes));
    MIO_HIP_CHECK(hipMalloc(&dx, (size_t)k * 4));
    MIO_HIP_CHECK(hipMalloc(&dy, (size_t)rows * 4));
    hipMemcpy(dw, host.data(), L.bytes, hipMemcpyHostToDevice);
    hipMemcpy(dx, x, (size_t)k * 4, hipMemcpyHostToDevice);
    mio::QMat q{(int)type, rows, k, dw + L.off[0], dw + L.off[1], dw + L.off[2], dw + L.off[3]};
    mio::launch_debug_matvec(q, dx, dy, d->n_cu > 0 ? d->n_cu : 256, d->stream);
    hipError_t e = hipStreamSynchronize(d->stream);
    if (e == hipSuccess) e = hipMemcpy(y, dy, (size_t)rows * 4, hipMemcpyDeviceToHost);
    hipFree(dw), hipFree(dx), hipFree(dy);
    MIO_HIP_CHECK(e);
    return MIO_OK;
}

extern "C" int mio_hip_debug_mmq(mio_hip_device *d, uint32_t type, const void *gguf_rows, int rows, int k,
                                 const float *x, int nt, int mode, const void *gguf_up, float *y) {
    MIO_REQUIRE(d && gguf_rows && x && y && rows > 0 && k > 0 && nt > 0 && nt <= 4096 && mode >= 0 && mode <= 2 &&
                    (mode != 2 || gguf_up),
                MIO_ERR_INVALID, "debug_mmq: bad args");
    MIO_REQUIRE(type == mio::GGML_Q8_0 || type == mio::GGML_Q4_K || type == mio::GGML_Q6_K, MIO_ERR_UNSUPPORTED,
                "debug_mmq: type %u", type);
    MIO_REQUIRE(k % (type == mio::GGML_Q8_0 ? 32 : 256) == 0, MIO_ERR_INVALID, "debug_mmq: k %d", k);
    int rc = mio::bind(d);
    if (rc) return rc;
    const mio::SplitLayout L = mio::split_layout(type, rows, k);
    const int nm = mode == 2 ? 2 : 1;
    std::vector<uint8_t> host(L.bytes * nm);
    mio::to_split(type, gguf_rows, rows, k, host.data());
    if (nm == 2) mio::to_split(type, gguf_up, rows, k, host.data() + L.bytes);
    uint8_t *dw = nullptr;
    float *dx = nullptr, *dy = nullptr;
    char *da = nullptr;
    MIO_HIP_CHECK(hipMalloc(&dw, L.bytes * nm));
    MIO_HIP_CHECK(hipMalloc(&dx, (size_t)nt * k * 4));
    MIO_HIP_CHECK(hipMalloc(&dy, (size_t)nt * rows * 4));
    MIO_HIP_CHECK(hipMalloc(&da, (size_t)nt * mio::debug_act_bytes(k)));
    hipMemcpy(dw, host.data(), L.bytes * nm, hipMemcpyHostToDevice);
    hipMemcpy(dx, x, (size_t)nt * k * 4, hipMemcpyHostToDevice);
    hipMemcpy(dy, y, (size_t)nt * rows * 4, hipMemcpyHostToDevice);  // mode 1 adds to y
    auto qm = [&](uint8_t *base) {
        return mio::QMat{(int)type, rows, k, base + L.off[0], base + L.off[1], base + L.off[2], base + L.off[3]};
    };
    const mio::QMat q = qm(dw), up = nm == 2 ? qm(dw + L.bytes) : mio::QMat{};
    mio::launch_debug_mmq(q, up, mode, dx, nt, da, dy, d->stream);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    if (e == hipSuccess) e = hipMemcpy(y, dy, (size_t)nt * rows * 4, hipMemcpyDeviceToHost);
    hipFree(dw), hipFree(dx), hipFree(dy), hipFree(da);
    MIO_HIP_CHECK(e);
    return MIO_OK;
}

extern "C" int mio_quantize_rows(uint32_t type, const float *x, int rows, int k, void *out) {
    MIO_REQUIRE(x && out && rows > 0 && k > 0, MIO_ERR_INVALID, "quantize_rows: bad args");
    const size_t rb = mio::ggml_row_bytes(type, k);
    MIO_REQUIRE(rb, MIO_ERR_UNSUPPORTED, "quantize_rows: type %u / k %d", type, k);
    for (int r = 0; r < rows; ++r)
        if (!mio::quantize_row(type, x + (size_t)r * k, (uint8_t *)out + r * rb, k)) return MIO_ERR_UNSUPPORTED;
    return MIO_OK;
}
