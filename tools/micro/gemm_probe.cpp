// Times mio::launch_gemm_f32 (codec f32 GEMM) on the codec's shapes and a 4096^3 calibration
// case with HIP events. Build: see tools/micro/Makefile.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "codec_kernels.h"

int main(int argc, char **argv) {
    struct Shape { int M, N, K, epi; const char *name; };
    std::vector<Shape> shapes = {
        {1400, 3072, 512, mio::EPI_SWIGLU, "dec gate_up"},  {1400, 1536, 512, mio::EPI_STORE, "dec qkv"},
        {1400, 512, 512, mio::EPI_GATED, "dec wo"},         {1400, 512, 1536, mio::EPI_GATED, "dec down"},
        {700, 4096, 768, mio::EPI_SWIGLU, "pre gate_up"},   {700, 2304, 768, mio::EPI_STORE, "pre qkv"},
        {700, 768, 768, mio::EPI_RESID, "pre wo"},          {700, 768, 2048, mio::EPI_RESID, "pre down"},
        {12600, 512, 512, mio::EPI_STORE, "head-like"},     {4096, 4096, 4096, mio::EPI_STORE, "calib 4096^3"},
    };
    size_t maxa = 0, maxb = 0, maxc = 0;
    for (auto &s : shapes) {
        maxa = std::max(maxa, (size_t)s.M * s.K);
        maxb = std::max(maxb, (size_t)s.N * s.K);
        maxc = std::max(maxc, (size_t)s.M * s.N);
    }
    float *A, *B, *C, *aux;
    hipMalloc(&A, maxa * 4);
    hipMalloc(&B, maxb * 4);
    hipMalloc(&C, maxc * 4);
    hipMalloc(&aux, 65536 * 4);
    std::vector<float> h(std::max(maxa, maxb));
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.0f - 0.5f;
    hipMemcpy(A, h.data(), maxa * 4, hipMemcpyHostToDevice);
    hipMemcpy(B, h.data(), maxb * 4, hipMemcpyHostToDevice);
    hipMemset(C, 0, maxc * 4);
    hipMemset(aux, 0, 65536 * 4);
    hipStream_t st;
    hipStreamCreate(&st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto &s : shapes) {
        mio::GemmArgs g{};
        g.A = A, g.a_seg = s.K, g.a_row_off = 0, g.a_rows = s.M, g.B = B, g.M = s.M, g.N = s.N, g.K = s.K;
        g.C = C, g.ldc = s.N, g.aux = aux;
        const int reps = s.M >= 4096 && s.N >= 4096 ? 5 : 50;
        // cfg 0: the default choice (launch_gemm_f32); then every forced tile configuration
        const int cfgs[][2] = {{0, 0}, {1, 11}, {2, 11}, {4, 11}, {1, 21}, {2, 21}, {1, 12}, {2, 12}, {1, 22}, {2, 22}};
        for (auto &c : cfgs) {
            auto run = [&] {
                if (c[0] == 0)
                    mio::launch_gemm_f32(g, s.epi, st);
                else
                    mio::launch_gemm_f32_cfg(g, s.epi, c[0], c[1], st);
            };
            for (int i = 0; i < 3; ++i) run();
            hipEventRecord(e0, st);
            for (int i = 0; i < reps; ++i) run();
            hipEventRecord(e1, st);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / reps, tf = 2.0 * s.M * s.N * s.K / (us * 1e-6) / 1e12;
            printf("%-14s M=%5d N=%5d K=%5d  kg %d wt %2d  %8.1f us  %6.1f TF/s\n", s.name, s.M, s.N, s.K, c[0], c[1],
                   us, tf);
        }
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 1;
    return 0;
}
