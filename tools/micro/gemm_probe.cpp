// Times mio::launch_gemm_f32 (codec f32 GEMM) on the codec's shapes and a 4096^3 calibration
// case with HIP events. Build: see tools/micro/Makefile.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <algorithm>
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
    float *A, *B, *C, *Cref, *aux;
    hipMalloc(&A, maxa * 4);
    hipMalloc(&B, maxb * 4);
    hipMalloc(&C, maxc * 4);
    hipMalloc(&Cref, maxc * 4);
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
        const int cfgs[][2] = {{0, 0}, {1, 11}, {2, 11}, {4, 11}};
        for (auto &c : cfgs) {
            auto run = [&] {
                if (c[0] == 0)
                    mio::launch_gemm_f32(g, s.epi, st);
                else
                    mio::launch_gemm_f32_cfg(g, s.epi, c[0], c[1], st);
            };
            // correctness against the default kernel (plain store epilogue)
            double maxrel = 0;
            if (c[0] != 0) {
                mio::GemmArgs gs = g;
                gs.C = Cref;
                mio::launch_gemm_f32(gs, mio::EPI_STORE, st);
                gs.C = C;
                if (mio::launch_gemm_f32_cfg(gs, mio::EPI_STORE, c[0], c[1], st) != 0) continue;
                hipStreamSynchronize(st);
                std::vector<float> h1((size_t)s.M * s.N), h2((size_t)s.M * s.N);
                hipMemcpy(h1.data(), Cref, h1.size() * 4, hipMemcpyDeviceToHost);
                hipMemcpy(h2.data(), C, h2.size() * 4, hipMemcpyDeviceToHost);
                double mx = 0, df = 0;
                for (size_t i = 0; i < h1.size(); ++i) {
                    mx = std::max(mx, (double)std::fabs(h1[i]));
                    df = std::max(df, (double)std::fabs(h1[i] - h2[i]));
                }
                maxrel = df / (mx > 0 ? mx : 1);
            }
            for (int i = 0; i < 3; ++i) run();
            hipEventRecord(e0, st);
            for (int i = 0; i < reps; ++i) run();
            hipEventRecord(e1, st);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / reps, tf = 2.0 * s.M * s.N * s.K / (us * 1e-6) / 1e12;
            printf("%-14s M=%5d N=%5d K=%5d  kg %d wt %3d  %8.1f us  %6.1f TF/s  maxrel %.1e\n", s.name, s.M, s.N, s.K,
                   c[0], c[1], us, tf, maxrel);
        }
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 1;
    return 0;
}
