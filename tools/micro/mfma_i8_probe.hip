// Operand lane maps of the gfx950 int8 MFMAs, checked with exact asymmetric integer data
// (cdna_hip_programming.md: "check the map with exact integer data before relying on it").
// For each instruction, lane l loads its A / B bytes under hypothesis H1 (lane holds K
// elements kb + j, kb = KL * (l / R), j < KL) and H2 (two halves: k = 8 (l / R) + j for
// j < 8, K/2 + 8 (l / R) + j - 8 for j >= 8); C/D: col = lane % R, row from the documented
// map. Prints which hypothesis reproduces the CPU product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__host__ __device__ inline int Aval(int i, int k) { return ((i * 7 + k * 3) % 11) - 5; }
__host__ __device__ inline int Bval(int k, int j) { return ((k * 5 + j * 2 + (k * j) % 3) % 13) - 6; }

// kidx(lane, j, R, K, hyp)
__device__ inline int kidx(int l, int j, int R, int K, int hyp, int KL) {
    const int h = l / R;
    if (hyp == 1) return KL * h + j;
    return j < 8 ? 8 * h + j : K / 2 + 8 * h + (j - 8);
}

template <int SHAPE>
__global__ void probe(int hyp, int *out) {
    const int l = threadIdx.x;
    if constexpr (SHAPE == 0) {  // 32x32x32 i8: 16 bytes per lane
        const int R = 32, K = 32;
        signed char a[16], b[16];
        for (int j = 0; j < 16; ++j) {
            const int k = kidx(l, j, R, K, hyp, 16);
            a[j] = (signed char)Aval(l % R, k);
            b[j] = (signed char)Bval(k, l % R);
        }
        v4i av, bv;
        __builtin_memcpy(&av, a, 16);
        __builtin_memcpy(&bv, b, 16);
        v16i c = {};
        c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
            out[row * 32 + col] = c[r];
        }
    } else if constexpr (SHAPE == 1) {  // 16x16x64 i8: 16 bytes per lane
        const int R = 16, K = 64;
        signed char a[16], b[16];
        for (int j = 0; j < 16; ++j) {
            const int h = l / R;
            const int k = hyp == 1 ? 16 * h + j : (j < 8 ? 8 * h + j : 32 + 8 * h + (j - 8));
            a[j] = (signed char)Aval(l % R, k);
            b[j] = (signed char)Bval(k, l % R);
        }
        v4i av, bv;
        __builtin_memcpy(&av, a, 16);
        __builtin_memcpy(&bv, b, 16);
        v4i c = {};
        c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
        for (int r = 0; r < 4; ++r) {
            const int row = (l >> 4) * 4 + r, col = l & 15;
            out[row * 16 + col] = c[r];
        }
    } else if constexpr (SHAPE == 2) {  // 32x32x16 i8 (CDNA3 form): 8 bytes per lane
        const int R = 32;
        signed char a[8], b[8];
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * (l / R) + j;
            a[j] = (signed char)Aval(l % R, k);
            b[j] = (signed char)Bval(k, l % R);
        }
        long av, bv;
        __builtin_memcpy(&av, a, 8);
        __builtin_memcpy(&bv, b, 8);
        v16i c = {};
        c = __builtin_amdgcn_mfma_i32_32x32x16_i8(av, bv, c, 0, 0, 0);
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
            out[row * 32 + col] = c[r];
        }
    } else {  // 16x16x32 i8 (CDNA3 form): 8 bytes per lane
        const int R = 16;
        signed char a[8], b[8];
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * (l / R) + j;
            a[j] = (signed char)Aval(l % R, k);
            b[j] = (signed char)Bval(k, l % R);
        }
        long av, bv;
        __builtin_memcpy(&av, a, 8);
        __builtin_memcpy(&bv, b, 8);
        v4i c = {};
        c = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, c, 0, 0, 0);
        for (int r = 0; r < 4; ++r) {
            const int row = (l >> 4) * 4 + r, col = l & 15;
            out[row * 16 + col] = c[r];
        }
    }
}

int main() {
    int *d = nullptr;
    hipMalloc(&d, 32 * 32 * 4);
    const char *names[4] = {"32x32x32_i8", "16x16x64_i8", "32x32x16_i8", "16x16x32_i8"};
    const int Rs[4] = {32, 16, 32, 16}, Ks[4] = {32, 64, 16, 32};
    for (int s = 0; s < 4; ++s)
        for (int hyp = 1; hyp <= 2; ++hyp) {
            if (s >= 2 && hyp == 2) continue;
            hipMemset(d, 0, 32 * 32 * 4);
            if (s == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, hyp, d);
            if (s == 1) hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, hyp, d);
            if (s == 2) hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, hyp, d);
            if (s == 3) hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, hyp, d);
            std::vector<int> h(32 * 32);
            hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
            const int R = Rs[s], K = Ks[s];
            int bad = 0;
            for (int i = 0; i < R; ++i)
                for (int j = 0; j < R; ++j) {
                    int ref = 0;
                    for (int k = 0; k < K; ++k) ref += Aval(i, k) * Bval(k, j);
                    bad += h[i * R + j] != ref;
                }
            printf("%s hyp %d: %s (%d of %d wrong)\n", names[s], hyp, bad ? "MISMATCH" : "OK", bad, R * R);
        }
    hipFree(d);
    return 0;
}
