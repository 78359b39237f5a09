// Microbenchmark (diagnostic): cost of executing N KB of straight-line VALU code ONCE per
// workgroup, cold (other kernels' code in between) vs warm (same kernel back to back).
// Each variant runs 256 workgroups x 512 threads; duration from HIP events over 200 launches.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int N>
__global__ __launch_bounds__(512) void straight(float *out, float a) {
    float x = a + threadIdx.x, y = a * 2.0f, z = a * 3.0f, w = a * 4.0f;
#pragma unroll
    for (int i = 0; i < N; ++i) {  // 4 independent chains: issue-bound, ~8 B per instruction
        x = x * 1.0001f + 0.5f;
        y = y * 0.9999f + 0.25f;
        z = z * 1.0002f + 0.125f;
        w = w * 0.9998f + 0.0625f;
    }
    if (x + y + z + w == 12345.0f) out[threadIdx.x] = x;
}

template <int N>
__global__ __launch_bounds__(512) void other(float *out, float a) {  // evicts the i-cache
    float x = a + threadIdx.x, y = a * 2.0f, z = a * 3.0f, w = a * 4.0f;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        x = x * 1.0003f + 0.75f;
        y = y * 0.9997f + 0.35f;
        z = z * 1.0004f + 0.145f;
        w = w * 0.9996f + 0.0665f;
    }
    if (x + y + z + w == 12345.0f) out[threadIdx.x] = x;
}

template <int N>
void run(float *d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0), hipEventCreate(&e1);
    float ms_warm, ms_cold, ms_other;
    for (int i = 0; i < 20; ++i) straight<N><<<256, 512>>>(d, 1.0f);
    hipEventRecord(e0);
    for (int i = 0; i < 200; ++i) straight<N><<<256, 512>>>(d, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_warm, e0, e1);
    hipEventRecord(e0);
    for (int i = 0; i < 200; ++i) other<N * 4><<<256, 512>>>(d, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_other, e0, e1);
    hipEventRecord(e0);
    for (int i = 0; i < 200; ++i) {
        other<N * 4><<<256, 512>>>(d, 1.0f);
        straight<N><<<256, 512>>>(d, 1.0f);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_cold, e0, e1);
    const double warm = ms_warm * 1e3 / 200, pair = ms_cold * 1e3 / 200, oth = ms_other * 1e3 / 200;
    printf("N=%5d (~%5.1f KB straight code): warm %.2f us/launch, cold (after other) %.2f us, other alone %.2f us\n", N,
           N * 4 * 2 * 8 / 1024.0, warm, pair - oth, oth);
}

int main() {
    float *d;
    hipMalloc(&d, 4096);
    run<16>(d);
    run<128>(d);
    run<256>(d);
    run<512>(d);
    hipFree(d);
    return 0;
}
