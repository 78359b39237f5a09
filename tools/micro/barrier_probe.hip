// Microbenchmark (diagnostic): cost of one chip-wide phase hand-off inside a persistent
// launch vs a kernel boundary, for the decode step's shape (256 workgroups x 512 threads,
// each phase: every workgroup publishes 8 floats of a 2048-float vector, then every
// workgroup reads the whole vector and reduces it).
//   persistent: sc1 (write-through) stores -> vmcnt(0) -> barrier -> one lane adds to its
//               per-XCD counter shard -> one wave polls the 8 shards by sc1 loads -> barrier
//               -> sc1 loads of the vector.
//   launches:   the same phase body as one kernel per phase, hipGraph-captured.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int T = 512, N = 2048;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

__device__ __forceinline__ void publish(float *x, float v, int p) {
    // 8 floats per workgroup, lanes 0..7 of wave 0; aux 16 = sc1 (write-through)
    const int b = blockIdx.x;
    if (threadIdx.x < 8) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v + threadIdx.x + p), rs(x, N * 4), (b * 8 + threadIdx.x) * 4, 0, 16);
}

__global__ __launch_bounds__(T) void k_persistent(float *xa, float *xb, unsigned *cnt, unsigned *err, int phases, float *out) {
    __shared__ float red[T / 64];
    float acc = 0.f;
    const unsigned shard = blockIdx.x & 7;
    for (int p = 0; p < phases; ++p) {
        float *dst = (p & 1) ? xb : xa;
        publish(dst, acc, p);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt + shard * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x < 64) {
            const unsigned target = (unsigned)gridDim.x * (p + 1);
            for (unsigned spins = 0;; ++spins) {
                unsigned v = threadIdx.x < 8 ? __hip_atomic_load(cnt + threadIdx.x * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                for (int o = 4; o >= 1; o >>= 1) v += __shfl_xor(v, o);
                v = __shfl(v, 0);
                if (v >= target) break;
                if (spins > (1u << 24)) {
                    if (threadIdx.x == 0) atomicExch(err, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs(dst, N * 4), threadIdx.x * 16, 0, 16);
        float s = __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        float t = 0.f;
        for (int w = 0; w < T / 64; ++w) t += red[w];
        __syncthreads();
        acc = t * 1e-9f;
    }
    if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// the same phase as its own launch
__global__ __launch_bounds__(T) void k_phase(const float *src, float *dst, int p, float *out) {
    __shared__ float red[T / 64];
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs(src, N * 4), threadIdx.x * 16, 0, 0);
    float s = __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    float t = 0.f;
    for (int w = 0; w < T / 64; ++w) t += red[w];
    if (threadIdx.x < 8) dst[blockIdx.x * 8 + threadIdx.x] = t * 1e-9f + threadIdx.x + p;
    if (threadIdx.x == 0 && p < 0) out[blockIdx.x] = t;
}

int main() {
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int G = ncu;  // one workgroup per CU, all resident
    printf("CUs %d, grid %d x %d\n", ncu, G, T);
    float *xa, *xb, *out;
    unsigned *cnt, *err;
    CK(hipMalloc(&xa, N * 4));
    CK(hipMalloc(&xb, N * 4));
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&cnt, 8 * 32 * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(xa, 0, N * 4));
    CK(hipMemset(xb, 0, N * 4));
    CK(hipMemset(err, 0, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int phases : {1, 142, 1420}) {
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipMemset(cnt, 0, 8 * 32 * 4));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_persistent, dim3(G), dim3(T), 0, 0, xa, xb, cnt, err, phases, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        unsigned herr = 0;
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        printf("persistent: %5d phases  %9.2f us total  %.3f us/phase  err=%u\n", phases, best * 1e3, best * 1e3 / phases, herr);
    }
    // launches, graph-captured
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int phases : {142, 1420}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int p = 0; p < phases; ++p)
            hipLaunchKernelGGL(k_phase, dim3(G), dim3(T), 0, s, (p & 1) ? xa : xb, (p & 1) ? xb : xa, p, out);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("launches:   %5d phases  %9.2f us total  %.3f us/phase\n", phases, best * 1e3, best * 1e3 / phases);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
