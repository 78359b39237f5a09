// Weight prefetch into the memory-side Infinity Cache (MALL): a read-only sweep whose data
// is discarded, so the next decode kernels find their weights cached instead of paying the
// HBM miss latency inside a latency-bound launch.
#include "prefetch.h"

namespace mio {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Each thread reads 64 B (four 16-B loads) per iteration; the xor of what it read is
// stored only under a condition no launch meets (sink != nullptr && bytes == 0), so the
// loads cannot be removed.
__global__ __launch_bounds__(256) void k_touch(const uint8_t *p, uint64_t bytes, uint32_t *sink) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, 0x7FFFFFF0, 0x00020000);
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 64;
    for (uint64_t off = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 64; off < bytes; off += stride) {
        const uint32_t base = (uint32_t)(off >> 31 << 31);
        const uint8_t *q = p + base;
        const auto rq = base ? __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(q), 0, 0x7FFFFFF0, 0x00020000) : r;
        const uint32_t o = (uint32_t)(off - base);
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rq, o, 0, 0);
        const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rq, o + 16, 0, 0);
        const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rq, o + 32, 0, 0);
        const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(rq, o + 48, 0, 0);
        acc ^= a.x ^ b.y ^ c.z ^ d.w;
    }
    if (sink && bytes == 0) sink[threadIdx.x] = acc;
}

}  // namespace

void launch_touch(const void *p, uint64_t bytes, int n_wg, hipStream_t s) {
    if (!p || !bytes) return;
    hipLaunchKernelGGL(k_touch, dim3(n_wg), dim3(256), 0, s, (const uint8_t *)p, bytes, (uint32_t *)nullptr);
}

}  // namespace mio
