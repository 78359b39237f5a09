// In-launch quantization producer over (token, 2048-element chunk) units, shared by the
// batched down launches (llm_prefill.hip k_pf_ffn_down_q on the dot4 engine, llm_mmq.hip
// k_mmq16 with QM 1 on the matrix cores). Workgroup blockIdx.x = t * nch + c quantizes chunk
// c of src row t (plain rows, K % 256 == 0) with k_bt_quant_split's arithmetic into an LDS
// image of t's act record, copies its code / scale / (Q8_K) bsum ranges out with 16-B
// write-through stores, drains them and adds 1 to each of the 8 counter shards at cnt;
// workgroup 0 first zeroes the other set (the next fused launch's). Also the one-wave-per-
// token RMSNorm + quantization of a launch's own prologue (xpre_issue / xpre_quant). Device
// code only.
#pragma once
#include "llm_device.h"

namespace mio {
namespace {

__device__ __forceinline__ void chunk_quant_producer(const float *src, int K, int kq, int nch, char *act, int *cnt,
                                                     int *other, char *lds) {
    const int t = blockIdx.x / nch, c = blockIdx.x - t * nch;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (blockIdx.x == 0 && threadIdx.x < 8)
        __hip_atomic_store((__attribute__((address_space(1))) int *)(other + 64 * threadIdx.x), 0, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const ActL a = carve_t(lds, K, 0).a;
    if (c * 2048 + wave * 256 < K) {  // wave-uniform
        const float4 x = *reinterpret_cast<const float4 *>(src + (size_t)t * K + c * 2048 + 4 * (int)threadIdx.x);
        const float v[4] = {x.x, x.y, x.z, x.w};
        if (kq)
            q8k_store(v, abs_max4(v), c * 8 + wave, a);
        else
            q80_store(v, c * 64 + wave * 8 + (lane >> 3), true, a);
    }
    __syncthreads();
    // the chunk's ranges of the record: codes [2048 c, +2048), Q8_0 scales [64 c, +64) or Q8_K
    // scales [8 c, +8) and bsums [128 c, +128); a partial last chunk copies its whole 256s only
    const int nsb = min(8, (K - c * 2048) >> 8);
    const int nq = nsb * 16, nd = kq ? (nsb * 4 + 15) / 16 : nsb * 2, nb = kq ? nsb * 2 : 0;
    const auto dst = rsrc(act + (size_t)t * act_bytes(K), (uint32_t)act_bytes(K));
    const int i = threadIdx.x;
    uint32_t off = 0xFFFFFFFFu;
    if (i < nq)
        off = c * 2048 + 16 * i;
    else if (i < nq + nd)
        off = K + (kq ? c * 32 : c * 256) + 16 * (i - nq);
    else if (i < nq + nd + nb)
        off = K + (K / 32 + 8) * 4 + c * 256 + 16 * (i - nq - nd);
    if (off != 0xFFFFFFFFu) {
        const uint4 v = *reinterpret_cast<const uint4 *>(lds + off);
        u32x4 u;
        u.x = v.x, u.y = v.y, u.z = v.z, u.w = v.w;
        __builtin_amdgcn_raw_buffer_store_b128(u, dst, off, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 8)
        __hip_atomic_fetch_add((__attribute__((address_space(1))) int *)(cnt + 64 * threadIdx.x), 1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// In-launch RMSNorm + quantization with the inputs loaded AHEAD of the weights (batched
// decode, K <= 2048, nt <= 8 tokens: wave t quantizes token t). The token row and the norm
// weights sit in registers (lane l, register vw: elements
// vw * 256 + 4 l .. +3, i.e. superblock vw / Q8_0 blocks 8 vw .. 8 vw + 7), issued before the
// first weight group, so the quantization waits only for them (in-order vmcnt) and never
// re-reads the row. The arithmetic is the workgroup prologue's (rmsnorm_quant), replayed by one
// wave: the sum of squares accumulates per virtual thread tid = 64 vw + lane over its elements
// (tid + i MT) * 4 in order, each virtual wave reduces by the same DPP tree (wave_sum_d) and
// the 8 partial sums add in wave order as block_sum does; each superblock / block is quantized
// by q8k_store / q80_store as any wave of the workgroup would, so the records equal
// k_bt_quant's bit for bit. Saves the k_bt_quant launch in front of the matvec.
struct XPre {
    float4 x[MW], w[MW];
};
__device__ __forceinline__ void xpre_issue(const float *src, const float *norm_w, int K, int nt, XPre &xp) {
    const int lane = threadIdx.x & 63;
    const int t = min((int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nt - 1);
    const float *x = src + (size_t)t * K;
#pragma unroll
    for (int vw = 0; vw < MW; ++vw) {
        const int e = min(vw * 256 + 4 * lane, K - 4);
        xp.x[vw] = ld4(x + e);
        xp.w[vw] = ld4(norm_w + e);
    }
}
__device__ __forceinline__ void xpre_quant(const XPre &xp, int K, float eps, bool kq, char *smem, int nt) {
    const int lane = threadIdx.x & 63;
    const int t = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t < nt) {
        const ActL a = carve_t(smem, K, t).a;
        double tot = 0.0;
#pragma unroll
        for (int vw = 0; vw < MW; ++vw) {
            const int e = vw * 256 + 4 * lane;
            const float4 v = xp.x[vw];
            double acc = 0.0;
            if (e < K) {
                acc += (double)(v.x * v.x);
                acc += (double)(v.y * v.y);
                acc += (double)(v.z * v.z);
                acc += (double)(v.w * v.w);
            }
            tot += wave_sum_d(acc);
        }
        const float scale = rms_scale(tot, K, eps);
        auto val4 = [&](int vw, float (&v)[4]) {
            const float4 xv = xp.x[vw], w = xp.w[vw];
            float q;
            q = xv.x * scale, v[0] = q * w.x;
            q = xv.y * scale, v[1] = q * w.y;
            q = xv.z * scale, v[2] = q * w.z;
            q = xv.w * scale, v[3] = q * w.w;
        };
        if (kq) {
#pragma unroll
            for (int b = 0; b < MW; ++b)
                if (b < K / 256) {
                    float v[4];
                    val4(b, v);
                    q8k_store(v, abs_max4(v), b, a);
                }
        } else {
            const int nb = K / 32;
#pragma unroll
            for (int m = 0; m < MW; ++m)
                if (8 * m < nb) {
                    const int b = 8 * m + (lane >> 3);
                    float v[4];
                    val4(m, v);
                    q80_store(v, b, b < nb, a);
                }
        }
    }
    lds_barrier();
}

}  // namespace
}  // namespace mio
