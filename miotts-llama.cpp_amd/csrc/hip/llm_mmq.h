// Launch interface of the int8-MFMA multi-token matmul (csrc/hip/llm_mmq.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "llm_kernels.h"

namespace mio {

enum MmqMode { MMQ_STORE = 0, MMQ_RESID = 1, MMQ_SWIGLU = 2 };

// One matrix of a launch: its rows go to out[t * ld + out_off + row]; tiles = mmq_tiles(rows).
struct MmqSeg {
    QMat w;
    int tiles;
    int out_off;
};

struct MmqArgs {
    const char *act;    // nt activation records (k_bt_quant), act_stride bytes apart
    size_t act_stride;
    int K;              // reduction length (the matrices' k)
    int nt;             // tokens
    float *out;         // MMQ_STORE: out = v; MMQ_RESID: out = v + out; MMQ_SWIGLU: silu(v) * v_up
    int ld;             // token stride of out (floats)
    QMat w_up;          // MMQ_SWIGLU: the up matrix (same rows / type as segment 0)
};

// In-launch quantization of the matmul's input (launch_mmq_q, batched decode): nt producer
// workgroups at the front of the grid quantize token t's input (mode 0: RMSNorm(src[t]) *
// norm_w, 1: src[t] as is; k = the matrices' K) into its act record exactly as k_bt_quant
// does, store the record write-through and add 1 to each of the 8 counter shards cnt[64 i];
// every 16x16 tile waits for nt adds on shard blockIdx % 8 (after issuing its first weight
// loads where the path allows) before its first activation read. The shards must be zero at
// launch; the launch zeroes `other` (the next fused launch's set).
struct MmqQuant {
    const float *src;
    const float *norm_w;
    int mode;
    float eps;
    int *cnt;
    int *other;
    int *flag;
    int early = 0;  // set by launch_mmq_q: K-quant tiles issue their weight loads before the wait
};

int mmq_tiles(int rows);
// Segments 0..nseg-1 (types: ggml ids 8 / 12 / 14; with 3 segments, 0 and 1 share a type).
void launch_mmq(const MmqSeg *seg, const int *types, int nseg, int mode, const MmqArgs &a, hipStream_t s);
// The same with the input quantized in the launch (MmqQuant); false (nothing launched) when
// this shape has no fused kernel: the caller then runs the quantization launch + launch_mmq.
bool launch_mmq_q(const MmqSeg *seg, const int *types, int nseg, int mode, const MmqArgs &a, const MmqQuant &q,
                  hipStream_t s);

}  // namespace mio
