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

int mmq_tiles(int rows);
// Segments 0..nseg-1 (types: ggml ids 8 / 12 / 14; with 3 segments, 0 and 1 share a type).
void launch_mmq(const MmqSeg *seg, const int *types, int nseg, int mode, const MmqArgs &a, hipStream_t s);

}  // namespace mio
