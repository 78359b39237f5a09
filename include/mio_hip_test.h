/* Test-support C-ABI: libmiotts_test.so (csrc/testlib/), built beside libmiotts.so and linked
 * to it; the product library exports none of these. Used by tests/, bench.py and tools/:
 * synthetic model files (no real GGUF exists offline) and parity entry points of the kernels. */
#ifndef MIO_HIP_TEST_H
#define MIO_HIP_TEST_H

#include "mio_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parity helpers: y[rows] = W x for a GGUF-layout quantized matrix (gguf_rows, ggml type
 * 8/12/14) with x re-quantized to the ggml vec_dot_type, on the GPU matvec kernels; and
 * the host quantizer used to build synthetic models (ggml block layout out). */
int mio_hip_debug_matvec(mio_hip_device *d, uint32_t type, const void *gguf_rows, int rows, int k,
                         const float *x, float *y);
int mio_quantize_rows(uint32_t type, const float *x, int rows, int k, void *out);
/* Parity helper: y[t][rows] = W x[t] for nt activation rows x[t][k] on the batched-prefill
 * matmul (int8 MFMA, csrc/hip/llm_mmq.hip); each row equals mio_hip_debug_matvec of x[t].
 * mode 0: y = W x; 1: y = W x + y (y in/out, the residual epilogue); 2: y = silu(W x) *
 * (Wup x) with gguf_up the up matrix (the SwiGLU epilogue). */
int mio_hip_debug_mmq(mio_hip_device *d, uint32_t type, const void *gguf_rows, int rows, int k,
                      const float *x, int nt, int mode, const void *gguf_up, float *y);

/* ---------------- synthetic model files ----------------
 * No GGUF model files exist offline. These write files with the
 * reference's tensor names and KV keys (miocodec.cpp:448-481, 599-728;
 * create_voice_emb.py:125-129) filled with seeded N(0, s) weights.
 * preset 0 = MioCodec-25Hz-44.1kHz shapes, 1 = tiny test codec. */
int mio_synth_codec_gguf(const char *path, int preset, uint64_t seed);
int mio_synth_voice_gguf(const char *path, uint64_t seed);
/* Synthetic LLM (llama.cpp GGUF conventions, byte-level vocab + 12,800 speech tokens):
 * preset 0 tiny Q8_0, 1 tiny Q4_K_M, 2 "0.1B" Q8_0, 3 "1.7B" Q4_K_M, 4 "2.6B" Q8_0,
 * 5 tiny Q8_0 qwen2 with attn_{q,k,v}.bias. */
int mio_synth_llm_gguf(const char *path, int preset, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* MIO_HIP_TEST_H */
