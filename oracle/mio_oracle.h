/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference MioTTS hot path, used as the parity
 * checker for the HIP path and as bench.py's CPU baseline ("kind": "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle (oracle/_build/libmiooracle.so). The product library never links it.
 *
 * Each function cites the reference file:line it follows.
 * Pinning status (see DESIGN.md "Oracle"):
 *   - iSTFT             : PINNED to reference istft.cpp built here (oracle/_ref).
 *   - codec forward     : parity unpinned (ggml absent, F1) — follows miocodec.cpp op
 *                         order + documented ggml CPU op semantics.
 *   - LLM decode step   : parity unpinned (llama.cpp absent, F1) — follows documented
 *                         ggml block formats / vec_dot semantics.
 */
#ifndef MIO_ORACLE_H
#define MIO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- iSTFT (istft.cpp:7-108) ---- */
void mo_istft_tables(int n_fft, int win_length, float *cos_tbl, float *sin_tbl, float *nyq,
                     float *hann);
int mo_istft(const float *spec, int n_frames, int n_fft, int win_length, int hop_length,
             float *out);

#ifdef __cplusplus
}
#endif
#endif
