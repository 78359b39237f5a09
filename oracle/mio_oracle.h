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

/* ---- codec forward (miocodec.cpp:519-810) ----
 * Stages for mo_codec_decode_stage (activation copied out after the stage):
 *   0 embed [T][Dp]          1 prenet+proj [T][Dd]   2 ConvT x2 [2T][Dd]
 *   3 wave_prior [2T][Dd]    4 decoder+final AdaLN   5 wave_post [2T][Dd]
 *   6..5+U upsampler stage s [L_s][C_s]               6+U out_proj+snake [L][Dd]
 *   7+U spectrogram [L][n_freq*2]   (U = upsampler stages) */
typedef struct mo_codec mo_codec;
mo_codec *mo_codec_load(const char *path);
void mo_codec_free(mo_codec *c);
void mo_codec_info(const mo_codec *c, int *info /* [8] */);
int mo_codec_n_stages(const mo_codec *c);
int mo_codec_decode_stage(mo_codec *c, const int *codes, int T, const float *emb, int stop_stage,
                          float *out, int *out_rows, int *out_cols);
int mo_codec_decode(mo_codec *c, const int *codes, int T, const float *emb, float *spec);
float mo_f16_round(float f);

#ifdef __cplusplus
}
#endif
#endif
