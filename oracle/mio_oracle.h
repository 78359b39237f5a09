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
/* Teacher forcing (tests): stages start_stage .. stop_stage run on `in`, the output of stage
 * start_stage - 1 (e.g. the GPU's), instead of on the oracle's own earlier stages. */
int mo_codec_stage_from(mo_codec *c, const int *codes, int T, const float *emb, int start_stage, const float *in,
                        int stop_stage, float *out, int *out_rows, int *out_cols);
float mo_f16_round(float f);

/* ---- streaming emission (test-to-speech.cpp:367-417,496-571), stream_ref.c ---- */
long mo_stream_emit(mo_codec *c, const float *emb, const int *codes, int n_codes, int check_interval,
                    int holdback, int min_commit, long chunk_samples, float *out, long out_cap,
                    long long *chunks, long chunk_cap, long *n_chunks, int *n_decodes);

/* ---- LLM decode step (llama_decode, test-to-speech.cpp:178-185) and sampler ---- */
typedef struct mo_llm mo_llm;
mo_llm *mo_llm_load(const char *path, int n_ctx);
void mo_llm_free(mo_llm *m);
/* info[8] = {n_vocab, n_embd, n_layer, n_head, n_head_kv, head_dim, n_ff, n_ctx} */
void mo_llm_info(const mo_llm *m, int *info);
void mo_llm_reset(mo_llm *m);
int mo_llm_eval(mo_llm *m, int token, int pos, float *logits /* [n_vocab] or NULL */);
/* the pieces of one eval: embedding row; decoder layer il at pos (writes its K/V row pos);
 * final norm + lm_head; F16 K/V rows [0, n_pos) of layer il as [n_kv][n_pos][hd] (set = 0:
 * copy out of the cache, 1: into it) */
int mo_llm_embed(mo_llm *m, int token, float *x);
int mo_llm_layer(mo_llm *m, int il, int pos, const float *x_in, float *x_out);
void mo_llm_head(mo_llm *m, const float *x, float *logits);
int mo_llm_kv(mo_llm *m, int il, int n_pos, uint16_t *k, uint16_t *v, int set);
float mo_gumbel(uint64_t seed, int step, int idx);
int mo_sample(const float *logits, float temp, uint64_t seed, int step, int lo, int hi);
int mo_set_threads(int n);
/* ggml block helpers (quant_ref.c) */
float mo_fp16_to_f32(uint16_t h);
uint16_t mo_f32_to_fp16(float f);
void mo_quantize_q8_0(const float *x, int64_t k, uint16_t *d, int8_t *qs);
void mo_quantize_q8_K(const float *x, int64_t k, float *d, int8_t *qs, int16_t *bsums);
int mo_dequantize_row(uint32_t type, const uint8_t *row, int64_t k, float *y);
int mo_matvec(uint32_t type, const uint8_t *w, int rows, int64_t k, const float *x, float *y);

#ifdef __cplusplus
}
#endif
#endif
