/*
 * mio_hip.h — thin C-ABI over the MI355X (gfx950) MioTTS hot path.
 *
 * Plain pointers and sizes only; no HIP or torch types in any signature
 * (streams are passed as `void *` = hipStream_t, NULL = the handle's own stream).
 * Every function returns an int status (MIO_OK = 0) unless noted; the text of the
 * last failure on the calling thread is in mio_hip_last_error().
 *
 * Buffers are caller-owned. Pointer arguments are HOST memory unless the matching
 * MIO_*_DEVICE flag says they are device memory of the handle's GPU.
 * One handle per device; a handle is used from one host thread at a time
 * (the reference TestToSpeech is single-threaded per instance, test-to-speech.h:26).
 *
 * Which reference interface each entry point replaces is cited per function.
 */
#ifndef MIO_HIP_H
#define MIO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIO_OK 0
#define MIO_ERR_INVALID (-1)
#define MIO_ERR_HIP (-2)
#define MIO_ERR_IO (-3)
#define MIO_ERR_FORMAT (-4)
#define MIO_ERR_OOM (-5)
#define MIO_ERR_UNSUPPORTED (-6)

/* buffer-location flags */
#define MIO_IN_DEVICE 1u
#define MIO_OUT_DEVICE 2u
/* codec decode: reuse the prenet rows of the previous MIO_CODEC_INCREMENTAL decode of the
 * same handle for the shared code prefix whose receptive field was complete (streaming
 * re-decodes, test-to-speech.cpp:526-529; host codes only, otherwise ignored) */
#define MIO_CODEC_INCREMENTAL 4u

typedef struct mio_hip_device mio_hip_device;
typedef struct mio_hip_istft mio_hip_istft;
typedef struct mio_hip_codec mio_hip_codec;
typedef struct mio_hip_llm mio_hip_llm;
typedef struct mio_tokenizer mio_tokenizer;

/* ---------------- device / memory ---------------- */
const char *mio_hip_last_error(void);
int mio_hip_device_count(int *n);
/* Opens GPU `dev` and creates its default stream. */
int mio_hip_device_open(int dev, mio_hip_device **out);
void mio_hip_device_close(mio_hip_device *d);
int mio_hip_device_sync(mio_hip_device *d);
/* Number of compute units of the opened device (256 on MI355X). */
int mio_hip_device_cu_count(const mio_hip_device *d, int *n_cu);
int mio_hip_malloc(mio_hip_device *d, size_t bytes, void **dptr);
int mio_hip_free(mio_hip_device *d, void *dptr);
int mio_hip_memcpy_h2d(mio_hip_device *d, void *dst, const void *src, size_t bytes);
int mio_hip_memcpy_d2h(mio_hip_device *d, void *dst, const void *src, size_t bytes);
int mio_hip_memset(mio_hip_device *d, void *dst, int value, size_t bytes);

/* Event timer on the handle's stream (or `stream`): returns ms between two marks.
 * mio_hip_timer_mark(d, stream, slot) records event `slot` (0..15). */
int mio_hip_timer_mark(mio_hip_device *d, void *stream, int slot);
int mio_hip_timer_elapsed(mio_hip_device *d, int slot_a, int slot_b, float *ms);

/* PCM epilogue on the device: the optional peak normalisation of test-to-speech.cpp:232-243
 * (gain 0.95 / max|s| when max|s| > 1e-8; skipped when normalize == 0) and the sample
 * conversion of wav_write (wav-writer.cpp:24-44: int16(clamp(s * 32767)), truncated) of n
 * samples. samples (16-byte aligned) and pcm16 are device pointers; the 44-byte RIFF header
 * stays with the host writer. peak (host, may be NULL) receives max|s| of the normalising pass
 * (0 when normalize == 0) and synchronizes the stream. Bit-exact with the host path and the
 * reference's x86 bytes (NaN -> 0). Scratch is per call (stream-ordered): calls on different
 * streams may overlap. */
int mio_hip_pcm_finish(mio_hip_device *d, const float *samples, int64_t n, int normalize,
                       int16_t *pcm16, float *peak, void *stream);
/* The peak normalisation alone (test-to-speech.cpp:232-243 / :289-298) on device floats:
 * out[i] = samples[i] * 0.95 / max|s| when max|s| > 1e-8, else samples[i]; out may equal
 * samples (in place). peak as in mio_hip_pcm_finish. Bit-exact with the host loop. */
int mio_hip_pcm_normalize(mio_hip_device *d, const float *samples, int64_t n, float *out,
                          float *peak, void *stream);

/* ---------------- iSTFT ----------------
 * Replaces istft_cache(n_fft, win_length) (istft.h:6-30, istft.cpp:7-32) and
 * istft(spec, n_frames, hop, cache) (istft.h:38-42, istft.cpp:68-108).
 * spec: [n_frames][n_fft/2+1][2] f32 (re, im) — the layout miocodec_decode returns
 * (miocodec.cpp:801-808). out: (n_frames-1)*hop + win - 2*((win-hop)/2) samples
 * (= hop*n_frames when win-hop is even); *out_len receives that count (0 if empty,
 * like the reference's empty vector). */
int mio_hip_istft_create(mio_hip_device *d, int n_fft, int win_length, mio_hip_istft **out);
void mio_hip_istft_destroy(mio_hip_istft *h);
int mio_hip_istft_out_len(const mio_hip_istft *h, int n_frames, int hop_length, int *out_len);
int mio_hip_istft_run(mio_hip_istft *h, const float *spec, int n_frames, int hop_length,
                      float *out, int *out_len, unsigned flags, void *stream);

/* ---------------- MioCodec decoder ----------------
 * Replaces miocodec_load (miocodec.h:10, miocodec.cpp:426-504): weights are read once
 * and uploaded once to the handle's GPU. */
int mio_hip_codec_load(mio_hip_device *d, const char *gguf_path, mio_hip_codec **out);
void mio_hip_codec_free(mio_hip_codec *c);
/* info[8] = {sample_rate, n_fft, hop_length, samples_per_token, n_freq, upsampler_stages,
 *            frames_per_code, n_codes}  (miocodec.h:38-41 accessors) */
int mio_hip_codec_info(const mio_hip_codec *c, int *info);
/* Replaces miocodec_decode (miocodec.h:28-34, miocodec.cpp:519-810): codes[n_codes] int32,
 * global_emb[128] f32 -> out_spec [frames][n_freq][2] f32 with frames = n_codes *
 * frames_per_code (*out_frames). MIO_IN_DEVICE: codes/emb are device pointers (codes are
 * then not range-checked on the host); MIO_OUT_DEVICE: out_spec is a device pointer. */
int mio_hip_codec_decode(mio_hip_codec *c, const int32_t *codes, int n_codes,
                         const float *global_emb, float *out_spec, int *out_frames,
                         unsigned flags, void *stream);
/* codec + fused iSTFT (test-to-speech.cpp:264-287 without the host round trip):
 * out_pcm receives n_codes * samples_per_token samples (*out_len). */
int mio_hip_codec_decode_pcm(mio_hip_codec *c, const int32_t *codes, int n_codes,
                             const float *global_emb, float *out_pcm, int *out_len,
                             unsigned flags, void *stream);
/* B independent utterances (test-to-speech.cpp:264-287 per utterance), each through codec +
 * fused iSTFT into out_pcm[b] (*out_len[b] samples): the decodes run on up to
 * MIO_CODEC_STREAMS (default 3) streams at once, each with its own workspace, so one decode's
 * small GEMM grids and row kernels leave the CUs to the others; every utterance's arithmetic is
 * mio_hip_codec_decode_pcm's (same kernels, same tiling: bit-identical PCM). Joined on `stream`
 * before return. Flags as mio_hip_codec_decode_pcm (no MIO_CODEC_INCREMENTAL). */
int mio_hip_codec_decode_pcm_batch(mio_hip_codec *c, const int32_t *const *codes, const int *n_codes, int B,
                                   const float *global_emb, float *const *out_pcm, int *out_len,
                                   unsigned flags, void *stream);
/* Debug/parity: run up to `stage` and copy that activation to host `out` (stage list as
 * in oracle/mio_oracle.h: 0 embed .. 7+U spectrogram). rows/cols receive its shape. */
int mio_hip_codec_decode_stage(mio_hip_codec *c, const int32_t *codes, int n_codes,
                               const float *global_emb, int stage, float *out, int *rows,
                               int *cols);

/* ---------------- LLM decode ----------------
 * Replaces llama_model_load_from_file + llama_init_from_model (test-to-speech.cpp:47-49,
 * :103-108): GGUF "llama" / "mistral" / "qwen2" / "qwen3" / "lfm2" (short-conv hybrid) with
 * Q8_0 / Q4_K / Q6_K matrices (Q4_K_M),
 * F16 KV cache of n_ctx positions (0 -> 2048, :104). */
int mio_hip_llm_load(mio_hip_device *d, const char *gguf_path, int n_ctx, mio_hip_llm **out);
void mio_hip_llm_free(mio_hip_llm *m);
/* info[8] = {n_vocab, n_embd, n_layer, n_head, n_head_kv, head_dim, n_ff, n_ctx} */
int mio_hip_llm_info(const mio_hip_llm *m, int *info);
/* Algorithmic HBM bytes streamed per decode step (all matrices incl. lm_head, norms;
 * one embedding row), the numerator of the decode-step roofline. */
int mio_hip_llm_weight_bytes(const mio_hip_llm *m, uint64_t *bytes);
/* Teacher-forced llama_decode of `token` at `pos` (KV cache of positions < pos must hold
 * earlier evals); logits[n_vocab] to host (NULL = skip). Parity entry point. */
int mio_hip_llm_eval(mio_hip_llm *m, int32_t token, int pos, float *logits);
/* The prefill llama_decode of test-to-speech.cpp:132-148 (logits for the last token only,
 * :138): positions 0..n_tokens-2 go through the batched prefill (one weight pass per chunk
 * of prompt tokens), the last token through one decode step; logits[n_vocab] to host (NULL
 * = skip). The KV cache then holds positions < n_tokens. */
int mio_hip_llm_prefill(mio_hip_llm *m, const int32_t *tokens, int n_tokens, float *logits);
/* Copies the logits of the last step to host. */
int mio_hip_llm_logits(mio_hip_llm *m, float *logits);
/* run_llm (test-to-speech.cpp:94-199): prefill prompt[n_prompt], then up to max_tokens
 * sampled tokens with temperature + seeded sampling restricted to ids [allow_lo, allow_hi)
 * (-1 = whole vocab); stops at eos0/eos1 (the end token itself is not returned). Sampling is
 * on the device (Gumbel-max over a counter-based hash of (seed, step, id)); temperature <= 0 is
 * greedy. The sampler stores the end token's flag to a mapped host word, and the host stops
 * issuing step graphs (8 steps each, at most 2 queued ahead) once it is set; check_interval is
 * accepted for ABI compatibility and no longer paces the stop (round 6). */
int mio_hip_llm_generate(mio_hip_llm *m, const int32_t *prompt, int n_prompt, int max_tokens,
                         float temperature, uint64_t seed, int32_t allow_lo, int32_t allow_hi,
                         int32_t eos0, int32_t eos1, int32_t check_interval,
                         int32_t *out_tokens, int *n_out);
/* B independent run_llm calls (test-to-speech.cpp:94-199, one per utterance in the
 * reference) decoded together on this device: every step streams the weights once for all
 * B streams (1 <= B <= 16). prompts = the B prompts concatenated, prompt_lens[B]; stream b
 * uses seeds[b] and returns its tokens in out_tokens[b * max_tokens ...], n_out[b] of them
 * (stopping before an end token as mio_hip_llm_generate does). Each stream's tokens equal
 * mio_hip_llm_generate of its prompt with its seed. Uses its own KV caches (B x the model's),
 * allocated on first use. */
int mio_hip_llm_generate_batch(mio_hip_llm *m, const int32_t *prompts, const int32_t *prompt_lens, int B,
                               int max_tokens, float temperature, const uint64_t *seeds, int32_t allow_lo,
                               int32_t allow_hi, int32_t eos0, int32_t eos1, int32_t check_interval,
                               int32_t *out_tokens, int32_t *n_out);

/* Parity helpers: one decode step of `token` at `pos` (as mio_hip_llm_eval), its residual
 * stream before layer 0 and after every layer into x_layers[(n_layer + 1) * n_embd] (and the
 * logits when not null); the F16 K / V cache rows [0, n_pos) of layer il as
 * [n_kv][n_pos][head_dim] half-precision bit patterns. */
int mio_hip_llm_eval_layers(mio_hip_llm *m, int32_t token, int pos, float *x_layers, float *logits);
int mio_hip_llm_kv_rows(mio_hip_llm *m, int il, int n_pos, uint16_t *k, uint16_t *v);

/* Live timing of one decode-step kernel (which: 0 attn_in, 1 attention, 2 attn_out,
 * 3 ffn_in, 4 ffn_down, 8 conv_in, 9 conv_out, 10 attention + O, 11 the attention block,
 * 12 the FFN pair, of the first layer at or after n_layer/2 that has it; 6 lm_head): `iters`
 * back-to-back launches on
 * the runner's stream between HIP events (state/buffers of the last generate/eval).
 * *avg_ms = mean duration; *bytes = algorithmic HBM bytes per launch (attention: K/V rows of
 * positions <= the decode state's pos, q|k|v, chunk partials). */
int mio_hip_llm_time_kernel(mio_hip_llm *m, int which, int iters, float *avg_ms, uint64_t *bytes);
/* Diagnostic: one launch of kernel `which` with in-kernel checkpoint tracing; out[0..15]
 * = s_memtime (shader clock) at checkpoints of workgroup 0 / thread 0 (0 = not reached),
 * out[16] / out[31] = s_memrealtime (100 MHz) at the first / last checkpoint. */
int mio_hip_llm_trace_kernel(mio_hip_llm *m, int which, uint64_t *out);
/* Diagnostic: one decode step replayed as a graph with the step timeline on; out has
 * max_launches * 512 * 8 slots: out[(i * 512 + w) * 8 + k] = start (k 0) / marks (1-6) /
 * end (7) (s_memrealtime, 100 MHz; 0 = not recorded) of workgroup w (mod 512) of launch i
 * (the order of mio_hip_llm_step_kinds). Marks: matvec launches 1 =
 * weight loads issued, 2 = activations quantized; attention 1 = K/V loads issued, 2 = heads
 * prepared; 3-6 = prologue steps in -DMIO_TL_DIAG builds.
 * Advances the decode state. */
int mio_hip_llm_timeline(mio_hip_llm *m, uint64_t *out, int max_launches, int *n_launches);
/* The launches of one decode step in order, as the `which` of mio_hip_llm_time_kernel: per
 * layer 0 attn_in, 1 attention, 2 attn_out (or 10 / 11: fused), or for an lfm2 short-conv
 * layer 8 conv_in, 9 conv_out; then 3 ffn_in, 4 ffn_down (or 12: fused); last 6 lm_head. *n = the count; kinds may be null (count only), else it needs
 * cap >= *n entries. */
int mio_hip_llm_step_kinds(const mio_hip_llm *m, int *kinds, int cap, int *n);
/* lfm2 short-conv state of layer il: [4][n_embd] floats, slot p & 3 = the B*X row of position
 * p (parity tests). set = 0 copies it out, 1 in. Error for an attention layer. */
int mio_hip_llm_conv_ring(mio_hip_llm *m, int il, float *ring, int set);
/* Wall time (ms) of mio_hip_llm_load: GGUF mmap, re-layout into pinned staging buffers,
 * asynchronous copies into the HBM weight arena (double-buffered). */
int mio_hip_llm_load_ms(const mio_hip_llm *m, double *ms);
/* Decode steps (one sampled token each) issued since the last generate began, look-ahead
 * included: generate keeps up to 2 step graphs queued ahead of the GPU, so a run that stops at
 * an end token after n_out tokens issued *steps - n_out - 1 steps for nothing (the rest of the
 * end token's graph plus at most one more: <= 15; 0 when it stops at max_tokens). */
int mio_hip_llm_steps_issued(const mio_hip_llm *m, int *steps);
/* Cost of those steps after the last mio_hip_llm_generate that stopped at an end token
 * (test-to-speech.cpp:168-170 decodes nothing after it): every decode launch after the end
 * token returns at entry (StepState.done), so such a step costs about its launch boundaries.
 * *steps = steps issued after the end token's step (0 when the run stopped at max_tokens);
 * *timed_steps / *timed_ms = the step graphs queued after the one that sampled the end token
 * and their GPU time (HIP events; 0 when none was queued). */
int mio_hip_llm_tail(const mio_hip_llm *m, int *steps, int *timed_steps, float *timed_ms);
/* Allocates now the device memory decodes of up to n_codes codes need (workspace, RoPE
 * table, incremental prenet cache), as miocodec_load's graph-allocator reserve
 * (miocodec.cpp:424-516); later decodes of at most n_codes allocate nothing. */
int mio_hip_codec_reserve(mio_hip_codec *c, int n_codes);
/* Prenet rows the last mio_hip_codec_decode_pcm took from the incremental cache. */
int mio_hip_codec_last_reused(const mio_hip_codec *c, int *rows);
/* Algorithmic FLOPs of the last mio_hip_codec_decode_pcm (2 per multiply-add of every GEMM,
 * conv and banded-attention dot product it issued; iSTFT excluded): the numerator of the
 * codec's compute roofline against the 157.3 TF f32 MFMA peak. */
int mio_hip_codec_last_flops(const mio_hip_codec *c, double *flops);
/* Stage times (ms, HIP events) of the last mio_hip_codec_decode_pcm: [0] codec, [1] iSTFT. */
int mio_hip_codec_last_timings(const mio_hip_codec *c, float *ms2);

/* ---------------- host text / file utilities ----------------
 * normalize_tts_text (text-normalize.h:7), parse_speech_tokens (token-parser.h:8) and the
 * WAV image wav_write writes (wav-writer.h:6), for FFI callers and tests. */
int mio_normalize_tts_text(const char *text, char *out, int cap, int *out_len);
int mio_parse_speech_tokens(const char *text, int32_t *codes, int cap, int *n);
int mio_wav_encode(const float *samples, int n, int sample_rate, uint8_t *out, int cap, int *out_len);

/* ---------------- GGUF tokenizer ----------------
 * Replaces llama_tokenize(vocab, text, add_special, parse_special) (test-to-speech.cpp:117-125),
 * llama_token_to_piece(..., special=true) (:173-176), llama_vocab_eos (:150) and the
 * "<|im_end|>" lookup (:151-159) for gpt2-type (byte-level BPE) and llama-type (SPM) GGUF
 * vocabularies.
 * info[4] = {n_vocab, bos, eos, im_end (-1 if not a single token)}. */
int mio_tokenizer_load(const char *gguf_path, mio_tokenizer **out);
void mio_tokenizer_free(mio_tokenizer *t);
int mio_tokenizer_info(const mio_tokenizer *t, int *info);
int mio_tokenize(const mio_tokenizer *t, const char *text, int add_special, int parse_special, int32_t *out,
                 int cap, int *n);
int mio_token_piece(const mio_tokenizer *t, int32_t id, char *out, int cap, int *len);
/* Streaming commit cadence (test-to-speech.cpp:496-571) for n_tokens speech tokens:
 * number of codec decode calls and total decoded codes (KAT: 700 -> 18 / 7160). */
int mio_stream_cadence(int n_tokens, int *decode_calls, int64_t *decoded_codes);

#ifdef __cplusplus
}
#endif
#endif /* MIO_HIP_H */
