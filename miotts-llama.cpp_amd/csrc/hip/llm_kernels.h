// Launch interface of the LLM decode-step kernels (csrc/hip/llm_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mio {

// attention positions per chunk (one attention workgroup), = LlmDims::split. Every path
// (decode step, batched decode, prefill) uses the same chunks and the same merge, so their
// results are bit-identical. MIO_ATT_CHUNK: A/B builds (32, 64 or 128); 64 by default
// (profiles/r04_att_chunk_ab.txt: 1.7B decode 0.823 / 0.773 / 0.775 ms per token at 32 / 64 / 128).
#ifndef MIO_ATT_CHUNK
#define MIO_ATT_CHUNK 64
#endif
constexpr int kAttChunk = MIO_ATT_CHUNK;
// step timeline (diagnostic): workgroup slots per launch (k_layer grids reach ~1,300)
constexpr int kTlSlots = 2048;
static_assert(kAttChunk == 32 || kAttChunk == 64 || kAttChunk == 128, "attention chunk");

// One quantized matrix in the split layout (csrc/host/quant.h), rows x k.
struct QMat {
    int type;  // ggml type id: 8 Q8_0, 12 Q4_K, 14 Q6_K
    int rows, k;
    const uint8_t *p0, *p1, *p2, *p3;
};

// Rows [r0, r0 + n) of q as a matrix of its own (every split-layout stream is row-major).
inline QMat qmat_rows(const QMat &q, int r0, int n) {
    size_t rb[4] = {0, 0, 0, 0};
    switch (q.type) {
        case 8: rb[0] = (size_t)q.k, rb[1] = (size_t)q.k / 32 * 2; break;
        case 12: rb[0] = (size_t)q.k / 2, rb[1] = (size_t)q.k / 256 * 16; break;
        case 14: rb[0] = (size_t)q.k / 2, rb[1] = (size_t)q.k / 4, rb[2] = (size_t)q.k / 16, rb[3] = (size_t)q.k / 256 * 2; break;
        default: break;
    }
    QMat v = q;
    v.rows = n;
    v.p0 = q.p0 + rb[0] * r0, v.p1 = q.p1 + rb[1] * r0, v.p2 = q.p2 + rb[2] * r0, v.p3 = q.p3 + rb[3] * r0;
    return v;
}

// Device-resident decode state (read by every kernel of a step; advanced by the sampler),
// so one captured hipGraph replays every token without host involvement.
// The sampler of step t runs inside step t+1's first launch (layer 0 attn_in) and the flush
// launch after the last step: `pending` = the lm_head partials of step `step` are not sampled
// yet, so the token being decoded sits at min(pos + pending, n_ctx - 1) (cur_pos) until
// layer 0's ffn_in folds pending into pos / step.
struct StepState {
    int pos;      // position of the last sampled token (cur_pos: of the token being decoded)
    int step;     // step counter (sampler RNG counter, output slot)
    int token;    // token being decoded
    int done;     // set once an end token was sampled
    int pending;  // 1: lm_head partials of this step await the sampler
};

struct SampleCfg {
    float temp;
    uint32_t seed_lo, seed_hi;
    int lo, hi;          // sampled ids restricted to [lo, hi)
    int eos0, eos1;      // end tokens (-1 = none)
    const int *force;    // force[step] >= 0: next token is forced (prompt prefill), or null
    int n_force;
    int *out_tokens;     // [max_steps] sampled/forced next token per step
    int max_steps;
    int *host_done;      // mapped host word set to 1 with StepState.done (null: none)
};

// lfm2 gated short conv: kernel width (shortconv.l_cache) and the ring of bx values kept per
// layer (slot p & 3 holds position p; positions p-2, p-1 are read while p is written)
constexpr int kConvL = 3;
constexpr int kConvSlots = 4;

struct LayerW {
    const float *attn_norm, *q_norm, *k_norm, *ffn_norm;
    const float *bqkv;  // [(H + 2 Hkv) hd] q|k|v biases (qwen2 attn_{q,k,v}.bias), or null
    QMat wq, wk, wv, wo, gate, up, down;
    // lfm2 short-conv layer (conv != 0; wq..wo unused): in_proj [3 n_embd][n_embd] -> B | C | X,
    // depthwise taps conv_w [n_embd][kConvL] f32, out_proj [n_embd][n_embd]
    int conv;
    QMat in_proj, out_proj;
    const float *conv_w;
};

struct LlmDims {
    int n_embd, n_head, n_kv, hd, n_ff, n_vocab, n_ctx;
    float eps, scale;
    int neox, qk_norm;
    int split;        // attention positions per chunk (kAttChunk)
    int max_splits;
    int n_wg;         // streaming-matvec workgroups (one per CU)
    int n_layer;
};

struct LlmBuffers {
    float *x;          // [n_embd] residual stream
    float *qkv;        // [(H + 2 Hkv) hd]
    float *h;          // [n_ff] ffn activation
    float *logits;     // [n_vocab]
    float *part;       // [H][max_splits][hd + 4] attention chunk partials {O, m, l}
    float *att;        // [H * hd] attention output (chunks merged by the last chunk workgroup)
    int *att_cnt;      // [Hkv] chunk arrival tickets (0 between launches); k_att_o's merge
                       // counters and wait-timeout flag at kRdyOff.. (kAttCntInts in all)
    float *smp;        // sampler partials [2 * n_lm_blocks]
    const float2 *rope;  // [n_ctx][hd/2] (cos, sin)
    StepState *st;
    const SampleCfg *cfg;       // sampling configuration (device-resident: graphs never re-capture)
    unsigned long long *trace;  // optional: per-kernel checkpoint timestamps (workgroup 0, thread 0)
    unsigned long long *tl;     // optional: step timeline {min start, max end} per launch (s_memrealtime)
    int seq;                    // launch index within the step (timeline slot)
    float *ring;   // lfm2: [n_layer][kConvSlots][n_embd] short-conv inputs bx by position
};

// Batched prompt prefill (csrc/hip/llm_prefill.hip): up to kPrefillB prompt tokens per chunk
// go through every layer with ONE weight pass per launch (the prefill llama_decode of
// test-to-speech.cpp:132-148); K/V rows are written, no logits are produced. 128 holds the
// chat-template prompts of the benchmarks (≈70 tokens) in one chunk: a 64-token chunk left
// their last few tokens to a second, dot4 weight pass (+1.5 ms per 68-token prompt).
// Memory: the chunk's attention partials (PrefillBuffers.part) are kPrefillB x n_head x
// ceil(n_ctx / kAttChunk) x (hd + 4) floats: at the default 64-position chunks 35 MB for the 1.7B
// model at n_ctx 2048 and 554 MB at the 32768 maximum (of 288 GB); the merged outputs pb.att
// add kPrefillB x n_head x hd floats (1 MB) and the tickets pb.att_cnt kPrefillB x n_kv ints.
constexpr int kPrefillB = 128;
// The same multi-token layers run the batched decode step of up to kBatchMax utterances.
constexpr int kBatchMax = 16;

// The batched decode step of B independent utterances runs the same layers (one token of
// each per step, weights streamed once for all of them).
struct PrefillBuffers {
    float *x;            // [kPrefillB][n_embd] residual streams
    float *qkv;          // [kPrefillB][(H + 2 Hkv) hd]; q rows are RoPE'd in place (lfm2 conv
                         // layers: [kPrefillB][3 n_embd] B | C | X rows)
    float *h;            // [kPrefillB][n_ff]
    float *part;         // [kPrefillB][H][max_splits][hd + 4] attention chunk partials
    float *att;          // [kPrefillB][H * hd] attention outputs (merged in the attention launch)
    int *att_cnt;        // [kPrefillB][Hkv] chunk arrival tickets (0 between launches)
    const float2 *rope;  // [n_ctx][hd/2]
    const int *tokens;   // device token ids (embedded token t of a chunk at tokens[p0 + t])
    const int *pos;      // position of token t: pos[t * pos_stride] (device-resident)
    const int *seq;      // sequence (KV cache) of token t: seq[t * seq_stride]
    int pos_stride, seq_stride;
    size_t seq_kv;       // K (and V) cache elements per sequence: [seq][layer][kv head][n_ctx][hd]
    float *ring;         // lfm2 short-conv rings [seq][n_layer][kConvSlots][n_embd], or null
    size_t seq_ring;     // ring elements per sequence
    char *act;           // [kPrefillB] quantized activation records of the next matvec
    int *qcnt;           // batched decode, in-launch quantization (launch_mmq_q): 2 sets of 8
                         // counter shards 64 ints apart, then the wait-timeout flag (kQcntFlag)
};
constexpr int kQcntFlag = 1024, kQcntInts = kQcntFlag + 64;
// bytes of the act records (pb.act) for K up to k_max (BF16 weights: pass prefill_rec_k)
size_t prefill_act_bytes(int k_max);
// K of the act record layout for a weight type (2K for BF16: K bf16 values)
int prefill_rec_k(int K, int type);

// One chunk of nt <= kPrefillB tokens (ids at tokens[p0 + t], positions/sequences from
// pb.pos / pb.seq) through every layer: embedding, K/V rows, residual streams in pb.x.
// n_chunks = attention chunks to sweep (>= max position / kAttChunk + 1).
void launch_prefill_chunk(const LlmDims &d, const LayerW *layers, int n_layer, _Float16 *kcache,
                          _Float16 *vcache, const QMat &tok_embd, const PrefillBuffers &pb, int p0, int nt,
                          int n_chunks, hipStream_t s);

// Batched decode of B <= kBatchMax utterances (mio_hip_llm_generate_batch): per sequence b,
// state st[b], sampling cfg[b] (cfg[b].out_tokens = its token ring), logits [B][n_vocab],
// sampler partials smp [B][lm blocks][2]; the residual streams are pb.x[b].
struct BatchBuffers {
    StepState *st;
    const SampleCfg *cfg;
    float *logits;
    float *smp;
};
// One decode step of all B sequences: every layer with one weight pass per launch, the
// lm_head for all B, then per-sequence sampling + next embedding + state advance.
void launch_batch_step(const LlmDims &d, const LayerW *layers, int n_layer, _Float16 *kcache, _Float16 *vcache,
                       const float *out_norm, const QMat &lm, const QMat &tok_embd, const PrefillBuffers &pb,
                       const BatchBuffers &bb, int B, hipStream_t s);
// B streams fit one batched step (B <= kBatchMax and the lm_head's LDS for its weight type)
bool batch_supported(const LlmDims &d, int B, int lm_type);
// Embedding of st[b].token into pb.x[b] for every sequence (decode start).
void launch_batch_embed(const LlmDims &d, const QMat &tok_embd, const PrefillBuffers &pb, const BatchBuffers &bb,
                        int B, hipStream_t s);

// Launch one kernel of a decode step (which: 0 attn_in, 1 attention, 2 attn_out, 3 ffn_in,
// 4 ffn_down of layer il; 6 lm_head, 7 sampler; lfm2 short-conv layers: 8 conv_in, 9
// conv_out in place of 0..2; 10 attention + O (k_att_o, for 1 + 2), 11 the whole attention
// block (k_layer_att, for 0 + 1 + 2), 12 the FFN pair (k_ffn, for 3 + 4), 13 the whole layer
// (k_layer, for 11 + 12)) on stream s.
// an empty one-workgroup launch (the timing reference of mio_hip_llm_time_kernel)
void launch_nop(hipStream_t s);
void launch_step_kernel(int which, const LlmDims &d, const LayerW *layers, int il, _Float16 *kcache,
                        _Float16 *vcache, const float *out_norm, const QMat &lm, const QMat &tok_embd,
                        const LlmBuffers &b, hipStream_t s);
// Embedding of `token` (row of token_embd) -> b.x, and state reset to (pos, token).
void launch_embed_token(const LlmDims &d, const QMat &tok_embd, const LlmBuffers &b, hipStream_t s);
int lm_head_blocks(const LlmDims &d);
// workgroups of a streaming matvec over `rows` rows (at least 8 rows per workgroup, at most
// one workgroup per CU); passes of 2048 weights for K. Kernels recompute it from their
// arguments instead of reading gridDim (an implicit kernel argument, one more scalar-load
// round trip before the first weight load).
__host__ __device__ inline int matvec_grid_n(int n_wg, int rows) {
    int g = rows / 8;
    g = g < n_wg ? g : n_wg;
    return g < 2 ? 2 : g;
}
int matvec_grid(const LlmDims &d, int rows);
// the fused attention + O launch (launch_step_kernel which = 10) exists for this head shape
bool att_o_supported(int hd, int G);
// the whole attention block of layer L as one launch (llm_layer_att.hip, which = 11) exists for
// its shapes and weight types
bool layer_att_supported(const LlmDims &d, const LayerW &L);
// the FFN pair of layer L as one launch (k_ffn, which = 12) exists for its weight types
bool ffn_fused_supported(const LlmDims &d, const LayerW &L);
void launch_layer_att(const LlmDims &d, const LayerW &L, _Float16 *kc, _Float16 *vc, const LlmBuffers &b, bool dg,
                      hipStream_t s);
// the whole decoder layer L (attention block + FFN pair) as one launch (k_layer, which = 13)
// exists for its shapes and weight types; launch_layer runs it for layer il (counter set il & 1)
bool layer_fused_supported(const LlmDims &d, const LayerW &L);
void launch_layer(const LlmDims &d, const LayerW &L, int il, _Float16 *kc, _Float16 *vc, const LlmBuffers &b,
                  bool dg, hipStream_t s);
// MIO_LAYER_GATE (k_layer): 1 = the FFN workgroups issue their weights only once their kv head's
// q|k|v rows are in (the producers' stream goes first), 0 = at dispatch
int layer_ffn_gate();
// k_att_o's merge counters in LlmBuffers.att_cnt: kRdyShards words kRdyStride ints (256 B)
// apart from int kRdyOff on (one per XCD: an O workgroup polls shard blockIdx % 8, so no word
// has more than 1/8 of the pollers; MI355X_MICROARCH "dequeue": one word saturates near 88
// accesses per us), then the wait-timeout flag. Needs n_kv <= kRdyOff.
// Then k_layer_att's q|k|v row counters, one per kv head (at most kQkvMax), kQkvStride apart.
constexpr int kRdyOff = 64, kRdyShards = 8, kRdyStride = 64;
constexpr int kRdyFlag = kRdyOff + kRdyShards * kRdyStride;
constexpr int kQkvOff = kRdyFlag + 64, kQkvStride = 64, kQkvMax = 64;
// Then the fused FFN launch's h counters (k_ffn, which = 12), two levels, every word kFfnStride
// ints apart: kFfnShards arrival shards (gate|up workgroup b adds 1 to shard b % 8: <= 32 adds
// per word at 256 producers; the price list's fan-in on one word is 3.6-4.5 us), then
// kFfnShards ready replicas (the producer whose shard add returns the shard's last count adds 1
// to every replica; a down workgroup polls replica b % 8 until all shards are in: <= 32 pollers
// per word). Zeroed by the launch after k_ffn (the next layer's attn_in / layer_att, lm_head).
constexpr int kFfnOff = kQkvOff + kQkvStride * kQkvMax, kFfnShards = 8, kFfnStride = 64;
constexpr int kFfnRdy = kFfnOff + kFfnShards * kFfnStride;
// The whole-layer launch (k_layer, which = 13) hands the O projection's x rows to its gate|up
// workgroups through one more two-level counter (arrival shards kXOff, ready replicas kXRdy),
// laid out after the counters above. k_layer runs with LlmBuffers.att_cnt pointing at counter
// SET il & 1 (kLaySet ints each, from kLayOff on; every offset above is the same inside a set):
// each k_layer zeroes the other set at entry (used by the previous k_layer: kernel boundary), so
// no counter of a set is reset while a launch may still poll it; lm_head zeroes both.
constexpr int kXOff = kFfnRdy + kFfnShards * kFfnStride, kXRdy = kXOff + kFfnShards * kFfnStride;
constexpr int kLaySet = kXRdy + kFfnShards * kFfnStride;
constexpr int kLayOff = kLaySet;  // the plain counters occupy [0, kLaySet) too
constexpr int kAttCntInts = kLayOff + 2 * kLaySet;
int pick_np(int K);
size_t matvec_lds(int K);
// units (row passes) of the busiest wave of a matvec over `rows` rows on `grid` workgroups,
// and the single-group size that covers them (0 = streaming groups)
int max_wave_units(int rows, int grid, int np, int nm);
int pick_su(int units, int np);
// Layer il's first launch (llm_attn_in.hip): RMSNorm + q|k|v matvec (+ layer 0: the
// previous step's sampler).
void launch_attn_in(const LlmDims &d, const LayerW &L, int il, const QMat &tok_embd, const LlmBuffers &b, bool dg,
                    hipStream_t s);
// y = W x with x re-quantized to the vec_dot_type (parity test of the matvec kernels).
void launch_debug_matvec(const QMat &W, const float *x, float *y, int n_wg, hipStream_t s);
// y[t][rows] = W x[t] for nt tokens on the int8-MFMA multi-token matmul (act: scratch of
// nt * debug_act_bytes(W.k) bytes); mode 0 store, 1 y += W x, 2 y = silu(W x) * (up x).
size_t debug_act_bytes(int K);
void launch_debug_mmq(const QMat &W, const QMat &up, int mode, const float *x, int nt, char *act, float *y,
                      hipStream_t s);

}  // namespace mio
