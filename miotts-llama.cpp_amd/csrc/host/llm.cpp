// LLM decode runner (see llm.h): GGUF load -> split-layout weights in HBM, F16 KV cache,
// one hipGraph per decode step, device-side sampling, C-ABI (include/mio_hip.h).
//
// Replaces, for the MioTTS path: llama_model_load_from_file (test-to-speech.cpp:47-49),
// llama_init_from_model (:103-108), the prefill llama_decode (:132-148), the decode loop
// llama_sampler_sample / llama_decode (:164-192) and the temp+dist sampler chain (:127-130).
#include "llm.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "common.h"
#include "gguf.h"
#include "llm_kernels.h"
#include "quant.h"

struct Stager;
void stager_free(Stager *s);

struct mio_hip_llm {
    mio_hip_device *d = nullptr;
    mio::LlmDims dims{};
    int n_layer = 0;
    std::vector<mio::LayerW> layers;
    mio::QMat tok{}, lm{};
    float *out_norm = nullptr;
    _Float16 *kc = nullptr, *vc = nullptr;
    mio::LlmBuffers buf{};
    int *d_tokens = nullptr, *d_force = nullptr, *d_prompt = nullptr;
    mio::PrefillBuffers pf{};  // batched prompt prefill (kPrefillB tokens per chunk)
    int *d_iota = nullptr;     // 0, 1, ..., n_ctx - 1 (prefill positions; batch stream ids)
    // batched decode of B utterances (mio_hip_llm_generate_batch), allocated on first use
    struct Batch {
        int B = 0;
        _Float16 *kc = nullptr, *vc = nullptr;  // [B][layer][kv head][n_ctx][hd]
        mio::StepState *st = nullptr;
        mio::SampleCfg *cfg = nullptr;
        float *logits = nullptr, *smp = nullptr;
        int *tokens = nullptr;                  // [B][n_ctx] token rings
        int *ppos = nullptr, *pseq = nullptr, *ptok = nullptr;  // flattened prompt prefill lists
        float *ring = nullptr;  // lfm2: [B][n_layer][kConvSlots][n_embd] short-conv rings
        hipGraphExec_t graph = nullptr, graph_n = nullptr;
        std::vector<void *> allocs;
    } bt;
    int max_steps = 0;
    std::vector<void *> allocs;
    uint64_t weight_bytes = 0;
    // BF16 matrices: the multi-token engine runs them on its streaming dot engine with bf16
    // act records (rec_k) when every matrix is BF16 and no layer is an lfm2 short conv (whose
    // in_proj / out_proj are on the int8 matrix cores); otherwise (bf16_mt false) the prompt is
    // prefilled as forced decode steps and batched decode is refused
    bool bf16 = false, int8 = false, has_conv = false;
    bool bf16_mt() const { return !bf16 || (!int8 && !has_conv); }
    // all quantized matrices live in one arena, in the order a step streams them
    uint8_t *arena = nullptr;
    std::map<std::string, size_t> arena_off;

    // decode-step graphs, captured once (the sampling config is device-resident):
    // one step, and graph_steps() steps back to back (fewer graph launches per token)
    hipGraphExec_t graph = nullptr, graph_n = nullptr;
    // prompt prefills replayed as graphs, by prompt length (the first prefill of a length runs
    // eagerly and is captured: ~280 launches that eager issue makes host-bound)
    std::map<int, hipGraphExec_t> prefill_graphs;
    std::map<int, int> prefill_seen;  // eager prefills per prompt length (capture on the second)
    mio::SampleCfg *d_cfg = nullptr;
    float *d_layers = nullptr;  // mio_hip_llm_eval_layers' residual snapshots (parity tests)
    // generation state
    int n_prompt = 0, max_new = 0, steps_total = 0, steps_issued = 0;
    mio::SampleCfg cfg{};
    double load_ms = 0.0;  // wall time of mio_hip_llm_load (GGUF mmap -> HBM arena)
    Stager *stager = nullptr;  // weight upload staging (load only)
    // token-ring snapshots (pinned host mirrors of the state and the ring): llm_run enqueues
    // one behind its steps, llm_poll waits for the OLDEST one, so a caller can enqueue the next
    // interval before it waits for the previous (the GPU never idles at a poll)
    struct Snap {
        hipEvent_t ev = nullptr;
        mio::StepState *st = nullptr;
        int *tok = nullptr;
        int hi = 0, issued = 0;
    };
    static constexpr int kSnaps = 2;
    Snap snaps[kSnaps];
    int snap_head = 0, snap_n = 0;  // oldest outstanding snapshot, number outstanding
    // steps run after the end token of the last generate (mio_hip_llm_tail): slot of the
    // snapshot whose poll found it (-1: none), steps issued in total after it, and the GPU
    // time of the whole intervals queued behind that snapshot
    int eos_snap = -1, tail_steps = 0, tail_timed_steps = 0;
    float tail_ms = 0.0f;
    // end-token words the samplers store to host memory (pinned, mapped: [0] the single-stream
    // decode, [1 + b] batched stream b), so the host stops enqueuing steps without a blocking
    // poll; and one event per step graph of the running generate (flow control: at most
    // kRunDepth graphs queued ahead of the GPU; the tail timing)
    int *host_done = nullptr, *host_done_dev = nullptr;
    std::vector<hipEvent_t> run_ev;
    int run_base = 0, run_graphs = 0;  // steps issued before the first graph; graphs issued

    ~mio_hip_llm() {
        if (d) hipSetDevice(d->dev);
        if (graph) hipGraphExecDestroy(graph);
        if (graph_n) hipGraphExecDestroy(graph_n);
        for (auto &kv : prefill_graphs) hipGraphExecDestroy(kv.second);
        if (bt.graph) hipGraphExecDestroy(bt.graph);
        if (bt.graph_n) hipGraphExecDestroy(bt.graph_n);
        for (void *p : bt.allocs) hipFree(p);
        for (void *p : allocs) hipFree(p);
        stager_free(stager);
        if (host_done) hipHostFree(host_done);
        for (hipEvent_t e : run_ev) hipEventDestroy(e);
        for (Snap &sn : snaps) {
            if (sn.ev) hipEventDestroy(sn.ev);
            if (sn.st) hipHostFree(sn.st);
            if (sn.tok) hipHostFree(sn.tok);
        }
    }
};

namespace {

}  // namespace

// Host -> HBM weight upload: every matrix is re-laid out (to_split) from the mmapped GGUF
// straight into one of two pinned staging buffers while the other buffer's DMA copy runs
// (hipMemcpyAsync on a load stream), instead of a pageable vector + a synchronous copy.
struct Stager {
    hipStream_t s = nullptr;
    void *buf[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int cur = 0;

    bool init() {
        return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
               hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) == hipSuccess;
    }
    // a staging buffer of >= bytes whose previous copy has finished
    uint8_t *acquire(size_t bytes) {
        const int i = cur;
        if (used[i] && hipEventSynchronize(ev[i]) != hipSuccess) return nullptr;
        if (cap[i] < bytes) {
            if (buf[i]) hipHostFree(buf[i]);
            buf[i] = nullptr, cap[i] = 0;
            const size_t want = std::max(bytes, (size_t)64 << 20);
            if (hipHostMalloc(&buf[i], want, hipHostMallocDefault) != hipSuccess) return nullptr;
            cap[i] = want;
        }
        return (uint8_t *)buf[i];
    }
    bool submit(void *dst, size_t bytes) {
        const int i = cur;
        cur ^= 1;
        used[i] = true;
        return hipMemcpyAsync(dst, buf[i], bytes, hipMemcpyHostToDevice, s) == hipSuccess &&
               hipEventRecord(ev[i], s) == hipSuccess;
    }
    bool finish() { return !s || hipStreamSynchronize(s) == hipSuccess; }
    ~Stager() {
        finish();
        for (int i = 0; i < 2; ++i) {
            if (buf[i]) hipHostFree(buf[i]);
            if (ev[i]) hipEventDestroy(ev[i]);
        }
        if (s) hipStreamDestroy(s);
    }
};

void stager_free(Stager *s) { delete s; }

namespace {

template <class T>
T *dalloc(mio_hip_llm *m, size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) return nullptr;
    m->allocs.push_back(p);
    // zero-filled on the null stream and waited for here: the weight upload that follows
    // runs on the stager's non-blocking stream, which does not order itself after it
    if (hipMemset(p, 0, n * sizeof(T) + 16) != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess)
        return nullptr;
    return (T *)p;
}

bool upload_qmat(mio_hip_llm *m, const mio::GgufTensor *t, mio::QMat &q) {
    if (!t || t->n_dims != 2) {
        mio::set_error("llm: matrix tensor %s missing or not 2-D", t ? t->name.c_str() : "?");
        return false;
    }
    const bool repack = mio::repacks_to_q8_0(t->type);
    if (t->type != mio::GGML_Q8_0 && t->type != mio::GGML_Q4_K && t->type != mio::GGML_Q6_K &&
        t->type != mio::GGML_BF16 && !repack) {
        mio::set_error("llm: tensor %s has type %s; supported: bf16, q8_0, q4_K, q6_K, q5_0 / q4_0 (run as q8_0)",
                       t->name.c_str(), mio::ggml_type_name(t->type));
        return false;
    }
    if (t->type == mio::GGML_BF16 && t->ne[0] % 32) {
        mio::set_error("llm: bf16 tensor %s: row length %lld is not a multiple of 32", t->name.c_str(),
                       (long long)t->ne[0]);
        return false;
    }
    // Q5_0 (llama-quantize's Q4_K fallback for rows not a multiple of 256) and Q4_0 rows run as
    // the Q8_0 rows they equal exactly (quant.h repack_to_q8_0)
    const uint32_t type = repack ? (uint32_t)mio::GGML_Q8_0 : t->type;
    std::vector<uint8_t> q80;
    const void *src = t->data;
    if (repack) {
        q80.resize((size_t)t->ne[1] * (size_t)(t->ne[0] / 32) * sizeof(mio::BlockQ8_0));
        if (!mio::repack_to_q8_0(t->type, t->data, t->ne[1], t->ne[0], q80.data())) {
            mio::set_error("llm: repacking %s (%s) as q8_0 failed", t->name.c_str(), mio::ggml_type_name(t->type));
            return false;
        }
        src = q80.data();
    }
    const mio::SplitLayout L = mio::split_layout(type, t->ne[1], t->ne[0]);
    const auto it = m->arena_off.find(t->name);
    uint8_t *dp = (m->arena && it != m->arena_off.end()) ? m->arena + it->second : dalloc<uint8_t>(m, L.bytes);
    uint8_t *host = dp && m->stager ? m->stager->acquire(L.bytes) : nullptr;
    if (!host) {
        mio::set_error("llm: staging / device buffer for %s failed", t->name.c_str());
        return false;
    }
    if (!mio::to_split(type, src, t->ne[1], t->ne[0], host)) {
        mio::set_error("llm: re-layout of %s failed", t->name.c_str());
        return false;
    }
    if (!m->stager->submit(dp, L.bytes)) {
        mio::set_error("llm: upload of %s failed", t->name.c_str());
        return false;
    }
    q.type = (int)type;
    if (type == mio::GGML_BF16)
        m->bf16 = true;
    else
        m->int8 = true;
    q.rows = (int)t->ne[1];
    q.k = (int)t->ne[0];
    q.p0 = dp + L.off[0];
    q.p1 = dp + L.off[1];
    q.p2 = dp + L.off[2];
    q.p3 = dp + L.off[3];
    m->weight_bytes += t->nbytes;
    return true;
}

float *upload_f32(mio_hip_llm *m, const mio::GgufFile &g, const std::string &name, int64_t n) {
    const mio::GgufTensor *t = g.tensor(name);
    if (!t || t->type != mio::GGML_F32 || t->nelements() != n) {
        mio::set_error("llm: norm tensor %s missing or not f32[%lld]", name.c_str(), (long long)n);
        return nullptr;
    }
    const auto it = m->arena_off.find(t->name);
    float *p = (m->arena && it != m->arena_off.end()) ? (float *)(m->arena + it->second) : dalloc<float>(m, n);
    if (p) hipMemcpy(p, t->data, n * 4, hipMemcpyHostToDevice);
    m->weight_bytes += n * 4;
    return p;
}

// steps per replayed step graph (MIO_GRAPH_STEPS, 1..64; A/B knob, default 8)
int graph_steps() {
    static const int n = [] {
        const char *e = getenv("MIO_GRAPH_STEPS");
        const int v = e && *e ? atoi(e) : 8;
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    return n;
}

// Launches of layer il in step order (launch_step_kernel's `which`): attn_in, attention,
// attn_out, or an lfm2 short-conv layer's conv_in, conv_out; then ffn_in, ffn_down. Returns
// the count (<= 5).
// MIO_ATT_FUSE_O (default 1): attention + O as one launch (k_att_o, which = 10) where the head
// shape has it; 0 keeps the two launches (A/B).
bool fuse_att_o(const mio_hip_llm *m) {
    static const bool env = [] {
        const char *e = getenv("MIO_ATT_FUSE_O");
        return !(e && *e == '0');
    }();
    return env && m->dims.n_kv <= mio::kRdyOff && mio::att_o_supported(m->dims.hd, m->dims.n_head / m->dims.n_kv);
}

// k_att_o's bounded wait (wait_count) raises att_cnt[kRdyFlag] if a merge signal never came:
// reported as an error instead of silently using stale attention outputs.
bool fuse_ffn(const mio_hip_llm *m, int il);
int check_handoff(mio_hip_llm *m) {
    bool any = fuse_att_o(m);
    for (int il = 0; il < m->n_layer && !any; ++il) any = fuse_ffn(m, il);
    if (!any) return MIO_OK;
    int flag = 0;
    // the plain counters' flag and the two k_layer counter sets' (each set has its own)
    int *f[3] = {m->buf.att_cnt + mio::kRdyFlag, m->buf.att_cnt + mio::kLayOff + mio::kRdyFlag,
                 m->buf.att_cnt + mio::kLayOff + mio::kLaySet + mio::kRdyFlag};
    int fl[3] = {0, 0, 0};
    for (int i = 0; i < 3; ++i)
        MIO_HIP_CHECK(hipMemcpyAsync(&fl[i], f[i], sizeof(int), hipMemcpyDeviceToHost, m->d->stream));
    MIO_HIP_CHECK(hipStreamSynchronize(m->d->stream));
    flag = fl[0] | fl[1] | fl[2];
    if (flag) {
        for (int i = 0; i < 3; ++i) MIO_HIP_CHECK(hipMemsetAsync(f[i], 0, sizeof(int), m->d->stream));
        mio::set_error("llm decode: an in-launch hand-off wait (attention -> O, or gate|up -> down) timed out");
        return MIO_ERR_HIP;
    }
    return MIO_OK;
}

// MIO_LAYER_ATT (default 1): layers >= 1 run their whole attention block as one launch
// (k_layer_att, which = 11) where it is instantiated; 0 keeps attn_in + the k_att_o launch.
// MIO_LAYER_ATT: unset = measured policy, "0" = never, "1" = wherever instantiated. The policy
// leaves the hd 64 / 3-query-head shape (0.1B) on attn_in + k_att_o: its q|k|v hand-off inside
// the launch costs more than the boundary it removes (C2 93.0x fused vs 97.5x, and 86.8-89.1x
// vs 97.4x with 4 polls in flight; 1.7B Q4_K_M 54.27x vs 53.8x, 2.6B 35.43x vs 35.16x, 1.7B BF16
// even: profiles/r05_layer_att_policy.txt).
bool fuse_layer_att(const mio_hip_llm *m, int il) {
    static const int env = [] {
        const char *e = getenv("MIO_LAYER_ATT");
        return e && *e == '0' ? 0 : (e && *e == '1' ? 1 : -1);
    }();
    if (env == 0 || il == 0 || !fuse_att_o(m) || !mio::layer_att_supported(m->dims, m->layers[il])) return false;
    const mio::LlmDims &d = m->dims;
    return env == 1 || !(d.hd == 64 && d.n_head == 3 * d.n_kv);
}

// MIO_FFN_FUSE (default 1): the FFN pair of a layer as one launch (k_ffn, which = 12) where it
// is instantiated (ffn_fused_supported); 0 keeps k_ffn_in + k_ffn_down (A/B).
bool fuse_ffn(const mio_hip_llm *m, int il) {
    static const bool env = !(getenv("MIO_FFN_FUSE") && getenv("MIO_FFN_FUSE")[0] == '0');
    return env && mio::ffn_fused_supported(m->dims, m->layers[il]);
}

// MIO_LAYER_FUSE (default 0, A/B): 1 = a layer whose attention block runs as k_layer_att and
// whose FFN pair runs as k_ffn runs both as ONE launch (k_layer, which = 13) where that is
// instantiated (layer_fused_supported). Bit-identical, but slower on the box (r06, 1.7B Q4_K_M:
// 0.800-0.812 vs 0.726-0.729 ms per token, profiles/r06/layer_fuse_ab.txt): the in-launch x and
// h hand-offs cost what the boundaries did, and the FFN weight burst slows the attention chain.
bool fuse_layer(const mio_hip_llm *m, int il) {
    static const bool env = getenv("MIO_LAYER_FUSE") && getenv("MIO_LAYER_FUSE")[0] == '1';
    return env && fuse_layer_att(m, il) && fuse_ffn(m, il) && mio::layer_fused_supported(m->dims, m->layers[il]);
}

int layer_kinds(const mio_hip_llm *m, int il, int *w) {
    int n = 0;
    if (!m->layers[il].conv && fuse_layer(m, il)) {
        w[n++] = 13;
        return n;
    }
    if (m->layers[il].conv) {
        w[n++] = 8, w[n++] = 9;
    } else if (fuse_layer_att(m, il)) {
        w[n++] = 11;
    } else if (fuse_att_o(m)) {
        w[n++] = 0, w[n++] = 10;
    } else {
        w[n++] = 0, w[n++] = 1, w[n++] = 2;
    }
    if (fuse_ffn(m, il))
        w[n++] = 12;
    else
        w[n++] = 3, w[n++] = 4;
    return n;
}

// every launch of a step in order: the layers', then lm_head (6)
std::vector<int> step_kinds(const mio_hip_llm *m) {
    std::vector<int> k;
    int w[5];
    for (int il = 0; il < m->n_layer; ++il) k.insert(k.end(), w, w + layer_kinds(m, il, w));
    k.push_back(6);
    return k;
}

// One decode step on m->d->stream (tl: optional step timeline, diagnostic).
int issue_step(mio_hip_llm *m, unsigned long long *tl = nullptr) {
    hipStream_t s = m->d->stream;
    int seq = 0;
    auto bufs = [&]() {
        mio::LlmBuffers b = m->buf;
        if (tl) b.tl = tl, b.seq = seq++;
        return b;
    };
    int w[5];
    for (int il = 0; il < m->n_layer; ++il)
        for (int i = 0, n = layer_kinds(m, il, w); i < n; ++i)
            mio::launch_step_kernel(w[i], m->dims, m->layers.data(), il, m->kc, m->vc, m->out_norm, m->lm, m->tok,
                                    bufs(), s);
    mio::launch_step_kernel(6, m->dims, m->layers.data(), 0, m->kc, m->vc, m->out_norm, m->lm, m->tok, bufs(), s);
    return MIO_OK;
}

// The sampler of the last issued step (the step graph samples each token inside the next
// step's layer-0 attn_in): leaves the state with no pending sample.
int flush_sample(mio_hip_llm *m) {
    mio::launch_step_kernel(7, m->dims, m->layers.data(), 0, m->kc, m->vc, m->out_norm, m->lm, m->tok, m->buf,
                            m->d->stream);
    MIO_HIP_CHECK(hipGetLastError());
    return MIO_OK;
}

int capture_steps(mio_hip_llm *m, int n, hipGraphExec_t *out) {
    hipStream_t s = m->d->stream;
    hipGraph_t g = nullptr;
    MIO_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = MIO_OK;
    for (int i = 0; i < n && !rc; ++i) rc = issue_step(m);
    MIO_HIP_CHECK(hipStreamEndCapture(s, &g));
    if (rc) return rc;
    MIO_HIP_CHECK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    return MIO_OK;
}

int ensure_graph(mio_hip_llm *m) {
    if (m->graph && m->graph_n) return MIO_OK;
    int rc;
    if (!m->graph && (rc = capture_steps(m, 1, &m->graph))) return rc;
    if (!m->graph_n && (rc = capture_steps(m, graph_steps(), &m->graph_n))) return rc;
    return MIO_OK;
}

int put_cfg(mio_hip_llm *m, mio::SampleCfg c) {
    m->cfg = c;
    MIO_HIP_CHECK(hipMemcpyAsync(m->d_cfg, &c, sizeof(c), hipMemcpyHostToDevice, m->d->stream));
    return MIO_OK;
}

int reset_tickets(mio_hip_llm *m);

int set_state(mio_hip_llm *m, int pos, int token, int step = 0) {
    if (int rc = reset_tickets(m)) return rc;
    mio::StepState st{pos, step, token, 0};
    MIO_HIP_CHECK(hipMemcpyAsync(m->buf.st, &st, sizeof(st), hipMemcpyHostToDevice, m->d->stream));
    mio::launch_embed_token(m->dims, m->tok, m->buf, m->d->stream);
    MIO_HIP_CHECK(hipGetLastError());
    return MIO_OK;
}

// Batched prefill of prompt positions [0, n) (tokens already in m->d_prompt): chunks of
// kPrefillB tokens, one weight pass per launch (llm_prefill.hip). MIO_SEQ_PREFILL=1 is not
// handled here (see llm_begin).
int prefill_issue(mio_hip_llm *m, int n) {
    for (int p0 = 0; p0 < n; p0 += mio::kPrefillB) {
        const int nt = n - p0 < mio::kPrefillB ? n - p0 : mio::kPrefillB;
        mio::PrefillBuffers pb = m->pf;
        pb.pos = m->d_iota + p0, pb.pos_stride = 1;  // positions p0 .. p0 + nt - 1
        pb.seq = m->d_iota, pb.seq_stride = 0;       // one sequence: the model's own cache
        pb.seq_kv = 0;
        mio::launch_prefill_chunk(m->dims, m->layers.data(), m->n_layer, m->kc, m->vc, m->tok, pb, p0, nt,
                                  (p0 + nt - 1) / mio::kAttChunk + 1, m->d->stream);
        MIO_HIP_CHECK(hipGetLastError());
    }
    return MIO_OK;
}

// Batched prefill of positions [0, n): every launch reads only device buffers whose addresses
// depend on n alone (prompt tokens in m->d_prompt), so one graph per prompt length replays it.
// The first prefill of a length runs eagerly (its launches set the kernels' LDS attributes
// outside any capture), the second too and is captured, later ones replay the graph. MIO_PREFILL_GRAPH=0 or
// MIO_NO_GRAPH=1 (every launch eager, for kernel tracing): eager.
int prefill(mio_hip_llm *m, int n) {
    static const bool use_graph = !(getenv("MIO_PREFILL_GRAPH") && getenv("MIO_PREFILL_GRAPH")[0] == '0') &&
                                  !(getenv("MIO_NO_GRAPH") && getenv("MIO_NO_GRAPH")[0] == '1');
    if (n <= 0) return MIO_OK;
    const auto it = m->prefill_graphs.find(n);
    if (use_graph && it != m->prefill_graphs.end()) {
        MIO_HIP_CHECK(hipGraphLaunch(it->second, m->d->stream));
        return MIO_OK;
    }
    int rc = prefill_issue(m, n);
    // a length is captured when it comes back (the second prefill of that length): a one-off
    // prompt does not pay for a capture it never replays
    if (rc || !use_graph || m->prefill_graphs.size() >= 16 || m->prefill_seen[n]++ == 0) return rc;
    // capture a second issue for the next utterance of this length; the prefill above already
    // ran eagerly, so a failed capture or instantiation only leaves this length uncached
    hipStream_t s = m->d->stream;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        return MIO_OK;
    }
    const int crc = prefill_issue(m, n);
    const hipError_t ec = hipStreamEndCapture(s, &g);
    const bool ok = crc == MIO_OK && ec == hipSuccess && g &&
                    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
    if (g) hipGraphDestroy(g);
    (void)hipGetLastError();
    if (ok)
        m->prefill_graphs[n] = ge;
    else if (ge)
        hipGraphExecDestroy(ge);
    return MIO_OK;
}

// The attention chunk tickets (attn_merge_last) are zeroed in stream order before every
// prefill, every decode start and every batched generate (the last chunk workgroup of each
// attention launch resets its ticket, so they are 0 here anyway; this keeps an interrupted
// run from carrying a count).
int reset_tickets(mio_hip_llm *m) {
    MIO_HIP_CHECK(hipMemsetAsync(m->buf.att_cnt, 0, (size_t)mio::kAttCntInts * sizeof(int), m->d->stream));
    MIO_HIP_CHECK(hipMemsetAsync(m->pf.att_cnt, 0, (size_t)mio::kPrefillB * m->dims.n_kv * sizeof(int), m->d->stream));
    MIO_HIP_CHECK(hipMemsetAsync(m->pf.qcnt, 0, (size_t)mio::kQcntInts * sizeof(int), m->d->stream));
    return MIO_OK;
}

int upload_prompt(mio_hip_llm *m, const int32_t *prompt, int n) {
    if (int rc = reset_tickets(m)) return rc;
    MIO_HIP_CHECK(hipMemcpyAsync(m->d_prompt, prompt, (size_t)n * 4, hipMemcpyHostToDevice, m->d->stream));
    return MIO_OK;
}

bool sequential_prefill() {
    static const bool seq = getenv("MIO_SEQ_PREFILL") && getenv("MIO_SEQ_PREFILL")[0] == '1';
    return seq;
}

}  // namespace

namespace mio {

namespace {
// Drops every outstanding snapshot (waits for its copies: the host buffers are reused).
int snaps_drain(mio_hip_llm *m) {
    for (; m->snap_n > 0; --m->snap_n, m->snap_head = (m->snap_head + 1) % mio_hip_llm::kSnaps)
        MIO_HIP_CHECK(hipEventSynchronize(m->snaps[m->snap_head].ev));
    return MIO_OK;
}

// Enqueues a snapshot of the state and of the token ring slots the issued steps write.
int snap_push(mio_hip_llm *m) {
    if (m->snap_n == mio_hip_llm::kSnaps) {  // reuse the oldest slot: its copies must be done
        MIO_HIP_CHECK(hipEventSynchronize(m->snaps[m->snap_head].ev));
        m->snap_head = (m->snap_head + 1) % mio_hip_llm::kSnaps;
        --m->snap_n;
    }
    mio_hip_llm::Snap &sn = m->snaps[(m->snap_head + m->snap_n) % mio_hip_llm::kSnaps];
    const int first = m->n_prompt - 1;
    sn.hi = std::min(m->steps_issued, m->max_steps);
    sn.issued = m->steps_issued;
    MIO_HIP_CHECK(hipMemcpyAsync(sn.st, m->buf.st, sizeof(mio::StepState), hipMemcpyDeviceToHost, m->d->stream));
    if (sn.hi > first)
        MIO_HIP_CHECK(hipMemcpyAsync(sn.tok + first, m->d_tokens + first, (size_t)(sn.hi - first) * 4,
                                     hipMemcpyDeviceToHost, m->d->stream));
    MIO_HIP_CHECK(hipEventRecord(sn.ev, m->d->stream));
    ++m->snap_n;
    return MIO_OK;
}
}  // namespace

LlmInfo llm_info(const mio_hip_llm *m) {
    return LlmInfo{m->dims.n_vocab, m->dims.n_embd, m->n_layer, m->dims.n_head, m->dims.n_kv,
                   m->dims.hd, m->dims.n_ff, m->dims.n_ctx};
}

uint64_t llm_step_weight_bytes(const mio_hip_llm *m) { return m->weight_bytes; }

int llm_begin(mio_hip_llm *m, const int32_t *prompt, int n_prompt, int max_new, const SamplingParams &sp) {
    MIO_REQUIRE(m && prompt && n_prompt >= 1 && max_new >= 1, MIO_ERR_INVALID, "llm_begin: bad args");
    MIO_REQUIRE(n_prompt <= m->dims.n_ctx, MIO_ERR_INVALID, "llm_begin: %d prompt tokens exceed n_ctx %d",
                n_prompt, m->dims.n_ctx);
    // the reference decodes until llama_decode fails at a full context and keeps the token
    // sampled last (test-to-speech.cpp:163-187): at most n_ctx - n_prompt + 1 new tokens
    max_new = std::min(max_new, m->dims.n_ctx - n_prompt + 1);
    for (int i = 0; i < n_prompt; ++i)
        MIO_REQUIRE(prompt[i] >= 0 && prompt[i] < m->dims.n_vocab, MIO_ERR_INVALID,
                    "llm_begin: token %d out of vocab", prompt[i]);
    int rc = mio::bind(m->d);
    if (rc || (rc = snaps_drain(m))) return rc;
    std::vector<int> force(m->max_steps, -1);
    for (int j = 0; j + 1 < n_prompt; ++j) force[j] = prompt[j + 1];
    MIO_HIP_CHECK(hipMemcpyAsync(m->d_force, force.data(), force.size() * 4, hipMemcpyHostToDevice, m->d->stream));
    SampleCfg c{};
    c.temp = sp.temperature;
    c.seed_lo = (uint32_t)sp.seed, c.seed_hi = (uint32_t)(sp.seed >> 32);
    c.lo = sp.allow_lo < 0 ? 0 : sp.allow_lo;
    c.hi = (sp.allow_hi < 0 || sp.allow_hi > m->dims.n_vocab) ? m->dims.n_vocab : sp.allow_hi;
    c.eos0 = sp.eos0, c.eos1 = sp.eos1;
    c.force = m->d_force, c.n_force = m->max_steps;
    c.out_tokens = m->d_tokens, c.max_steps = m->max_steps;
    __atomic_store_n(m->host_done, 0, __ATOMIC_SEQ_CST);  // the cfg copy below is stream-ordered behind it
    c.host_done = m->host_done_dev;
    if ((rc = put_cfg(m, c)) || (rc = ensure_graph(m))) return rc;
    m->n_prompt = n_prompt;
    m->max_new = max_new;
    m->steps_total = n_prompt - 1 + max_new;
    // prompt positions [0, P) are prefilled here: batched (one weight pass per chunk of
    // kPrefillB tokens), or, with MIO_SEQ_PREFILL=1, as P forced decode steps; decoding
    // then starts at position P with the step counter at P either way (same sampler stream)
    const int P = n_prompt - 1;
    if (sequential_prefill() || !m->bf16_mt()) {
        m->steps_issued = 0;
        if ((rc = set_state(m, 0, prompt[0]))) return rc;
        return llm_run(m, P);
    }
    if ((rc = upload_prompt(m, prompt, n_prompt)) || (rc = prefill(m, P))) return rc;
    m->steps_issued = P;
    return set_state(m, P, prompt[P], P);
}

int llm_run(mio_hip_llm *m, int n_steps) {
    int rc = mio::bind(m->d);
    if (rc) return rc;
    // MIO_NO_GRAPH=1: eager launches (rocprofv3 kernel tracing of graph replays crashes on
    // ROCm 7.2 here; kernels and arguments are identical either way)
    static const bool eager = getenv("MIO_NO_GRAPH") && getenv("MIO_NO_GRAPH")[0] == '1';
    int n = std::min(n_steps, m->steps_total - m->steps_issued);
    m->steps_issued += n > 0 ? n : 0;
    if (eager) {
        for (int i = 0; i < n; ++i)
            if ((rc = issue_step(m))) return rc;
    } else {
        for (const int gs = graph_steps(); n >= gs; n -= gs) MIO_HIP_CHECK(hipGraphLaunch(m->graph_n, m->d->stream));
        for (; n > 0; --n) MIO_HIP_CHECK(hipGraphLaunch(m->graph, m->d->stream));
    }
    if ((rc = flush_sample(m))) return rc;
    return snap_push(m);
}

int llm_graph_steps() { return graph_steps(); }

// Steps until the end: graphs of graph_steps() steps, at most kRunDepth queued ahead of the GPU
// (the host waits for the event of the graph kRunDepth back, while the next one still runs),
// and none issued once the sampler has stored the end token's host word. After an end token the
// rest of its graph and at most kRunDepth - 1 more run (returning at entry), instead of the
// rest of a 32-step poll interval and one more interval. Then the flush sampler + a snapshot
// (llm_poll collects the tokens).
int llm_run_to_end(mio_hip_llm *m) {
    constexpr int kRunDepth = 2;
    int rc = mio::bind(m->d);
    if (rc) return rc;
    static const bool eager = getenv("MIO_NO_GRAPH") && getenv("MIO_NO_GRAPH")[0] == '1';
    const int gs = graph_steps();
    m->run_base = m->steps_issued;
    int k = 0;
    while (m->steps_issued < m->steps_total) {
        if (k >= kRunDepth) MIO_HIP_CHECK(hipEventSynchronize(m->run_ev[k - kRunDepth]));
        if (__atomic_load_n(m->host_done, __ATOMIC_ACQUIRE)) break;
        const int n = std::min(gs, m->steps_total - m->steps_issued);
        if (eager) {
            for (int i = 0; i < n; ++i)
                if ((rc = issue_step(m))) return rc;
        } else if (n == gs) {
            MIO_HIP_CHECK(hipGraphLaunch(m->graph_n, m->d->stream));
        } else {
            for (int i = 0; i < n; ++i) MIO_HIP_CHECK(hipGraphLaunch(m->graph, m->d->stream));
        }
        m->steps_issued += n;
        if ((int)m->run_ev.size() <= k) {
            hipEvent_t e = nullptr;
            MIO_HIP_CHECK(hipEventCreate(&e));
            m->run_ev.push_back(e);
        }
        MIO_HIP_CHECK(hipEventRecord(m->run_ev[k], m->d->stream));
        ++k;
    }
    m->run_graphs = k;
    if ((rc = flush_sample(m))) return rc;
    return snap_push(m);
}

int llm_poll(mio_hip_llm *m, std::vector<int32_t> &out, bool *done) {
    int rc = mio::bind(m->d);
    if (rc) return rc;
    if (m->snap_n == 0 && (rc = snap_push(m))) return rc;
    // the oldest outstanding snapshot: steps enqueued after it keep the GPU busy meanwhile
    const int slot = m->snap_head;
    const mio_hip_llm::Snap &sn = m->snaps[slot];
    MIO_HIP_CHECK(hipEventSynchronize(sn.ev));
    m->snap_head = (m->snap_head + 1) % mio_hip_llm::kSnaps;
    --m->snap_n;
    const int first = m->n_prompt - 1;
    const StepState st = *sn.st;
    const int n = std::min(st.step, sn.hi) > first ? std::min(st.step, sn.hi) - first : 0;
    out.assign(sn.tok + first, sn.tok + first + n);
    bool d = false;
    for (int i = 0; i < n; ++i)
        if (out[i] == m->cfg.eos0 || out[i] == m->cfg.eos1) {
            out.resize(i);  // the reference stops before appending the end token (:168-170)
            d = true;
            m->eos_snap = slot;
            break;
        }
    if (done) *done = d || sn.issued >= m->steps_total;
    return MIO_OK;
}

}  // namespace mio

extern "C" int mio_hip_llm_load(mio_hip_device *d, const char *path, int n_ctx, mio_hip_llm **out) {
    MIO_REQUIRE(d && path && out, MIO_ERR_INVALID, "llm_load: null argument");
    if (n_ctx <= 0) n_ctx = 2048;  // test-to-speech.cpp:104
    int rc = mio::bind(d);
    if (rc) return rc;
    const auto t_load0 = std::chrono::steady_clock::now();
    mio::GgufFile g;
    if (!g.open(path)) return MIO_ERR_IO;
    const std::string arch = g.get_str("general.architecture");
    // lfm2 (LiquidAI LFM2, the <|startoftext|><|im_start|> template family): attention layers
    // (NEOX RoPE, q/k RMSNorm) interleaved with gated short-conv layers (llama.cpp build_lfm2)
    const bool lfm2 = arch == "lfm2";
    MIO_REQUIRE(arch == "llama" || arch == "qwen3" || arch == "qwen2" || arch == "mistral" || lfm2,
                MIO_ERR_UNSUPPORTED, "llm_load: architecture '%s' not supported (llama, mistral, qwen2, qwen3, lfm2)",
                arch.c_str());
    // the only bias tensors any supported block has are qwen2's attn_{q,k,v}.bias: anything
    // else (output / ffn biases) would be silently dropped, so refuse the file instead
    for (const mio::GgufTensor &t : g.tensors()) {
        const std::string &n = t.name;
        if (n.size() > 5 && n.compare(n.size() - 5, 5, ".bias") == 0 &&
            !(n.find(".attn_q.bias") != std::string::npos || n.find(".attn_k.bias") != std::string::npos ||
              n.find(".attn_v.bias") != std::string::npos)) {
            mio::set_error("llm_load: bias tensor %s is not supported (only attn_{q,k,v}.bias)", n.c_str());
            return MIO_ERR_UNSUPPORTED;
        }
    }
    auto *m = new mio_hip_llm();
    m->d = d;
    m->stager = new Stager();
    if (!m->stager->init()) {
        delete m;
        mio::set_error("llm_load: staging stream failed");
        return MIO_ERR_HIP;
    }
    auto fail = [&](int code) {
        delete m;
        return code;
    };
    mio::LlmDims &D = m->dims;
    D.n_embd = (int)g.get_int(arch + ".embedding_length", 0);
    m->n_layer = (int)g.get_int(arch + ".block_count", 0);
    D.n_ff = (int)g.get_int(arch + ".feed_forward_length", 0);
    D.n_head = (int)g.get_int(arch + ".attention.head_count", 0);
    // head_count_kv: a scalar, or per layer (lfm2: 0 marks a short-conv layer)
    std::vector<int64_t> kv_arr;
    if (const mio::GgufValue *hv = g.get(arch + ".attention.head_count_kv"); hv && !hv->arr_i.empty()) {
        kv_arr = hv->arr_i;
        D.n_kv = 0;
        for (int64_t v : kv_arr) D.n_kv = std::max(D.n_kv, (int)v);
    } else {
        D.n_kv = (int)g.get_int(arch + ".attention.head_count_kv", D.n_head);
    }
    D.hd = (int)g.get_int(arch + ".attention.key_length", D.n_head ? D.n_embd / D.n_head : 0);
    D.eps = (float)g.get_float(arch + ".attention.layer_norm_rms_epsilon", 1e-6);
    const float base = (float)g.get_float(arch + ".rope.freq_base", 10000.0);
    D.neox = (arch == "qwen3" || arch == "qwen2" || lfm2) ? 1 : 0;
    D.qk_norm = (arch == "qwen3" || lfm2) ? 1 : 0;
    MIO_REQUIRE(!lfm2 || g.get_int(arch + ".shortconv.l_cache", mio::kConvL) == mio::kConvL, MIO_ERR_UNSUPPORTED,
                "llm_load: lfm2 shortconv.l_cache %lld not supported (%d)",
                (long long)g.get_int(arch + ".shortconv.l_cache", 0), mio::kConvL);
    D.n_ctx = n_ctx;
    D.scale = 1.0f / sqrtf((float)D.hd);
    D.split = mio::kAttChunk;
    D.max_splits = (n_ctx + D.split - 1) / D.split;
    // matvec workgroups: one per CU (MIO_WGM=2..4 launches that many per CU, for A/B)
    {
        const char *e = getenv("MIO_WGM");
        const int wgm = e ? std::max(1, std::min(4, atoi(e))) : 1;
        D.n_wg = (d->n_cu > 0 ? d->n_cu : 256) * wgm;
    }
    D.n_layer = m->n_layer;
    MIO_REQUIRE(n_ctx <= 32768, MIO_ERR_UNSUPPORTED, "llm_load: n_ctx %d > 32768", n_ctx);
    const int G = D.n_kv ? D.n_head / D.n_kv : 0;
    if (D.n_embd <= 0 || m->n_layer <= 0 || D.n_head <= 0 || D.n_kv <= 0 || D.n_head % D.n_kv ||
        !(G == 1 || G == 2 || G == 3 || G == 4 || G == 8) || !(D.hd == 64 || D.hd == 128) ||
        (D.n_embd % 256 != 0 && D.n_embd % 32 != 0)) {
        mio::set_error("llm_load: unsupported dims (n_embd %d, heads %d/%d, head_dim %d)", D.n_embd, D.n_head,
                       D.n_kv, D.hd);
        return fail(MIO_ERR_UNSUPPORTED);
    }
    {
        // arena: layer matrices in step order, then the lm_head, then the embedding table
        std::vector<std::string> order;
        static const char *mats[] = {"attn_q",   "attn_k",  "attn_v",   "shortconv.in_proj", "attn_output",
                                     "shortconv.out_proj", "ffn_gate", "ffn_up", "ffn_down"};
        for (int i = 0; i < m->n_layer; ++i)
            for (const char *n : mats) order.push_back("blk." + std::to_string(i) + "." + n + ".weight");
        order.push_back("output.weight");
        order.push_back("token_embd.weight");
        // then every f32 norm vector (kept out of many small allocations: one large mapping
        // serves all of them)
        static const char *norms[] = {"attn_norm", "ffn_norm", "attn_q_norm", "attn_k_norm", "shortconv.conv"};
        for (int i = 0; i < m->n_layer; ++i)
            for (const char *n : norms) order.push_back("blk." + std::to_string(i) + "." + n + ".weight");
        order.push_back("output_norm.weight");
        order.push_back("token_embd_norm.weight");
        size_t total = 0;
        for (const std::string &n : order) {
            const mio::GgufTensor *t = g.tensor(n);
            if (!t) continue;
            size_t bytes = 0;
            if (t->n_dims == 2 && t->type != mio::GGML_F32) {
                const uint32_t ty = mio::repacks_to_q8_0(t->type) ? (uint32_t)mio::GGML_Q8_0 : t->type;
                bytes = mio::split_layout(ty, t->ne[1], t->ne[0]).bytes;
            } else if (t->type == mio::GGML_F32) {
                bytes = (size_t)t->nelements() * 4;
            }
            if (!bytes) continue;
            m->arena_off[n] = total;
            total += (bytes + 255) & ~(size_t)255;
        }
        m->arena = dalloc<uint8_t>(m, total);
        if (!m->arena) {
            mio::set_error("llm_load: weight arena of %zu bytes: allocation failed", total);
            return fail(MIO_ERR_OOM);
        }
    }
    const mio::GgufTensor *te = g.tensor("token_embd.weight");
    if (!te || te->ne[0] != D.n_embd) {
        mio::set_error("llm_load: token_embd.weight missing");
        return fail(MIO_ERR_FORMAT);
    }
    D.n_vocab = (int)te->ne[1];
    MIO_REQUIRE(D.n_vocab <= 128 * 8 * D.n_wg, MIO_ERR_UNSUPPORTED, "llm_load: vocab %d > %d", D.n_vocab,
                128 * 8 * D.n_wg);
    if (!upload_qmat(m, te, m->tok)) return fail(MIO_ERR_FORMAT);
    const uint64_t embd_bytes = te->nbytes;
    m->weight_bytes -= embd_bytes;  // one embedding row per step, not the whole table
    const mio::GgufTensor *to = g.tensor("output.weight");
    if (to) {
        if (!upload_qmat(m, to, m->lm)) return fail(MIO_ERR_FORMAT);
    } else {
        m->lm = m->tok;  // tied embeddings: the table is streamed as the lm_head every step
        m->weight_bytes += embd_bytes;
    }
    // lfm2's final norm is token_embd_norm (llama.cpp model.tok_norm)
    if (!(m->out_norm = upload_f32(m, g, lfm2 ? "token_embd_norm.weight" : "output_norm.weight", D.n_embd)))
        return fail(MIO_ERR_FORMAT);
    bool any_conv = false;
    auto fam = [](int t) { return t == mio::GGML_Q8_0 ? 0 : (t == mio::GGML_BF16 ? 2 : 1); };
    for (int i = 0; i < m->n_layer; ++i) {
        const std::string p = "blk." + std::to_string(i) + ".";
        mio::LayerW L{};
        if (!(L.attn_norm = upload_f32(m, g, p + "attn_norm.weight", D.n_embd)) ||
            !(L.ffn_norm = upload_f32(m, g, p + "ffn_norm.weight", D.n_embd)))
            return fail(MIO_ERR_FORMAT);
        L.conv = g.tensor(p + "shortconv.in_proj.weight") ? 1 : 0;
        if (lfm2 && (size_t)i < kv_arr.size() && (kv_arr[i] == 0) != (L.conv != 0)) {
            mio::set_error("llm_load: layer %d: head_count_kv %lld disagrees with its tensors", i, (long long)kv_arr[i]);
            return fail(MIO_ERR_FORMAT);
        }
        if (L.conv) {
            // gated short conv: in_proj [3 n_embd][n_embd], taps [n_embd][3] f32, out_proj
            MIO_REQUIRE(lfm2, MIO_ERR_UNSUPPORTED, "llm_load: layer %d: short-conv tensors in a '%s' model", i,
                        arch.c_str());
            const mio::GgufTensor *tc = g.tensor(p + "shortconv.conv.weight");
            if (!tc || tc->type != mio::GGML_F32 || tc->ne[0] != mio::kConvL || tc->ne[1] != D.n_embd) {
                mio::set_error("llm_load: layer %d: shortconv.conv.weight must be f32 [%d][%d]", i, D.n_embd,
                               mio::kConvL);
                return fail(MIO_ERR_FORMAT);
            }
            if (!(L.conv_w = upload_f32(m, g, p + "shortconv.conv.weight", (int64_t)D.n_embd * mio::kConvL)) ||
                !upload_qmat(m, g.tensor(p + "shortconv.in_proj.weight"), L.in_proj) ||
                !upload_qmat(m, g.tensor(p + "shortconv.out_proj.weight"), L.out_proj) ||
                !upload_qmat(m, g.tensor(p + "ffn_gate.weight"), L.gate) ||
                !upload_qmat(m, g.tensor(p + "ffn_up.weight"), L.up) ||
                !upload_qmat(m, g.tensor(p + "ffn_down.weight"), L.down))
                return fail(MIO_ERR_FORMAT);
            if (L.in_proj.rows != 3 * D.n_embd || L.in_proj.k != D.n_embd || L.out_proj.rows != D.n_embd ||
                L.out_proj.k != D.n_embd || L.gate.rows != D.n_ff || L.down.k != D.n_ff ||
                L.gate.type != L.up.type || D.n_ff > 12288 || D.n_embd > 64 * 8 * D.n_wg) {
                mio::set_error("llm_load: layer %d (short conv) shapes / quant families not supported", i);
                return fail(MIO_ERR_UNSUPPORTED);
            }
            any_conv = true;
            m->has_conv = true;
            m->layers.push_back(L);
            continue;
        }
        if (D.qk_norm) {
            if (!(L.q_norm = upload_f32(m, g, p + "attn_q_norm.weight", D.hd)) ||
                !(L.k_norm = upload_f32(m, g, p + "attn_k_norm.weight", D.hd)))
                return fail(MIO_ERR_FORMAT);
        }
        if (!upload_qmat(m, g.tensor(p + "attn_q.weight"), L.wq) || !upload_qmat(m, g.tensor(p + "attn_k.weight"), L.wk) ||
            !upload_qmat(m, g.tensor(p + "attn_v.weight"), L.wv) ||
            !upload_qmat(m, g.tensor(p + "attn_output.weight"), L.wo) ||
            !upload_qmat(m, g.tensor(p + "ffn_gate.weight"), L.gate) ||
            !upload_qmat(m, g.tensor(p + "ffn_up.weight"), L.up) || !upload_qmat(m, g.tensor(p + "ffn_down.weight"), L.down))
            return fail(MIO_ERR_FORMAT);
        {
            // qwen2 q/k/v projection biases, one f32 vector in qkv order (added before
            // RoPE by the attention kernels' head preparation)
            const mio::GgufTensor *bt[3] = {g.tensor(p + "attn_q.bias"), g.tensor(p + "attn_k.bias"),
                                            g.tensor(p + "attn_v.bias")};
            const int64_t bn[3] = {(int64_t)D.n_head * D.hd, (int64_t)D.n_kv * D.hd, (int64_t)D.n_kv * D.hd};
            if (bt[0] || bt[1] || bt[2]) {
                std::vector<float> hb;
                for (int j = 0; j < 3; ++j) {
                    if (!bt[j] || bt[j]->type != mio::GGML_F32 || bt[j]->nelements() != bn[j]) {
                        mio::set_error("llm_load: layer %d: attn_q/k/v.bias must all be f32 of the projection sizes", i);
                        return fail(MIO_ERR_FORMAT);
                    }
                    const float *f = (const float *)bt[j]->data;
                    hb.insert(hb.end(), f, f + bn[j]);
                }
                float *db = dalloc<float>(m, hb.size());
                if (!db || hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
                    mio::set_error("llm_load: bias upload failed");
                    return fail(MIO_ERR_OOM);
                }
                L.bqkv = db;
                m->weight_bytes += hb.size() * 4;
            }
        }
        if (L.wq.rows != D.n_head * D.hd || L.wk.rows != D.n_kv * D.hd || L.wv.rows != D.n_kv * D.hd ||
            L.gate.rows != D.n_ff || L.down.k != D.n_ff || fam(L.wq.type) != fam(L.wk.type) ||
            fam(L.wq.type) != fam(L.wv.type) || L.wq.type != L.wk.type || L.gate.type != L.up.type ||
            D.n_ff > 12288 ||
            D.n_embd > 64 * 8 * D.n_wg) {
            mio::set_error("llm_load: layer %d shapes / quant families not supported", i);
            return fail(MIO_ERR_UNSUPPORTED);
        }
        m->layers.push_back(L);
    }
    // buffers
    const int qkv = (D.n_head + 2 * D.n_kv) * D.hd;
    // q|k|v rows, or an lfm2 short-conv layer's B | C | X rows
    const int qkv_rows = std::max(qkv, any_conv ? 3 * D.n_embd : 0);
    const size_t kv = (size_t)m->n_layer * D.n_kv * n_ctx * D.hd;
    m->kc = dalloc<_Float16>(m, kv);
    m->vc = dalloc<_Float16>(m, kv);
    // every per-step buffer (activations, partials, state, token rings, RoPE table, prefill
    // staging) is carved from ONE allocation: one large mapping instead of many small ones
    // (the activation vectors are read by every CU at the start of every launch)
    std::vector<std::pair<void **, size_t>> carve;
    auto want = [&](auto *&ptr, size_t count) {
        carve.push_back({reinterpret_cast<void **>(&ptr), count * sizeof(*ptr)});
    };
    float2 *dr = nullptr;
    want(m->buf.x, D.n_embd);
    want(m->buf.qkv, qkv_rows);
    if (any_conv) want(m->buf.ring, (size_t)m->n_layer * mio::kConvSlots * D.n_embd);
    want(m->buf.h, D.n_ff);
    want(m->buf.logits, D.n_vocab);
    want(m->buf.part, (size_t)D.n_head * D.max_splits * (D.hd + 4));
    want(m->buf.att, (size_t)D.n_head * D.hd);
    want(m->buf.att_cnt, (size_t)mio::kAttCntInts);  // + k_att_o's merge counters and timeout flag
    want(m->buf.smp, 2 * std::max(mio::lm_head_blocks(D), 4 * D.n_wg) + 16);
    want(m->buf.st, 1);
    want(m->d_cfg, 1);
    m->max_steps = n_ctx;
    for (mio_hip_llm::Snap &sn : m->snaps)
        if (hipHostMalloc((void **)&sn.st, sizeof(mio::StepState), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&sn.tok, (size_t)m->max_steps * 4, hipHostMallocDefault) != hipSuccess ||
            hipEventCreate(&sn.ev) != hipSuccess) {
            mio::set_error("llm_load: pinned host buffers / events failed");
            return fail(MIO_ERR_OOM);
        }
    if (hipHostMalloc((void **)&m->host_done, 64 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&m->host_done_dev, m->host_done, 0) != hipSuccess) {
        mio::set_error("llm_load: mapped host end-token words failed");
        return fail(MIO_ERR_OOM);
    }
    std::memset(m->host_done, 0, 64 * sizeof(int));
    want(m->d_tokens, m->max_steps);
    want(m->d_force, m->max_steps);
    want(m->d_prompt, n_ctx);
    want(m->pf.x, (size_t)mio::kPrefillB * D.n_embd);
    want(m->pf.qkv, (size_t)mio::kPrefillB * qkv_rows);
    want(m->pf.h, (size_t)mio::kPrefillB * D.n_ff);
    want(m->pf.part, (size_t)mio::kPrefillB * D.n_head * D.max_splits * (D.hd + 4));
    want(m->pf.att, (size_t)mio::kPrefillB * D.n_head * D.hd);
    want(m->pf.att_cnt, (size_t)mio::kPrefillB * D.n_kv);
    want(m->pf.qcnt, (size_t)mio::kQcntInts);  // batched decode in-launch quantization counters
    want(m->pf.act, mio::prefill_act_bytes(
                        mio::prefill_rec_k(std::max(std::max(D.n_embd, D.n_ff), D.n_head * D.hd), m->bf16 ? 30 : 8)));
    want(dr, (size_t)n_ctx * (D.hd / 2));
    want(m->d_iota, (size_t)n_ctx + mio::kPrefillB);
    size_t io_bytes = 0;
    for (auto &c : carve) io_bytes += (c.second + 255) & ~(size_t)255;
    uint8_t *io = dalloc<uint8_t>(m, (io_bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1));
    if (io) {
        size_t off = 0;
        for (auto &c : carve) {
            *c.first = io + off;
            off += (c.second + 255) & ~(size_t)255;
        }
    }
    m->buf.cfg = m->d_cfg;
    m->pf.tokens = m->d_prompt;
    m->pf.ring = m->buf.ring;  // the single-stream prefill is sequence 0 of the decode rings
    m->pf.seq_ring = 0;
    // RoPE table, ggml rope-cache recurrence (theta = p; theta *= base^(-2/hd) per pair)
    std::vector<float2> rope((size_t)n_ctx * (D.hd / 2));
    const float theta_scale = powf(base, -2.0f / D.hd);
    for (int p = 0; p < n_ctx; ++p) {
        float theta = (float)p;
        for (int i = 0; i < D.hd / 2; ++i) {
            rope[(size_t)p * (D.hd / 2) + i] = make_float2(cosf(theta), sinf(theta));
            theta *= theta_scale;
        }
    }
    if (!m->kc || !m->vc || !m->buf.x || !m->buf.qkv || !m->buf.h || !m->buf.logits ||
        !m->buf.part || !m->buf.att || !m->buf.att_cnt || !m->pf.att || !m->pf.att_cnt || !m->pf.qcnt || !m->buf.smp || !m->buf.st || !m->d_cfg || !m->d_tokens || !m->d_force || !dr ||
        !m->d_prompt || !m->pf.x || !m->pf.qkv || !m->pf.h || !m->pf.part || !m->pf.act || !m->d_iota ||
        (any_conv && !m->buf.ring)) {
        mio::set_error("llm_load: device allocation failed");
        return fail(MIO_ERR_OOM);
    }
    hipMemcpy(dr, rope.data(), rope.size() * sizeof(float2), hipMemcpyHostToDevice);
    {
        std::vector<int> iota((size_t)n_ctx + mio::kPrefillB);
        for (size_t i = 0; i < iota.size(); ++i) iota[i] = (int)i;
        hipMemcpy(m->d_iota, iota.data(), iota.size() * 4, hipMemcpyHostToDevice);
    }
    m->buf.rope = dr;
    m->pf.rope = dr;
    // every memset / copy above ran on the null stream or the staging stream; the runner's
    // stream is non-blocking
    if (!m->stager->finish() || hipDeviceSynchronize() != hipSuccess) {
        mio::set_error("llm_load: device synchronize failed");
        return fail(MIO_ERR_HIP);
    }
    delete m->stager;
    m->stager = nullptr;
    // the decode-step graphs are captured here, as llama_init_from_model reserves its compute
    // graphs at context creation: the first generate replays them instead of capturing
    if ((rc = ensure_graph(m))) return fail(rc);
    m->load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_load0).count();
    *out = m;
    return MIO_OK;
}

extern "C" int mio_hip_llm_step_kinds(const mio_hip_llm *m, int *kinds, int cap, int *n) {
    MIO_REQUIRE(m && n, MIO_ERR_INVALID, "llm_step_kinds: null");
    const std::vector<int> k = step_kinds(m);
    *n = (int)k.size();
    MIO_REQUIRE(!kinds || cap >= (int)k.size(), MIO_ERR_INVALID, "llm_step_kinds: need %d slots", (int)k.size());
    if (kinds) std::memcpy(kinds, k.data(), k.size() * sizeof(int));
    return MIO_OK;
}

// lfm2 short-conv ring of layer il, [kConvSlots][n_embd] (bx of position p in slot p & 3;
// parity tests). get: copied out; set: copied in.
extern "C" int mio_hip_llm_conv_ring(mio_hip_llm *m, int il, float *ring, int set) {
    MIO_REQUIRE(m && ring && il >= 0 && il < m->n_layer && m->layers[il].conv && m->buf.ring, MIO_ERR_INVALID,
                "llm_conv_ring: layer %d is not a short-conv layer", il);
    int rc = mio::bind(m->d);
    if (rc) return rc;
    const size_t n = (size_t)mio::kConvSlots * m->dims.n_embd;
    float *dr = m->buf.ring + (size_t)il * n;
    hipStream_t s = m->d->stream;
    if (set)
        MIO_HIP_CHECK(hipMemcpyAsync(dr, ring, n * 4, hipMemcpyHostToDevice, s));
    else
        MIO_HIP_CHECK(hipMemcpyAsync(ring, dr, n * 4, hipMemcpyDeviceToHost, s));
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    return MIO_OK;
}

extern "C" int mio_hip_llm_load_ms(const mio_hip_llm *m, double *ms) {
    MIO_REQUIRE(m && ms, MIO_ERR_INVALID, "llm_load_ms: null");
    *ms = m->load_ms;
    return MIO_OK;
}

extern "C" int mio_hip_llm_steps_issued(const mio_hip_llm *m, int *steps) {
    MIO_REQUIRE(m && steps, MIO_ERR_INVALID, "llm_steps_issued: null");
    *steps = std::max(0, m->steps_issued - (m->n_prompt - 1));
    return MIO_OK;
}

extern "C" void mio_hip_llm_free(mio_hip_llm *m) { delete m; }

extern "C" int mio_hip_llm_info(const mio_hip_llm *m, int *info) {
    MIO_REQUIRE(m && info, MIO_ERR_INVALID, "llm_info: null");
    mio::LlmInfo i = mio::llm_info(m);
    info[0] = i.n_vocab, info[1] = i.n_embd, info[2] = i.n_layer, info[3] = i.n_head;
    info[4] = i.n_kv, info[5] = i.head_dim, info[6] = i.n_ff, info[7] = i.n_ctx;
    return MIO_OK;
}

extern "C" int mio_hip_llm_weight_bytes(const mio_hip_llm *m, uint64_t *bytes) {
    MIO_REQUIRE(m && bytes, MIO_ERR_INVALID, "llm_weight_bytes: null");
    *bytes = m->weight_bytes;
    return MIO_OK;
}

extern "C" int mio_hip_llm_eval(mio_hip_llm *m, int32_t token, int pos, float *logits) {
    MIO_REQUIRE(m && token >= 0 && token < m->dims.n_vocab && pos >= 0 && pos < m->dims.n_ctx,
                MIO_ERR_INVALID, "llm_eval: bad token/pos");
    int rc = mio::bind(m->d);
    if (rc) return rc;
    mio::SampleCfg c{};
    c.temp = 0.0f, c.lo = 0, c.hi = m->dims.n_vocab, c.eos0 = c.eos1 = -1;
    c.force = m->d_force, c.n_force = m->max_steps, c.out_tokens = m->d_tokens, c.max_steps = m->max_steps;
    if ((rc = put_cfg(m, c)) || (rc = ensure_graph(m))) return rc;
    const int zero = 0;
    MIO_HIP_CHECK(hipMemcpyAsync(m->d_force, &zero, 4, hipMemcpyHostToDevice, m->d->stream));
    if ((rc = set_state(m, pos, token))) return rc;
    MIO_HIP_CHECK(hipGraphLaunch(m->graph, m->d->stream));
    if (logits)
        MIO_HIP_CHECK(hipMemcpyAsync(logits, m->buf.logits, (size_t)m->dims.n_vocab * 4, hipMemcpyDeviceToHost,
                                     m->d->stream));
    // the step left its sample pending (k_lm_head): take it, so the state is a settled one
    if ((rc = flush_sample(m))) return rc;
    MIO_HIP_CHECK(hipStreamSynchronize(m->d->stream));
    return check_handoff(m);
}

// One decode step like mio_hip_llm_eval, launched kernel by kernel, with the residual stream
// captured before layer 0 (the embedding) and after every layer: x_layers[(n_layer + 1) *
// n_embd] (parity tests: the oracle re-runs each layer on the GPU's input).
extern "C" int mio_hip_llm_eval_layers(mio_hip_llm *m, int32_t token, int pos, float *x_layers, float *logits) {
    MIO_REQUIRE(m && x_layers && token >= 0 && token < m->dims.n_vocab && pos >= 0 && pos < m->dims.n_ctx,
                MIO_ERR_INVALID, "llm_eval_layers: bad args");
    int rc = mio::bind(m->d);
    if (rc) return rc;
    mio::SampleCfg c{};
    c.temp = 0.0f, c.lo = 0, c.hi = m->dims.n_vocab, c.eos0 = c.eos1 = -1;
    c.force = m->d_force, c.n_force = m->max_steps, c.out_tokens = m->d_tokens, c.max_steps = m->max_steps;
    if ((rc = put_cfg(m, c)) || (rc = ensure_graph(m))) return rc;
    const int zero = 0;
    hipStream_t s = m->d->stream;
    const size_t D = (size_t)m->dims.n_embd;
    MIO_HIP_CHECK(hipMemcpyAsync(m->d_force, &zero, 4, hipMemcpyHostToDevice, s));
    if ((rc = set_state(m, pos, token))) return rc;
    if (!m->d_layers) {
        void *p = nullptr;
        MIO_HIP_CHECK(hipMalloc(&p, (m->n_layer + 1) * D * 4));
        m->allocs.push_back(p);
        m->d_layers = (float *)p;
    }
    float *dx = m->d_layers;
    MIO_HIP_CHECK(hipMemcpyAsync(dx, m->buf.x, D * 4, hipMemcpyDeviceToDevice, s));
    int w[5];
    for (int il = 0; il < m->n_layer; ++il) {
        for (int i = 0, n = layer_kinds(m, il, w); i < n; ++i)
            mio::launch_step_kernel(w[i], m->dims, m->layers.data(), il, m->kc, m->vc, m->out_norm, m->lm, m->tok,
                                    m->buf, s);
        MIO_HIP_CHECK(hipMemcpyAsync(dx + (il + 1) * D, m->buf.x, D * 4, hipMemcpyDeviceToDevice, s));
    }
    mio::launch_step_kernel(6, m->dims, m->layers.data(), 0, m->kc, m->vc, m->out_norm, m->lm, m->tok, m->buf, s);
    MIO_HIP_CHECK(hipGetLastError());
    MIO_HIP_CHECK(hipMemcpyAsync(x_layers, dx, (m->n_layer + 1) * D * 4, hipMemcpyDeviceToHost, s));
    if (logits)
        MIO_HIP_CHECK(hipMemcpyAsync(logits, m->buf.logits, (size_t)m->dims.n_vocab * 4, hipMemcpyDeviceToHost, s));
    if ((rc = flush_sample(m))) return rc;
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    return check_handoff(m);
}

// F16 K / V cache rows [0, n_pos) of layer il as [n_kv][n_pos][head_dim] (parity tests).
extern "C" int mio_hip_llm_kv_rows(mio_hip_llm *m, int il, int n_pos, uint16_t *k, uint16_t *v) {
    MIO_REQUIRE(m && k && v && il >= 0 && il < m->n_layer && n_pos >= 0 && n_pos <= m->dims.n_ctx, MIO_ERR_INVALID,
                "llm_kv_rows: bad args");
    int rc = mio::bind(m->d);
    if (rc) return rc;
    const mio::LlmDims &D = m->dims;
    hipStream_t s = m->d->stream;
    for (int h = 0; h < D.n_kv; ++h) {
        const size_t src = (((size_t)il * D.n_kv + h) * D.n_ctx) * D.hd, dst = (size_t)h * n_pos * D.hd;
        MIO_HIP_CHECK(hipMemcpyAsync(k + dst, m->kc + src, (size_t)n_pos * D.hd * 2, hipMemcpyDeviceToHost, s));
        MIO_HIP_CHECK(hipMemcpyAsync(v + dst, m->vc + src, (size_t)n_pos * D.hd * 2, hipMemcpyDeviceToHost, s));
    }
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    return MIO_OK;
}

extern "C" int mio_hip_llm_tail(const mio_hip_llm *m, int *steps, int *timed_steps, float *timed_ms) {
    MIO_REQUIRE(m && steps && timed_steps && timed_ms, MIO_ERR_INVALID, "llm_tail: null argument");
    *steps = m->tail_steps, *timed_steps = m->tail_timed_steps, *timed_ms = m->tail_ms;
    return MIO_OK;
}

extern "C" int mio_hip_llm_generate(mio_hip_llm *m, const int32_t *prompt, int n_prompt, int max_tokens,
                                    float temperature, uint64_t seed, int32_t allow_lo, int32_t allow_hi,
                                    int32_t eos0, int32_t eos1, int32_t check_interval, int32_t *out_tokens,
                                    int *n_out) {
    MIO_REQUIRE(m && out_tokens && n_out, MIO_ERR_INVALID, "llm_generate: null argument");
    mio::SamplingParams sp;
    sp.temperature = temperature, sp.seed = seed, sp.allow_lo = allow_lo, sp.allow_hi = allow_hi;
    sp.eos0 = eos0, sp.eos1 = eos1;
    int rc = mio::llm_begin(m, prompt, n_prompt, max_tokens, sp);
    if (rc) return rc;
    (void)check_interval;  // the end token reaches the host through its mapped word (r06)
    std::vector<int32_t> toks;
    bool done = false;
    m->eos_snap = -1, m->tail_steps = 0, m->tail_timed_steps = 0, m->tail_ms = 0.0f;
    if ((rc = mio::llm_run_to_end(m))) return rc;
    if ((rc = mio::llm_poll(m, toks, &done))) return rc;
    if (m->eos_snap >= 0) {
        // steps after the end token's: they return at entry (StepState.done). The end token is
        // sampled by step e + 1 (inside its layer-0 launch, or the flush after the last graph);
        // the graphs queued after the one holding that step are timed by their events
        const int e1 = (n_prompt - 1) + (int)toks.size() + 1;
        m->tail_steps = m->steps_issued - e1;
        const int gs = mio::llm_graph_steps();
        const int g = (e1 - 1 - m->run_base) / gs;  // step numbers are 0-based: e1 - 1 is step e + 1
        if (g >= 0 && g + 1 < m->run_graphs) {
            MIO_HIP_CHECK(hipEventSynchronize(m->run_ev[m->run_graphs - 1]));
            MIO_HIP_CHECK(hipEventElapsedTime(&m->tail_ms, m->run_ev[g], m->run_ev[m->run_graphs - 1]));
            m->tail_timed_steps = m->steps_issued - std::min(m->steps_total, m->run_base + (g + 1) * gs);
        }
    }
    if ((rc = check_handoff(m))) return rc;
    const int n = (int)toks.size() < max_tokens ? (int)toks.size() : max_tokens;
    std::memcpy(out_tokens, toks.data(), (size_t)n * 4);
    *n_out = n;
    return MIO_OK;
}

namespace {

size_t batch_seq_ring(const mio_hip_llm *m) { return (size_t)m->n_layer * mio::kConvSlots * m->dims.n_embd; }

// Batch state for B streams (re-allocated when B changes; graphs re-captured).
int batch_ensure(mio_hip_llm *m, int B) {
    auto &bt = m->bt;
    if (bt.B == B) return MIO_OK;
    if (bt.graph) hipGraphExecDestroy(bt.graph), bt.graph = nullptr;
    if (bt.graph_n) hipGraphExecDestroy(bt.graph_n), bt.graph_n = nullptr;
    for (void *p : bt.allocs) hipFree(p);
    bt.allocs.clear();
    bt.B = 0;
    const mio::LlmDims &D = m->dims;
    const size_t seq_kv = (size_t)m->n_layer * D.n_kv * D.n_ctx * D.hd;
    auto al = [&](size_t bytes) -> void * {
        void *p = nullptr;
        if (hipMalloc(&p, bytes + 256) != hipSuccess) return nullptr;
        bt.allocs.push_back(p);
        // stream-ordered: the runner's stream is non-blocking, so a null-stream memset could
        // still be clearing the caches while the prefill below writes them
        hipMemsetAsync(p, 0, bytes + 256, m->d->stream);
        return p;
    };
    bt.kc = (_Float16 *)al((size_t)B * seq_kv * 2);
    bt.vc = (_Float16 *)al((size_t)B * seq_kv * 2);
    bt.st = (mio::StepState *)al((size_t)B * sizeof(mio::StepState));
    bt.cfg = (mio::SampleCfg *)al((size_t)B * sizeof(mio::SampleCfg));
    bt.logits = (float *)al((size_t)B * D.n_vocab * 4);
    bt.smp = (float *)al((size_t)B * mio::lm_head_blocks(D) * 2 * 4);
    bt.tokens = (int *)al((size_t)B * D.n_ctx * 4);
    bt.ppos = (int *)al((size_t)B * D.n_ctx * 4);
    bt.pseq = (int *)al((size_t)B * D.n_ctx * 4);
    bt.ptok = (int *)al((size_t)B * D.n_ctx * 4);
    bt.ring = m->buf.ring ? (float *)al(B * batch_seq_ring(m) * 4) : nullptr;
    if (!bt.kc || !bt.vc || !bt.st || !bt.cfg || !bt.logits || !bt.smp || !bt.tokens || !bt.ppos || !bt.pseq ||
        !bt.ptok || (m->buf.ring && !bt.ring)) {
        for (void *p : bt.allocs) hipFree(p);
        bt.allocs.clear();
        mio::set_error("llm_generate_batch: device allocation for %d streams failed", B);
        return MIO_ERR_OOM;
    }
    bt.B = B;
    MIO_HIP_CHECK(hipStreamSynchronize(m->d->stream));
    return MIO_OK;
}

// the decode step's view of the batch: stream b's position is st[b].pos, its cache is b
mio::PrefillBuffers batch_pb(mio_hip_llm *m) {
    mio::PrefillBuffers pb = m->pf;
    pb.pos = &m->bt.st[0].pos, pb.pos_stride = (int)(sizeof(mio::StepState) / sizeof(int));
    pb.seq = m->d_iota, pb.seq_stride = 1;
    pb.seq_kv = (size_t)m->n_layer * m->dims.n_kv * m->dims.n_ctx * m->dims.hd;
    pb.ring = m->bt.ring, pb.seq_ring = batch_seq_ring(m);
    return pb;
}

mio::BatchBuffers batch_bb(mio_hip_llm *m) { return mio::BatchBuffers{m->bt.st, m->bt.cfg, m->bt.logits, m->bt.smp}; }

void issue_batch_step(mio_hip_llm *m) {
    mio::launch_batch_step(m->dims, m->layers.data(), m->n_layer, m->bt.kc, m->bt.vc, m->out_norm, m->lm, m->tok,
                           batch_pb(m), batch_bb(m), m->bt.B, m->d->stream);
}

int capture_batch(mio_hip_llm *m, int n, hipGraphExec_t *out) {
    hipStream_t s = m->d->stream;
    hipGraph_t g = nullptr;
    MIO_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) issue_batch_step(m);
    MIO_HIP_CHECK(hipStreamEndCapture(s, &g));
    MIO_HIP_CHECK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    return MIO_OK;
}

// n batched steps: the first ever step for this B runs eagerly (its launches set the
// kernels' LDS attributes outside any capture), then 1- and graph_steps()-step graphs replay.
int run_batch(mio_hip_llm *m, int n) {
    static const bool eager = getenv("MIO_NO_GRAPH") && getenv("MIO_NO_GRAPH")[0] == '1';
    auto &bt = m->bt;
    if (n > 0 && (eager || !bt.graph)) {
        issue_batch_step(m);
        MIO_HIP_CHECK(hipGetLastError());
        --n;
        if (eager) {
            for (; n > 0; --n) issue_batch_step(m);
            MIO_HIP_CHECK(hipGetLastError());
            return MIO_OK;
        }
        int rc;
        if ((rc = capture_batch(m, 1, &bt.graph)) || (rc = capture_batch(m, graph_steps(), &bt.graph_n))) return rc;
    }
    for (const int gs = graph_steps(); n >= gs; n -= gs) MIO_HIP_CHECK(hipGraphLaunch(bt.graph_n, m->d->stream));
    for (; n > 0; --n) MIO_HIP_CHECK(hipGraphLaunch(bt.graph, m->d->stream));
    return MIO_OK;
}

}  // namespace

// B independent utterances decoded together (the reference runs them one after another, one
// llama_context each: test-to-speech.cpp:94-199 per call). Prompts are concatenated;
// stream b's sampled tokens go to out_tokens[b * max_tokens ...], n_out[b] of them (up to,
// not including, an end token). Each stream's tokens equal a single-stream generate with
// its seed (same kernels' arithmetic per token, same sampler noise).
extern "C" int mio_hip_llm_generate_batch(mio_hip_llm *m, const int32_t *prompts, const int32_t *prompt_lens, int B,
                                          int max_tokens, float temperature, const uint64_t *seeds,
                                          int32_t allow_lo, int32_t allow_hi, int32_t eos0, int32_t eos1,
                                          int32_t check_interval, int32_t *out_tokens, int32_t *n_out) {
    MIO_REQUIRE(m && prompts && prompt_lens && seeds && out_tokens && n_out && max_tokens >= 1, MIO_ERR_INVALID,
                "llm_generate_batch: bad args");
    MIO_REQUIRE(mio::batch_supported(m->dims, B, m->lm.type), MIO_ERR_UNSUPPORTED,
                "llm_generate_batch: %d streams not supported (1..%d, lm_head LDS)", B, mio::kBatchMax);
    MIO_REQUIRE(m->bf16_mt(), MIO_ERR_UNSUPPORTED,
                "llm_generate_batch: BF16 weights mixed with quantized ones, or in an lfm2 model, run on the "
                "single-stream decode only (mio_hip_llm_generate)");
    const mio::LlmDims &D = m->dims;
    std::vector<int> off(B + 1, 0);
    for (int b = 0; b < B; ++b) {
        MIO_REQUIRE(prompt_lens[b] >= 1 && prompt_lens[b] <= D.n_ctx, MIO_ERR_INVALID,
                    "llm_generate_batch: stream %d: %d prompt tokens exceed n_ctx %d", b, prompt_lens[b], D.n_ctx);
        off[b + 1] = off[b] + prompt_lens[b];
    }
    for (int i = 0; i < off[B]; ++i)
        MIO_REQUIRE(prompts[i] >= 0 && prompts[i] < D.n_vocab, MIO_ERR_INVALID,
                    "llm_generate_batch: token %d out of vocab", prompts[i]);
    int rc = mio::bind(m->d);
    if (rc || (rc = batch_ensure(m, B)) || (rc = reset_tickets(m))) return rc;
    auto &bt = m->bt;
    hipStream_t s = m->d->stream;
    // prompt positions [0, P_b) of every stream: one flattened list, kPrefillB tokens per
    // chunk whatever stream they belong to (one weight pass per chunk)
    std::vector<int> ftok, fpos, fseq;
    for (int b = 0; b < B; ++b)
        for (int p = 0; p + 1 < prompt_lens[b]; ++p) {
            ftok.push_back(prompts[off[b] + p]);
            fpos.push_back(p);
            fseq.push_back(b);
        }
    const int nf = (int)ftok.size();
    if (nf) {
        MIO_HIP_CHECK(hipMemcpyAsync(bt.ptok, ftok.data(), (size_t)nf * 4, hipMemcpyHostToDevice, s));
        MIO_HIP_CHECK(hipMemcpyAsync(bt.ppos, fpos.data(), (size_t)nf * 4, hipMemcpyHostToDevice, s));
        MIO_HIP_CHECK(hipMemcpyAsync(bt.pseq, fseq.data(), (size_t)nf * 4, hipMemcpyHostToDevice, s));
    }
    for (int c0 = 0; c0 < nf; c0 += mio::kPrefillB) {
        const int nt = nf - c0 < mio::kPrefillB ? nf - c0 : mio::kPrefillB;
        int pmax = 0;
        for (int t = 0; t < nt; ++t) pmax = std::max(pmax, fpos[c0 + t]);
        mio::PrefillBuffers pb = m->pf;
        pb.tokens = bt.ptok;
        pb.pos = bt.ppos + c0, pb.pos_stride = 1;
        pb.seq = bt.pseq + c0, pb.seq_stride = 1;
        pb.seq_kv = (size_t)m->n_layer * D.n_kv * D.n_ctx * D.hd;
        pb.ring = bt.ring, pb.seq_ring = batch_seq_ring(m);
        mio::launch_prefill_chunk(D, m->layers.data(), m->n_layer, bt.kc, bt.vc, m->tok, pb, c0, nt,
                                  pmax / mio::kAttChunk + 1, s);
        MIO_HIP_CHECK(hipGetLastError());
    }
    // per-stream state: decoding starts at position P_b = len_b - 1 with the step counter at
    // P_b (the single-stream generate's sampler stream)
    std::vector<mio::StepState> st(B);
    std::vector<mio::SampleCfg> cf(B);
    for (int b = 0; b < B; ++b) {
        const int P = prompt_lens[b] - 1;
        st[b] = mio::StepState{P, P, prompts[off[b] + P], 0};
        mio::SampleCfg &c = cf[b];
        c.temp = temperature;
        c.seed_lo = (uint32_t)seeds[b], c.seed_hi = (uint32_t)(seeds[b] >> 32);
        c.lo = allow_lo < 0 ? 0 : allow_lo;
        c.hi = (allow_hi < 0 || allow_hi > D.n_vocab) ? D.n_vocab : allow_hi;
        c.eos0 = eos0, c.eos1 = eos1;
        c.force = nullptr, c.n_force = 0;
        c.out_tokens = bt.tokens + (size_t)b * D.n_ctx;
        c.host_done = m->host_done_dev + 1 + b;
        __atomic_store_n(m->host_done + 1 + b, 0, __ATOMIC_SEQ_CST);
        // as llm_begin: a full context ends the stream after n_ctx - len + 1 tokens
        c.max_steps = P + std::min(max_tokens, D.n_ctx - prompt_lens[b] + 1);
    }
    MIO_HIP_CHECK(hipMemcpyAsync(bt.st, st.data(), B * sizeof(mio::StepState), hipMemcpyHostToDevice, s));
    MIO_HIP_CHECK(hipMemcpyAsync(bt.cfg, cf.data(), B * sizeof(mio::SampleCfg), hipMemcpyHostToDevice, s));
    mio::launch_batch_embed(D, m->tok, batch_pb(m), batch_bb(m), B, s);
    MIO_HIP_CHECK(hipGetLastError());
    // graphs of graph_steps() steps, at most 2 queued ahead of the GPU; none issued once every
    // stream has stored its end token's host word or spent its step budget (check_interval no
    // longer paces this: r06)
    (void)check_interval;
    std::vector<int> budget(B);
    for (int b = 0; b < B; ++b) budget[b] = std::min(max_tokens, D.n_ctx - prompt_lens[b] + 1);
    constexpr int kRunDepth = 2;
    const int gs = graph_steps();
    for (int issued = 0, k = 0; issued < max_tokens; ++k) {
        if (k >= kRunDepth) MIO_HIP_CHECK(hipEventSynchronize(m->run_ev[k - kRunDepth]));
        bool all = true;
        for (int b = 0; b < B && all; ++b)
            all = issued >= budget[b] || __atomic_load_n(m->host_done + 1 + b, __ATOMIC_ACQUIRE);
        if (all) break;
        const int n = std::min(gs, max_tokens - issued);
        if ((rc = run_batch(m, n))) return rc;
        issued += n;
        if ((int)m->run_ev.size() <= k) {
            hipEvent_t e = nullptr;
            MIO_HIP_CHECK(hipEventCreate(&e));
            m->run_ev.push_back(e);
        }
        MIO_HIP_CHECK(hipEventRecord(m->run_ev[k], s));
    }
    std::vector<mio::StepState> hs(B);
    MIO_HIP_CHECK(hipMemcpyAsync(hs.data(), bt.st, B * sizeof(mio::StepState), hipMemcpyDeviceToHost, s));
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<int32_t> ring(max_tokens);
    for (int b = 0; b < B; ++b) {
        const int P = prompt_lens[b] - 1;
        const int n = std::max(0, std::min(hs[b].step - P, max_tokens));
        if (n) MIO_HIP_CHECK(hipMemcpy(ring.data(), bt.tokens + (size_t)b * D.n_ctx + P, (size_t)n * 4,
                                       hipMemcpyDeviceToHost));
        int k = 0;
        while (k < n && ring[k] != eos0 && ring[k] != eos1) ++k;
        std::memcpy(out_tokens + (size_t)b * max_tokens, ring.data(), (size_t)k * 4);
        n_out[b] = k;
    }
    // the in-launch quantization's bounded wait (launch_mmq_q) raises this flag if a producer's
    // signal never came: an error instead of tokens computed from stale records
    int qflag = 0;
    MIO_HIP_CHECK(hipMemcpy(&qflag, m->pf.qcnt + mio::kQcntFlag, sizeof(int), hipMemcpyDeviceToHost));
    if (qflag) {
        MIO_HIP_CHECK(hipMemsetAsync(m->pf.qcnt + mio::kQcntFlag, 0, sizeof(int), m->d->stream));
        mio::set_error("llm_generate_batch: the in-launch quantization hand-off wait timed out");
        return MIO_ERR_HIP;
    }
    return MIO_OK;
}

extern "C" int mio_hip_llm_prefill(mio_hip_llm *m, const int32_t *tokens, int n_tokens, float *logits) {
    MIO_REQUIRE(m && tokens && n_tokens >= 1 && n_tokens <= m->dims.n_ctx, MIO_ERR_INVALID,
                "llm_prefill: bad args");
    for (int i = 0; i < n_tokens; ++i)
        MIO_REQUIRE(tokens[i] >= 0 && tokens[i] < m->dims.n_vocab, MIO_ERR_INVALID, "llm_prefill: token %d",
                    tokens[i]);
    int rc = mio::bind(m->d);
    if (rc) return rc;
    if (!m->bf16_mt()) {
        // forced decode steps as llm_begin runs them (the multi-token engine is int8-only):
        // step j decodes tokens[j] at position j and its sampler is forced to tokens[j + 1]
        if (n_tokens > 1) {
            mio::SampleCfg c{};
            c.temp = 0.0f, c.lo = 0, c.hi = m->dims.n_vocab, c.eos0 = c.eos1 = -1;
            c.force = m->d_force, c.n_force = m->max_steps, c.out_tokens = m->d_tokens, c.max_steps = m->max_steps;
            std::vector<int> force(m->max_steps, -1);
            for (int j = 0; j + 1 < n_tokens && j < m->max_steps; ++j) force[j] = tokens[j + 1];
            MIO_HIP_CHECK(hipMemcpyAsync(m->d_force, force.data(), force.size() * 4, hipMemcpyHostToDevice,
                                         m->d->stream));
            if ((rc = put_cfg(m, c)) || (rc = ensure_graph(m)) || (rc = set_state(m, 0, tokens[0]))) return rc;
            for (int j = 0; j + 1 < n_tokens; ++j) MIO_HIP_CHECK(hipGraphLaunch(m->graph, m->d->stream));
        }
    } else if ((rc = upload_prompt(m, tokens, n_tokens)) || (rc = prefill(m, n_tokens - 1))) {
        return rc;
    }
    return mio_hip_llm_eval(m, tokens[n_tokens - 1], n_tokens - 1, logits);
}

extern "C" int mio_hip_llm_logits(mio_hip_llm *m, float *logits) {
    MIO_REQUIRE(m && logits, MIO_ERR_INVALID, "llm_logits: null");
    int rc = mio::bind(m->d);
    if (rc) return rc;
    MIO_HIP_CHECK(hipMemcpyAsync(logits, m->buf.logits, (size_t)m->dims.n_vocab * 4, hipMemcpyDeviceToHost,
                                 m->d->stream));
    MIO_HIP_CHECK(hipStreamSynchronize(m->d->stream));
    return MIO_OK;
}

// The layer a diagnostic launch of kernel `which` runs on: the first layer at or after
// n_layer / 2 (wrapping) that has it (attention kernels 0..2: an attention layer; 8, 9: an
// lfm2 short-conv layer; others: any), or -1.
static int kernel_layer(const mio_hip_llm *m, int which) {
    for (int i = 0; i < m->n_layer; ++i) {
        const int il = (m->n_layer / 2 + i) % m->n_layer;
        const bool conv = m->layers[il].conv != 0;
        if (which == 11   ? !conv && fuse_layer_att(m, il)
            : which == 12 ? fuse_ffn(m, il)
            : which == 13 ? !conv && fuse_layer(m, il)
                          : (which <= 2 || which == 10 ? !conv : (which >= 8 ? conv : true)))
            return il;
    }
    return -1;
}

// Decode state a diagnostic launch may change, saved at entry and put back on exit: the
// StepState (k_lm_head sets `pending`, layer 0's k_ffn_in folds it into pos) and the
// residual x (attn_out / ffn_down / conv_out add into it; after a flush it holds the next
// token's embedding). The other buffers a launch writes are rewritten by the next real step
// before anything reads them: the K/V row and the short-conv ring slot of cur_pos (the
// owner stores them first), q|k|v, h, the chunk partials and the lm_head partials (the same
// inputs give the same values).
struct DiagStateGuard {
    mio_hip_llm *m;
    mio::StepState st{};
    float *x = nullptr;
    int rc = MIO_OK;
    explicit DiagStateGuard(mio_hip_llm *mm) : m(mm) {
        const size_t xb = (size_t)m->dims.n_embd * sizeof(float);
        if (hipStreamSynchronize(m->d->stream) != hipSuccess ||
            hipMemcpy(&st, m->buf.st, sizeof(st), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMalloc(&x, xb) != hipSuccess || hipMemcpy(x, m->buf.x, xb, hipMemcpyDeviceToDevice) != hipSuccess)
        {
            mio::set_error("llm diagnostic: saving the decode state failed");
            rc = MIO_ERR_HIP;
        }
    }
    ~DiagStateGuard() {
        hipStreamSynchronize(m->d->stream);
        if (x) {
            hipMemcpy(m->buf.x, x, (size_t)m->dims.n_embd * sizeof(float), hipMemcpyDeviceToDevice);
            hipFree(x);
        }
        if (rc == MIO_OK) hipMemcpy(m->buf.st, &st, sizeof(st), hipMemcpyHostToDevice);
    }
};

// Live timing of one kernel of the decode step (bench.py roofline): launches kernel
// `which` (0 attn_in, 1 attention, 2 attn_out, 3 ffn_in, 4 ffn_down, 6 lm_head, 8 conv_in,
// 9 conv_out, 10-13 the fused launches) of layer kernel_layer() `iters` times on the runner's
// stream between HIP events (MIO_TK_MODE below), with the buffers and
// device state left by the last generate/eval. Returns the mean duration and the
// algorithmic HBM bytes of one launch (weights of the matrices it streams + activations;
// attention: F16 K and V rows of positions 0..pos (the row at pos is written, the rest
// read) + q|k|v in + partial records out, at the decode state's current pos).
extern "C" int mio_hip_llm_time_kernel(mio_hip_llm *m, int which, int iters, float *avg_ms, uint64_t *bytes) {
    MIO_REQUIRE(m && avg_ms && bytes && iters > 0 && m->graph, MIO_ERR_INVALID,
                "llm_time_kernel: run generate/eval first");
    MIO_REQUIRE(which >= 0 && which <= 13 && which != 5 && which != 7, MIO_ERR_INVALID,
                "llm_time_kernel: which %d", which);
    MIO_REQUIRE(which < 10 || which == 12 || fuse_att_o(m), MIO_ERR_INVALID,
                "llm_time_kernel: no fused attention launch");
    const int il = kernel_layer(m, which);
    MIO_REQUIRE(il >= 0, MIO_ERR_INVALID, "llm_time_kernel: the model has no layer with kernel %d", which);
    int rc = mio::bind(m->d);
    if (rc) return rc;
    const mio::LayerW &L = m->layers[il];
    auto qbytes = [](const mio::QMat &q) {
        return (uint64_t)mio::ggml_row_bytes(q.type, q.k) * (uint64_t)q.rows;
    };
    const mio::LlmDims &D = m->dims;
    // attention reads the K/V rows of positions <= pos of the current decode state; the
    // decode state is put back on exit (DiagStateGuard)
    DiagStateGuard guard(m);
    if (guard.rc) return guard.rc;
    const mio::StepState &st = guard.st;
    // the position the attention kernels work at (cur_pos: pos + pending)
    const uint64_t pos = (uint64_t)std::max(0, std::min(st.pos + st.pending, D.n_ctx - 1));
    const uint64_t nch = pos / mio::kAttChunk + 1, qkv = (uint64_t)(D.n_head + 2 * D.n_kv) * D.hd;
    // chunk partial records {O, m, l}: written by the chunk workgroups, read back by the
    // merging one (attn_merge_last), which writes the n_head * hd outputs
    const uint64_t part = 4ull * D.n_head * nch * (D.hd + 2);
    uint64_t b = 0;
    const uint64_t att_bytes = 2ull * 2 * D.n_kv * D.hd * (pos + 1) + 4ull * qkv + 8ull * (D.hd / 2) + 2 * part +
                               4ull * D.n_head * D.hd;
    switch (which) {
        case 0: b = qbytes(L.wq) + qbytes(L.wk) + qbytes(L.wv) + 4ull * D.n_embd + 4ull * qkv; break;
        case 1: b = att_bytes; break;
        case 2: b = qbytes(L.wo) + 4ull * D.n_head * D.hd + 4ull * D.n_embd * 2; break;
        case 10: b = att_bytes + qbytes(L.wo) + 4ull * D.n_head * D.hd + 4ull * D.n_embd * 2; break;
        // q|k|v written and read back by the attention workgroups: counted once each way
        case 11:
            b = qbytes(L.wq) + qbytes(L.wk) + qbytes(L.wv) + 4ull * D.n_embd + att_bytes + qbytes(L.wo) +
                4ull * D.n_head * D.hd + 4ull * D.n_embd * 2;
            break;
        case 3: b = qbytes(L.gate) + qbytes(L.up) + 4ull * (D.n_embd * 2 + D.n_ff); break;
        case 4: b = qbytes(L.down) + 4ull * (D.n_ff + 2 * D.n_embd); break;
        // the whole layer: k_layer_att's bytes + k_ffn's (x handed over in-launch: counted once
        // each way like q|k|v and h)
        case 13:
            b = qbytes(L.wq) + qbytes(L.wk) + qbytes(L.wv) + 4ull * D.n_embd + att_bytes + qbytes(L.wo) +
                4ull * D.n_head * D.hd + 4ull * D.n_embd * 2 + qbytes(L.gate) + qbytes(L.up) +
                4ull * (D.n_embd * 2 + D.n_ff) + qbytes(L.down) + 4ull * (D.n_ff + 2 * D.n_embd);
            break;
        // h written and read back by the down workgroups: counted once each way
        case 12:
            b = qbytes(L.gate) + qbytes(L.up) + 4ull * (D.n_embd * 2 + D.n_ff) + qbytes(L.down) +
                4ull * (D.n_ff + 2 * D.n_embd);
            break;
        case 6: b = qbytes(m->lm) + 4ull * D.n_vocab; break;
        case 8: b = qbytes(L.in_proj) + 4ull * D.n_embd * 4; break;
        // B | C | X in, taps, the two window rows, this position's bx (one workgroup), x in / out
        case 9: b = qbytes(L.out_proj) + 4ull * D.n_embd * (3 + mio::kConvL + 2 + 1 + 2); break;
    }
    hipEvent_t e0, e1;
    MIO_HIP_CHECK(hipEventCreate(&e0));
    MIO_HIP_CHECK(hipEventCreate(&e1));
    hipStream_t s = m->d->stream;
    // The fused launches' hand-off counters are zeroed by the launch after them in a step: here
    // a memset does it before every launch. MIO_TK_MODE (default 1): how the iters launches are
    // timed with HIP events.
    //   0: issued eagerly, minus an eager loop of the memsets alone (rounds 4-6; the host issues
    //      a memset + launch pair in about the GPU time of one, so both loops are partly
    //      host-paced: k_layer_att's figure moved 11.7-14.9 us between runs of one tree);
    //   1: both loops captured as hipGraphs and replayed (GPU-paced, +-0.3 % between reps):
    //      k_layer_att 12.1 us vs the eager rocprof mean 12.65 of a real step, k_ffn 10.65 vs
    //      10.9, lm_head 46-48 vs 47.2 (profiles/r06/time_kernel_modes.txt);
    //   2: as 1, with the reference loop launching an empty one-workgroup kernel (launch_nop)
    //      after each memset: per launch = the kernel minus an empty launch (1.5-2 us below the
    //      rocprof durations, which count a launch's dispatch).
    static const int tk_mode = getenv("MIO_TK_MODE") ? atoi(getenv("MIO_TK_MODE")) : 1;
    const bool fused = which >= 10;
    int *rdy = m->buf.att_cnt + mio::kRdyOff;
    const size_t rdy_bytes = (size_t)(mio::kAttCntInts - mio::kRdyOff) * sizeof(int);
    // ref: 0 = the kernel itself, 1 = nothing (memset only), 2 = the empty launch
    auto launch = [&](int ref) {
        if (fused) MIO_HIP_CHECK(hipMemsetAsync(rdy, 0, rdy_bytes, s));
        if (ref == 0)
            mio::launch_step_kernel(which, D, m->layers.data(), il, m->kc, m->vc, m->out_norm, m->lm, m->tok, m->buf,
                                    s);
        else if (ref == 2)
            mio::launch_nop(s);
        return MIO_OK;
    };
    auto timed = [&](int ref, float &ms) {
        hipGraphExec_t ge = nullptr;
        if (tk_mode >= 1) {
            hipGraph_t g = nullptr;
            MIO_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            int rc = MIO_OK;
            for (int i = 0; i < iters && rc == MIO_OK; ++i) rc = launch(ref);
            const hipError_t ec = hipStreamEndCapture(s, &g);
            if (rc) return rc;
            MIO_HIP_CHECK(ec);
            const hipError_t ei = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            hipGraphDestroy(g);
            MIO_HIP_CHECK(ei);
            MIO_HIP_CHECK(hipGraphLaunch(ge, s));  // warm replay
        }
        MIO_HIP_CHECK(hipEventRecord(e0, s));
        if (ge) {
            MIO_HIP_CHECK(hipGraphLaunch(ge, s));
        } else {
            for (int i = 0; i < iters; ++i)
                if (int rc = launch(ref)) return rc;
        }
        MIO_HIP_CHECK(hipEventRecord(e1, s));
        MIO_HIP_CHECK(hipEventSynchronize(e1));
        MIO_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ge) hipGraphExecDestroy(ge);
        return MIO_OK;
    };
    if (int rc = launch(0)) return rc;  // warm
    float ms = 0, ms_ref = 0;
    if (int rc = timed(0, ms)) return rc;
    const int ref = tk_mode == 2 ? 2 : (fused ? 1 : -1);
    if (ref > 0) {
        if (int rc = timed(ref, ms_ref)) return rc;
        ms = std::max(0.0f, ms - ms_ref);
    }
    hipEventDestroy(e0), hipEventDestroy(e1);
    *avg_ms = ms / iters;
    *bytes = b;
    return MIO_OK;
}

// Runs kernel `which` once (after a warm launch) with checkpoint tracing on; out[0..31]:
// s_memtime at checkpoints 0..15 of workgroup 0 / thread 0, s_memrealtime (100 MHz) at
// checkpoints 0 and 15 in out[16] / out[31]. Diagnostic only.
extern "C" int mio_hip_llm_trace_kernel(mio_hip_llm *m, int which, uint64_t *out) {
    MIO_REQUIRE(m && out && m->graph, MIO_ERR_INVALID, "llm_trace_kernel: run generate/eval first");
    MIO_REQUIRE(which >= 0 && which <= 13 && which != 5, MIO_ERR_INVALID, "llm_trace_kernel: which %d", which);
    MIO_REQUIRE(which < 10 || fuse_att_o(m), MIO_ERR_INVALID, "llm_trace_kernel: no fused attention launch");
    const int il = kernel_layer(m, which);
    MIO_REQUIRE(il >= 0, MIO_ERR_INVALID, "llm_trace_kernel: the model has no layer with kernel %d", which);
    int rc = mio::bind(m->d);
    if (rc) return rc;
    hipStream_t s = m->d->stream;
    DiagStateGuard guard(m);  // the decode state is put back on exit
    if (guard.rc) return guard.rc;
    unsigned long long *dt = nullptr;
    MIO_HIP_CHECK(hipMalloc(&dt, 32 * sizeof(unsigned long long)));
    MIO_HIP_CHECK(hipMemsetAsync(dt, 0, 32 * sizeof(unsigned long long), s));
    if (which >= 10)
        MIO_HIP_CHECK(hipMemsetAsync(m->buf.att_cnt + mio::kRdyOff, 0,
                                     (size_t)(mio::kAttCntInts - mio::kRdyOff) * sizeof(int), s));
    mio::launch_step_kernel(which, m->dims, m->layers.data(), il, m->kc, m->vc, m->out_norm, m->lm, m->tok, m->buf,
                            s);
    // evict L2 / MALL so the traced launch streams its weights from HBM as in a real step
    void *flush = nullptr;
    const size_t flush_bytes = (size_t)1 << 30;
    if (hipMalloc(&flush, flush_bytes) == hipSuccess) {
        hipMemsetAsync(flush, 1, flush_bytes, s);
        hipMemsetAsync(flush, 2, flush_bytes, s);
    }
    mio::LlmBuffers tb = m->buf;
    tb.trace = dt;
    if (which >= 10)
        MIO_HIP_CHECK(hipMemsetAsync(m->buf.att_cnt + mio::kRdyOff, 0,
                                     (size_t)(mio::kAttCntInts - mio::kRdyOff) * sizeof(int), s));
    mio::launch_step_kernel(which, m->dims, m->layers.data(), il, m->kc, m->vc, m->out_norm, m->lm, m->tok, tb,
                            s);
    MIO_HIP_CHECK(hipMemcpyAsync(out, dt, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    hipFree(dt);
    if (flush) hipFree(flush);
    return MIO_OK;
}

// Diagnostic: captures one decode step as a graph with the step timeline on, replays it
// (advancing the decode state by 3 steps: reset/eval afterwards), and returns per launch
// and workgroup {start, marks 1-6, end} in s_memrealtime ticks (100 MHz).
extern "C" int mio_hip_llm_timeline(mio_hip_llm *m, uint64_t *out, int max_launches, int *n_launches) {
    MIO_REQUIRE(m && out && n_launches && m->graph, MIO_ERR_INVALID, "llm_timeline: run generate/eval first");
    int rc = mio::bind(m->d);
    if (rc) return rc;
    const int nl = (int)step_kinds(m).size();
    MIO_REQUIRE(max_launches >= nl, MIO_ERR_INVALID, "llm_timeline: need %d launch slots", nl);
    hipStream_t s = m->d->stream;
    const size_t nslot = (size_t)nl * mio::kTlSlots * 8;  // MIO_TL_SLOT: kTlSlots workgroup slots per launch
    unsigned long long *tl = nullptr;
    MIO_HIP_CHECK(hipMalloc(&tl, sizeof(unsigned long long) * nslot));
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    MIO_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    rc = issue_step(m, tl);
    MIO_HIP_CHECK(hipStreamEndCapture(s, &g));
    MIO_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
        MIO_HIP_CHECK(hipMemsetAsync(tl, 0, sizeof(unsigned long long) * nslot, s));
        MIO_HIP_CHECK(hipGraphLaunch(ge, s));
    }
    std::vector<unsigned long long> h(nslot);
    MIO_HIP_CHECK(hipMemcpyAsync(h.data(), tl, sizeof(unsigned long long) * nslot, hipMemcpyDeviceToHost, s));
    MIO_HIP_CHECK(hipStreamSynchronize(s));
    std::memcpy(out, h.data(), sizeof(unsigned long long) * nslot);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    hipFree(tl);
    *n_launches = nl;
    return MIO_OK;
}
