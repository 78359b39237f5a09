// The reference's C++ call surface on the MI355X path: VoiceModel / TestToSpeech
// (test-to-speech.h:11-123), miocodec_* (miocodec.h:10-43) and istft_cache / istft
// (istft.h:6-42). The synthesis policy (prompt template, sampling defaults, stop tokens,
// peak normalisation, the streaming holdback / commit / crossfade schedule) follows
// test-to-speech.cpp; the work runs on the GPU through the C-ABI handles:
//   run_llm              -> BpeTokenizer + mio::llm_begin/run/poll (one hipGraph per token,
//                           on-device temperature + Gumbel-max sampling, no per-token sync)
//   decode_*_to_audio    -> mio_hip_codec_decode_pcm (codec kernels + fused iSTFT) into HBM
//   peak normalisation   -> mio_hip_pcm_normalize / mio_hip_pcm_finish (device, bit-exact)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "gguf.h"
#include "istft.h"
#include "llm.h"
#include "stream_policy.h"
#include "mio_hip.h"
#include "miocodec.h"
#include "test-to-speech.h"
#include "text-normalize.h"
#include "token-parser.h"
#include "tokenizer.h"
#include "wav-writer.h"
#include "wav.h"

namespace mio {

// Process-wide device handles: opened once per GPU index, kept for the process lifetime.
mio_hip_device *default_device(int want) {
    static std::mutex mu;
    static std::map<int, mio_hip_device *> open;
    int dev = want;
    if (dev < 0) {
        const char *e = getenv("MIO_DEVICE");
        if (!e || !*e) e = getenv("LOCAL_RANK");
        dev = (e && *e) ? atoi(e) : 0;
    }
    std::lock_guard<std::mutex> lk(mu);
    auto it = open.find(dev);
    if (it != open.end()) return it->second;
    mio_hip_device *d = nullptr;
    if (mio_hip_device_open(dev, &d) != MIO_OK) {
        fprintf(stderr, "miotts: cannot open GPU %d: %s\n", dev, mio_hip_last_error());
        return nullptr;
    }
    open[dev] = d;
    return d;
}

}  // namespace mio

// ------------------------------------------------------------------ istft.h
struct istft_cache::gpu_state {
    mio_hip_device *dev = nullptr;
    mio_hip_istft *h = nullptr;
    ~gpu_state() {
        if (h) mio_hip_istft_destroy(h);
    }
};

istft_cache::istft_cache(int n_fft, int win_length)
    : n_fft_(n_fft), win_length_(win_length), n_freq_(n_fft / 2 + 1), n_mid_(std::max(0, n_fft / 2 - 1)) {
    // trig tables with the argument formed in float (istft.cpp:18-26), periodic Hann (:29-31)
    cos_table_.resize((size_t)n_fft_ * n_mid_);
    sin_table_.resize((size_t)n_fft_ * n_mid_);
    nyquist_sign_.resize(n_fft_);
    hann_window_.resize(win_length_);
    const float step = 2.0f * (float)M_PI / (float)n_fft_;
    for (int n = 0; n < n_fft_; ++n) {
        nyquist_sign_[n] = (n % 2) ? -1.0f : 1.0f;
        float *c = cos_table_.data() + (size_t)n * n_mid_;
        float *s = sin_table_.data() + (size_t)n * n_mid_;
        for (int k = 1; k <= n_mid_; ++k) {
            const float arg = step * (float)k * (float)n;
            c[k - 1] = cosf(arg);
            s[k - 1] = sinf(arg);
        }
    }
    for (int i = 0; i < win_length_; ++i) hann_window_[i] = 0.5f * (1.0f - cosf(2.0f * (float)M_PI * i / win_length_));
}

istft_cache::~istft_cache() = default;

int istft_cache::n_fft() const { return n_fft_; }
int istft_cache::win_length() const { return win_length_; }
int istft_cache::n_freq() const { return n_freq_; }
int istft_cache::n_mid() const { return n_mid_; }
const std::vector<float> &istft_cache::cos_table() const { return cos_table_; }
const std::vector<float> &istft_cache::sin_table() const { return sin_table_; }
const std::vector<float> &istft_cache::nyquist_sign() const { return nyquist_sign_; }
const std::vector<float> &istft_cache::hann_window() const { return hann_window_; }

istft_cache::gpu_state *istft_cache::gpu(int device) const {
    if (gpu_) return gpu_.get();
    auto g = std::make_unique<gpu_state>();
    g->dev = mio::default_device(device);
    if (!g->dev || mio_hip_istft_create(g->dev, n_fft_, win_length_, &g->h) != MIO_OK) {
        fprintf(stderr, "istft: GPU iSTFT unavailable: %s\n", mio_hip_last_error());
        return nullptr;
    }
    gpu_ = std::move(g);
    return gpu_.get();
}

std::vector<float> istft(const float *spec, int n_frames, int hop_length, const istft_cache &cache) {
    if (!spec || n_frames <= 0 || hop_length <= 0) return {};
    istft_cache::gpu_state *g = cache.gpu();
    if (!g) return {};
    int len = 0;
    if (mio_hip_istft_out_len(g->h, n_frames, hop_length, &len) != MIO_OK || len <= 0) return {};
    std::vector<float> out(len);
    if (mio_hip_istft_run(g->h, spec, n_frames, hop_length, out.data(), &len, 0, nullptr) != MIO_OK) {
        fprintf(stderr, "istft: %s\n", mio_hip_last_error());
        return {};
    }
    out.resize(len);
    return out;
}

// ------------------------------------------------------------------ miocodec.h
struct miocodec_context {
    mio_hip_device *dev = nullptr;
    mio_hip_codec *codec = nullptr;
    int info[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // sample_rate, n_fft, hop, spt, n_freq, stages, fpc, n_codes
};

miocodec_context *miocodec_load(const std::string &model_path) {
    mio_hip_device *d = mio::default_device(-1);
    if (!d) return nullptr;
    auto *c = new miocodec_context();
    c->dev = d;
    if (mio_hip_codec_load(d, model_path.c_str(), &c->codec) != MIO_OK ||
        mio_hip_codec_info(c->codec, c->info) != MIO_OK) {
        fprintf(stderr, "miocodec: failed to load %s: %s\n", model_path.c_str(), mio_hip_last_error());
        if (c->codec) mio_hip_codec_free(c->codec);
        delete c;
        return nullptr;
    }
    return c;
}

void miocodec_free(miocodec_context *ctx) {
    if (!ctx) return;
    if (ctx->codec) mio_hip_codec_free(ctx->codec);
    delete ctx;
}

std::vector<float> miocodec_decode(miocodec_context *ctx, const int *codes, int n_codes, const float *global_emb,
                                   int audio_length, int *out_n_frames) {
    if (!ctx || !codes || n_codes <= 0 || !global_emb) return {};
    const int frames = n_codes * ctx->info[6];
    if (audio_length == 0) audio_length = n_codes * ctx->info[3];
    fprintf(stderr, "miocodec: T=%d codes -> %d STFT frames -> %d audio samples (MI355X)\n", n_codes, frames,
            audio_length);
    std::vector<float> spec((size_t)frames * ctx->info[4] * 2);
    int got = 0;
    if (mio_hip_codec_decode(ctx->codec, codes, n_codes, global_emb, spec.data(), &got, 0, nullptr) != MIO_OK) {
        fprintf(stderr, "miocodec: decode failed: %s\n", mio_hip_last_error());
        return {};
    }
    if (out_n_frames) *out_n_frames = got;
    return spec;
}

int miocodec_sample_rate(const miocodec_context *ctx) { return ctx ? ctx->info[0] : 0; }
int miocodec_n_fft(const miocodec_context *ctx) { return ctx ? ctx->info[1] : 0; }
int miocodec_hop_length(const miocodec_context *ctx) { return ctx ? ctx->info[2] : 0; }
int miocodec_samples_per_token(const miocodec_context *ctx) { return ctx ? ctx->info[3] : 0; }

std::vector<float> load_voice_embedding(const std::string &path) {
    mio::GgufFile g;
    if (!g.open(path)) {
        fprintf(stderr, "voice_emb: failed to open %s: %s\n", path.c_str(), mio::last_error());
        return {};
    }
    if (g.tensors().empty()) {
        fprintf(stderr, "voice_emb: no tensors in %s\n", path.c_str());
        return {};
    }
    const mio::GgufTensor &t = g.tensors()[0];
    if (t.type != mio::GGML_F32) {
        fprintf(stderr, "voice_emb: unsupported type %u\n", t.type);
        return {};
    }
    std::vector<float> emb((size_t)t.nelements());
    std::copy((const float *)t.data, (const float *)t.data + emb.size(), emb.begin());
    fprintf(stderr, "voice_emb: loaded %zu-dim from %s\n", emb.size(), path.c_str());
    return emb;
}

void miocodec_print_tensors(const std::string &path) {
    mio::GgufFile g;
    if (!g.open(path)) {
        fprintf(stderr, "failed to open %s\n", path.c_str());
        return;
    }
    printf("Tensors in %s: %lld\n", path.c_str(), (long long)g.tensors().size());
    for (const mio::GgufTensor &t : g.tensors())
        printf("  %-60s [%5lld, %5lld, %5lld, %5lld] type=%u\n", t.name.c_str(), (long long)t.ne[0],
               (long long)t.ne[1], (long long)t.ne[2], (long long)t.ne[3], t.type);
}

// ------------------------------------------------------------------ test-to-speech.h
bool VoiceModel::load_from_file(const std::string &path) {
    std::vector<float> e = load_voice_embedding(path);
    if (e.empty()) return false;
    path_ = path;
    embedding_ = std::move(e);
    return true;
}
bool VoiceModel::is_ready() const { return !embedding_.empty(); }
const std::vector<float> &VoiceModel::embedding() const { return embedding_; }
const std::string &VoiceModel::path() const { return path_; }

struct TestToSpeech::Impl {
    mio_hip_device *dev = nullptr;
    mio_hip_llm *llm = nullptr;
    miocodec_context *codec = nullptr;
    mio::BpeTokenizer tok;
    int32_t eos = -1, im_end = -1;
    int sample_rate = 0, n_fft = 0, hop = 0, spt = 0;

    // PCM of the last decode in HBM (f32) and its PCM16 image (synthesize_to_file)
    void *d_pcm = nullptr, *d_pcm16 = nullptr;
    size_t pcm_cap = 0, pcm16_cap = 0;
    // batch synthesis: one f32 PCM buffer per utterance of a group (concurrent codec decodes)
    std::vector<void *> d_pcmb;
    std::vector<size_t> pcmb_cap;
    // streaming decodes run on their own stream, beside the LLM's next check interval
    hipStream_t cstream = nullptr;

    ~Impl() {
        if (cstream) hipStreamDestroy(cstream);
        if (llm) mio_hip_llm_free(llm);
        if (dev && d_pcm) mio_hip_free(dev, d_pcm);
        if (dev && d_pcm16) mio_hip_free(dev, d_pcm16);
        for (void *p : d_pcmb)
            if (dev && p) mio_hip_free(dev, p);
        miocodec_free(codec);
    }

    bool ensure(void *&p, size_t &cap, size_t bytes) {
        if (cap >= bytes) return true;
        bytes = std::max(bytes, 2 * cap);  // geometric growth: a free waits for the device
        if (p) mio_hip_free(dev, p);
        p = nullptr, cap = 0;
        if (mio_hip_malloc(dev, bytes, &p) != MIO_OK) {
            fprintf(stderr, "TestToSpeech: device buffer of %zu bytes: %s\n", bytes, mio_hip_last_error());
            return false;
        }
        cap = bytes;
        return true;
    }

    // "<|startoftext|><|im_start|>user\n" + text + "<|im_end|>\n<|im_start|>assistant\n"
    // (test-to-speech.cpp:90-92)
    static std::string prompt_of(const std::string &text) {
        return "<|startoftext|><|im_start|>user\n" + text + "<|im_end|>\n<|im_start|>assistant\n";
    }

    std::vector<int32_t> prompt_tokens(const std::string &text) const {
        return tok.tokenize(prompt_of(normalize_tts_text(text)), true, true);
    }

    // benchmark-harness options (flagged deviations): speech ids only / no stop
    void harness(const Options &o, mio::SamplingParams &sp) const {
        if (o.speech_only) {
            const int32_t a = tok.special_id("<|s_0|>"), z = tok.special_id("<|s_12799|>");
            if (a >= 0 && z == a + 12799) sp.allow_lo = a, sp.allow_hi = z + 1;
        }
        if (o.ignore_eos) sp.eos0 = sp.eos1 = -1;
    }

    // codes -> PCM in HBM (d_pcm, *len samples): codec + fused iSTFT, stage seconds from GPU
    // events
    // incremental: streaming re-decodes reuse the prenet rows of the previous one
    // (MIO_CODEC_INCREMENTAL; the output equals a full decode up to f32 summation order)
    bool decode_codes_dev(const VoiceModel &voice, const std::vector<int> &codes, int *len, double *codec_sec,
                          double *istft_sec, bool incremental = false, hipStream_t stream = nullptr) {
        if (!ensure(d_pcm, pcm_cap, (size_t)codes.size() * spt * sizeof(float) + 64)) return false;
        const unsigned flags = MIO_OUT_DEVICE | (incremental ? MIO_CODEC_INCREMENTAL : 0u);
        if (mio_hip_codec_decode_pcm(codec->codec, codes.data(), (int)codes.size(), voice.embedding().data(),
                                     (float *)d_pcm, len, flags, stream) != MIO_OK) {
            fprintf(stderr, "TestToSpeech: codec decode failed: %s\n", mio_hip_last_error());
            return false;
        }
        float ms[2] = {0.0f, 0.0f};
        if (mio_hip_codec_last_timings(codec->codec, ms) == MIO_OK) {
            if (codec_sec) *codec_sec += ms[0] * 1e-3;
            if (istft_sec) *istft_sec += ms[1] * 1e-3;
        }
        return true;
    }

    // codes -> host PCM; the peak normalisation of test-to-speech.cpp:232-243 (when asked)
    // runs on the device before the copy (mio_hip_pcm_normalize, bit-exact with the host loop)
    // stream (optional): decode and copy on that stream (the streaming path's codec stream)
    bool decode_codes(const VoiceModel &voice, const std::vector<int> &codes, std::vector<float> &pcm,
                      double *codec_sec, double *istft_sec, bool normalize = false, bool incremental = false,
                      hipStream_t stream = nullptr) {
        int len = 0;
        if (!decode_codes_dev(voice, codes, &len, codec_sec, istft_sec, incremental, stream)) return false;
        if (stream) {
            pcm.resize(len);
            if (len && (hipMemcpyAsync(pcm.data(), d_pcm, (size_t)len * sizeof(float), hipMemcpyDeviceToHost,
                                       stream) != hipSuccess ||
                        hipStreamSynchronize(stream) != hipSuccess)) {
                fprintf(stderr, "TestToSpeech: PCM copy failed\n");
                return false;
            }
            return true;
        }
        if (normalize && mio_hip_pcm_normalize(dev, (const float *)d_pcm, len, (float *)d_pcm, nullptr, nullptr)) {
            fprintf(stderr, "TestToSpeech: peak normalisation failed: %s\n", mio_hip_last_error());
            return false;
        }
        pcm.resize(len);
        if (len && mio_hip_memcpy_d2h(dev, pcm.data(), d_pcm, (size_t)len * sizeof(float)) != MIO_OK) {
            fprintf(stderr, "TestToSpeech: PCM copy failed: %s\n", mio_hip_last_error());
            return false;
        }
        return true;
    }
};

static int cstream_priority() {
    int least = 0, greatest = 0;
    hipDeviceGetStreamPriorityRange(&least, &greatest);
    const char *e = getenv("MIO_CSTREAM_PRIO");
    const std::string v = e ? e : "normal";
    if (v == "low") return least;
    if (v == "high") return greatest;
    return 0;
}

TestToSpeech::TestToSpeech(const Config &config) : config_(config), impl_(std::make_unique<Impl>()) {
    Impl &I = *impl_;
    I.dev = mio::default_device(config_.device);
    if (!I.dev) return;
    if (!config_.model_path.empty()) {
        mio::GgufFile g;
        if (!g.open(config_.model_path) || !I.tok.load(g)) {
            fprintf(stderr, "TestToSpeech: failed to load LLM tokenizer: %s (%s)\n", config_.model_path.c_str(),
                    mio::last_error());
            return;
        }
        g.close();
        if (mio_hip_llm_load(I.dev, config_.model_path.c_str(), 2048, &I.llm) != MIO_OK) {
            fprintf(stderr, "TestToSpeech: failed to load LLM model: %s (%s)\n", config_.model_path.c_str(),
                    mio_hip_last_error());
            I.llm = nullptr;
            return;
        }
        I.eos = I.tok.eos();
        I.im_end = I.tok.special_id("<|im_end|>");
    }
    I.codec = miocodec_load(config_.codec_path);
    if (!I.codec) {
        fprintf(stderr, "TestToSpeech: failed to load codec: %s\n", config_.codec_path.c_str());
        return;
    }
    I.sample_rate = miocodec_sample_rate(I.codec);
    I.n_fft = miocodec_n_fft(I.codec);
    I.hop = miocodec_hop_length(I.codec);
    I.spt = miocodec_samples_per_token(I.codec);
    // device memory for utterances of up to max_tokens codes, allocated with the models (as
    // llama_init_from_model / miocodec_load reserve theirs): codec workspace and prenet cache,
    // the PCM and PCM16 buffers; a synthesis then allocates nothing on the device
    const int reserve = config_.max_tokens > 0 ? config_.max_tokens : 700;
    if (mio_hip_codec_reserve(I.codec->codec, reserve) != MIO_OK ||
        (I.spt > 0 && (!I.ensure(I.d_pcm, I.pcm_cap, (size_t)reserve * I.spt * sizeof(float) + 64) ||
                       !I.ensure(I.d_pcm16, I.pcm16_cap, (size_t)reserve * I.spt * 2 + 64)))) {
        fprintf(stderr, "TestToSpeech: device buffers for %d codes failed: %s\n", reserve, mio_hip_last_error());
        miocodec_free(I.codec);
        I.codec = nullptr;
        return;
    }
    // the streaming path's codec stream (MIO_CSTREAM_PRIO=low|normal|high: its priority
    // relative to the LLM's normal-priority stream)
    if (hipStreamCreateWithPriority(&I.cstream, hipStreamNonBlocking, cstream_priority()) != hipSuccess) {
        fprintf(stderr, "TestToSpeech: codec stream creation failed\n");
        I.cstream = nullptr;
    }
}

TestToSpeech::~TestToSpeech() = default;

bool TestToSpeech::is_ready() const { return impl_ && impl_->codec != nullptr; }
int TestToSpeech::sample_rate() const { return impl_ ? impl_->sample_rate : 0; }

bool TestToSpeech::generate_token_text(const std::string &text, const Options &options, std::string &out) {
    out.clear();
    if (options.skip_llm) {
        out = text;
        return true;
    }
    Impl &I = *impl_;
    if (!I.llm) {
        fprintf(stderr, "TestToSpeech: LLM model is not loaded\n");
        return false;
    }
    const float temp = options.temperature >= 0.0f ? options.temperature : config_.temperature;
    const int max_tokens = options.max_tokens > 0 ? options.max_tokens : config_.max_tokens;
    const std::vector<int32_t> prompt = I.prompt_tokens(text);
    if (prompt.empty()) {
        fprintf(stderr, "TestToSpeech: tokenization failed\n");
        return false;
    }
    mio::SamplingParams sp;
    sp.temperature = temp, sp.seed = 42, sp.eos0 = I.eos, sp.eos1 = I.im_end;
    I.harness(options, sp);
    std::vector<int32_t> toks((size_t)max_tokens);
    int n = 0;
    if (mio_hip_llm_generate(I.llm, prompt.data(), (int)prompt.size(), max_tokens, temp, sp.seed, sp.allow_lo,
                             sp.allow_hi, sp.eos0, sp.eos1, 32, toks.data(), &n) != MIO_OK) {
        fprintf(stderr, "TestToSpeech: decode failed: %s\n", mio_hip_last_error());
        return false;
    }
    for (int i = 0; i < n; ++i) out += I.tok.piece(toks[i]);
    return !out.empty();
}

bool TestToSpeech::synthesize_to_vector(const VoiceModel &voice, const std::string &text, std::vector<float> &out_audio,
                                        const Options &options) {
    if (!is_ready()) {
        fprintf(stderr, "TestToSpeech: not ready\n");
        return false;
    }
    if (!voice.is_ready()) {
        fprintf(stderr, "TestToSpeech: voice model is not ready\n");
        return false;
    }
    std::string token_text;
    if (!generate_token_text(text, options, token_text)) return false;
    const std::vector<int> codes = parse_speech_tokens(token_text);
    if (codes.empty()) {
        fprintf(stderr, "TestToSpeech: no speech codes parsed from text\n");
        return false;
    }
    return impl_->decode_codes(voice, codes, out_audio, nullptr, nullptr, options.apply_peak_normalization);
}

bool TestToSpeech::synthesize_to_vector(const VoiceModel &voice, const std::string &text,
                                        std::vector<float> &out_audio) {
    return synthesize_to_vector(voice, text, out_audio, Options{});
}

// synthesize_to_vector + wav_write (test-to-speech.cpp:322-330) with the PCM kept in HBM:
// peak normalisation and the PCM16 conversion run on the device (mio_hip_pcm_finish), only the
// 2-byte samples cross PCIe; the file bytes equal wav_write(normalised floats).
bool TestToSpeech::synthesize_to_file(const VoiceModel &voice, const std::string &text,
                                      const std::string &output_path, const Options &options) {
    if (!is_ready() || !voice.is_ready()) {
        fprintf(stderr, "TestToSpeech: %s\n", !is_ready() ? "not ready" : "voice model is not ready");
        return false;
    }
    std::string token_text;
    if (!generate_token_text(text, options, token_text)) return false;
    const std::vector<int> codes = parse_speech_tokens(token_text);
    if (codes.empty()) {
        fprintf(stderr, "TestToSpeech: no speech codes parsed from text\n");
        return false;
    }
    Impl &I = *impl_;
    int len = 0;
    if (!I.decode_codes_dev(voice, codes, &len, nullptr, nullptr) ||
        !I.ensure(I.d_pcm16, I.pcm16_cap, (size_t)len * 2 + 64))
        return false;
    std::vector<int16_t> pcm16(len);
    if (mio_hip_pcm_finish(I.dev, (const float *)I.d_pcm, len, options.apply_peak_normalization ? 1 : 0,
                           (int16_t *)I.d_pcm16, nullptr, nullptr) != MIO_OK ||
        (len && mio_hip_memcpy_d2h(I.dev, pcm16.data(), I.d_pcm16, (size_t)len * 2) != MIO_OK)) {
        fprintf(stderr, "TestToSpeech: PCM epilogue failed: %s\n", mio_hip_last_error());
        return false;
    }
    return mio::wav_write_pcm16(output_path, pcm16.data(), pcm16.size(), sample_rate());
}

bool TestToSpeech::synthesize_to_file(const VoiceModel &voice, const std::string &text,
                                      const std::string &output_path) {
    return synthesize_to_file(voice, text, output_path, Options{});
}

// Batched synthesis (extension): prompts in groups of up to 16 through the batched decode
// engine, the group's codec + iSTFT decodes concurrently, then the PCM epilogue per utterance as
// synthesize_to_file does it.
// Every stream uses synthesize_to_file's seed, so each file has the bytes a single call writes
// (mio_hip_llm_generate_batch's streams equal mio_hip_llm_generate of their prompts).
bool TestToSpeech::synthesize_batch_to_files(const VoiceModel &voice, const std::vector<std::string> &texts,
                                             const std::vector<std::string> &output_paths, const Options &options) {
    if (!is_ready() || !voice.is_ready() || texts.size() != output_paths.size()) {
        fprintf(stderr, "TestToSpeech: %s\n",
                !is_ready() ? "not ready" : (!voice.is_ready() ? "voice model is not ready" : "texts / paths mismatch"));
        return false;
    }
    Impl &I = *impl_;
    if (options.skip_llm || !I.llm) {
        for (size_t i = 0; i < texts.size(); ++i)
            if (!synthesize_to_file(voice, texts[i], output_paths[i], options)) return false;
        return true;
    }
    const float temp = options.temperature >= 0.0f ? options.temperature : config_.temperature;
    const int max_tokens = options.max_tokens > 0 ? options.max_tokens : config_.max_tokens;
    mio::SamplingParams sp;
    sp.temperature = temp, sp.seed = 42, sp.eos0 = I.eos, sp.eos1 = I.im_end;
    I.harness(options, sp);
    constexpr size_t kGroup = 16;
    for (size_t g0 = 0; g0 < texts.size(); g0 += kGroup) {
        const int B = (int)std::min(kGroup, texts.size() - g0);
        std::vector<int32_t> prompts, lens;
        for (int b = 0; b < B; ++b) {
            const std::vector<int32_t> p = I.prompt_tokens(texts[g0 + b]);
            if (p.empty()) {
                fprintf(stderr, "TestToSpeech: tokenization failed\n");
                return false;
            }
            prompts.insert(prompts.end(), p.begin(), p.end());
            lens.push_back((int32_t)p.size());
        }
        std::vector<uint64_t> seeds((size_t)B, sp.seed);
        std::vector<int32_t> toks((size_t)B * max_tokens), n_out((size_t)B);
        if (mio_hip_llm_generate_batch(I.llm, prompts.data(), lens.data(), B, max_tokens, temp, seeds.data(),
                                       sp.allow_lo, sp.allow_hi, sp.eos0, sp.eos1, 32, toks.data(),
                                       n_out.data()) != MIO_OK) {
            // a model the batched engine does not take (or a failed hand-off): one utterance
            // at a time, said on stderr so the fallback is visible
            fprintf(stderr, "TestToSpeech: batched decode unavailable (%s); decoding one utterance at a time\n",
                    mio_hip_last_error());
            for (int b = 0; b < B; ++b)
                if (!synthesize_to_file(voice, texts[g0 + b], output_paths[g0 + b], options)) return false;
            continue;
        }
        // every stream's codes decoded concurrently (mio_hip_codec_decode_pcm_batch: the same
        // kernels per utterance, so the PCM is a single decode's), then synthesize_to_file's
        // epilogue (peak normalisation + PCM16 on the device, WAV) per utterance
        std::vector<std::vector<int32_t>> codes((size_t)B);
        for (int b = 0; b < B; ++b) {
            std::string text;
            for (int i = 0; i < n_out[b]; ++i) text += I.tok.piece(toks[(size_t)b * max_tokens + i]);
            const std::vector<int> c = parse_speech_tokens(text);
            if (c.empty()) {
                fprintf(stderr, "TestToSpeech: no speech codes parsed from text\n");
                fprintf(stderr, "TestToSpeech: utterance %zu failed\n", g0 + b);
                return false;
            }
            codes[b].assign(c.begin(), c.end());
        }
        I.d_pcmb.resize(std::max(I.d_pcmb.size(), (size_t)B), nullptr);
        I.pcmb_cap.resize(I.d_pcmb.size(), 0);
        std::vector<const int32_t *> cp((size_t)B);
        std::vector<float *> op((size_t)B);
        std::vector<int> nc((size_t)B), len((size_t)B);
        for (int b = 0; b < B; ++b) {
            if (!I.ensure(I.d_pcmb[b], I.pcmb_cap[b], codes[b].size() * I.spt * sizeof(float) + 64)) return false;
            cp[b] = codes[b].data(), op[b] = (float *)I.d_pcmb[b], nc[b] = (int)codes[b].size();
        }
        if (mio_hip_codec_decode_pcm_batch(I.codec->codec, cp.data(), nc.data(), B, voice.embedding().data(), op.data(),
                                           len.data(), MIO_OUT_DEVICE, nullptr) != MIO_OK) {
            fprintf(stderr, "TestToSpeech: codec decode failed: %s\n", mio_hip_last_error());
            return false;
        }
        for (int b = 0; b < B; ++b) {
            std::vector<int16_t> pcm16((size_t)len[b]);
            if (!I.ensure(I.d_pcm16, I.pcm16_cap, (size_t)len[b] * 2 + 64) ||
                mio_hip_pcm_finish(I.dev, op[b], len[b], options.apply_peak_normalization ? 1 : 0,
                                   (int16_t *)I.d_pcm16, nullptr, nullptr) != MIO_OK ||
                (len[b] && mio_hip_memcpy_d2h(I.dev, pcm16.data(), I.d_pcm16, (size_t)len[b] * 2) != MIO_OK)) {
                fprintf(stderr, "TestToSpeech: PCM epilogue failed: %s\n", mio_hip_last_error());
                return false;
            }
            if (!mio::wav_write_pcm16(output_paths[g0 + b], pcm16.data(), pcm16.size(), sample_rate())) return false;
        }
    }
    return true;
}

bool TestToSpeech::synthesize_stream(const VoiceModel &voice, const std::string &text, const StreamCallback &callback,
                                     size_t chunk_samples, const Options &options) {
    StreamProfile p;
    return synthesize_stream_profiled(voice, text, callback, chunk_samples, options, p);
}

bool TestToSpeech::synthesize_stream(const VoiceModel &voice, const std::string &text, const StreamCallback &callback,
                                     size_t chunk_samples) {
    return synthesize_stream(voice, text, callback, chunk_samples, Options{});
}

// Streaming (test-to-speech.cpp:435-614): the LLM runs 20 steps per check on the GPU
// (stream_check_interval); every check re-decodes all codes so far (the reference's
// quality-first full decode), commits all but a 32-code holdback once at least 24 new codes
// are committable, and emits them in chunk_samples pieces with a 30 ms linear crossfade.
bool TestToSpeech::synthesize_stream_profiled(const VoiceModel &voice, const std::string &text,
                                              const StreamCallback &callback, size_t chunk_samples,
                                              const Options &options, StreamProfile &profile) {
    using clk = std::chrono::steady_clock;
    auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
    profile = StreamProfile{};
    const auto t0 = clk::now();
    if (!callback || !is_ready()) return false;
    if (chunk_samples == 0) chunk_samples = 4096;
    Impl &I = *impl_;
    const int sr = I.sample_rate;
    const size_t xfade = std::min<size_t>((size_t)(sr * 3 / 100), 4096);
    std::vector<float> tail;

    auto call = [&](const float *p, size_t n, bool last) {
        const auto a = clk::now();
        const bool ok = callback(p, n, sr, last);
        profile.callback_sec += secs(a, clk::now());
        return ok;
    };
    auto emit = [&](const std::vector<float> &audio, size_t begin, size_t end, bool final_) -> bool {
        if (begin >= end) return final_ ? call(nullptr, 0, true) : true;
        for (size_t i = begin; i < end;) {
            const size_t n = std::min(chunk_samples, end - i);
            std::vector<float> chunk(audio.begin() + i, audio.begin() + i + n);
            if (i == begin && !tail.empty()) {
                const size_t m = std::min(tail.size(), n);
                for (size_t j = 0; j < m; ++j) {
                    const float a = (float)(j + 1) / (float)(m + 1);
                    chunk[j] = (1.0f - a) * tail[j] + a * chunk[j];
                }
            }
            if (n >= xfade)
                tail.assign(chunk.end() - xfade, chunk.end());
            else
                tail = chunk;
            if (!call(chunk.data(), n, final_ && i + n >= end)) return false;
            profile.emitted_samples += n;
            i += n;
        }
        return true;
    };

    if (options.skip_llm) {
        const std::vector<int> codes = parse_speech_tokens(text);
        std::vector<float> audio;
        if (codes.empty() || !I.decode_codes(voice, codes, audio, &profile.codec_sec, &profile.istft_sec)) {
            if (codes.empty()) fprintf(stderr, "TestToSpeech: no speech codes parsed from text\n");
            return false;
        }
        const bool ok = emit(audio, 0, audio.size(), true);
        profile.total_sec = secs(t0, clk::now());
        return ok;
    }
    if (!I.llm) {
        fprintf(stderr, "TestToSpeech: LLM model is not loaded\n");
        return false;
    }
    if (!voice.is_ready()) {
        fprintf(stderr, "TestToSpeech: voice model is not ready\n");
        return false;
    }
    const float temp = options.temperature >= 0.0f ? options.temperature : config_.temperature;
    const int max_tokens = options.max_tokens > 0 ? options.max_tokens : config_.max_tokens;
    const std::vector<int32_t> prompt = I.prompt_tokens(text);
    if (prompt.empty()) {
        fprintf(stderr, "TestToSpeech: tokenization failed\n");
        return false;
    }
    constexpr int kCheck = mio::StreamPolicy::kCheckInterval;
    mio::StreamPolicy policy;
    size_t &committed = policy.committed;
    std::string generated;
    bool ok = true;

    auto maybe_emit = [&](bool final_) -> bool {
        const std::vector<int> codes = parse_speech_tokens(generated);
        if (codes.empty()) return !final_;
        size_t target = 0;
        if (!policy.plan(codes.size(), final_, &target))
            return (final_ && target <= committed) ? call(nullptr, 0, true) : true;
        int len = 0;
        if (!I.decode_codes_dev(voice, codes, &len, &profile.codec_sec, &profile.istft_sec, true, I.cstream))
            return false;
        profile.decode_calls++;
        profile.decoded_codes += codes.size();
        if (int reused = 0; mio_hip_codec_last_reused(I.codec->codec, &reused) == MIO_OK)
            profile.prenet_rows_reused += (size_t)reused;
        const double per_code = (double)len / (double)codes.size();
        const size_t b = (size_t)std::llround((double)committed * per_code);
        const size_t e = std::min((size_t)std::llround((double)target * per_code), (size_t)len);
        if (b >= e) return final_ ? call(nullptr, 0, true) : true;
        // only the samples this check emits leave the device (emit reads audio[b, e) alone)
        std::vector<float> audio(e - b);
        if (hipMemcpyAsync(audio.data(), (const float *)I.d_pcm + b, (e - b) * sizeof(float), hipMemcpyDeviceToHost,
                           I.cstream) != hipSuccess ||
            hipStreamSynchronize(I.cstream) != hipSuccess) {
            fprintf(stderr, "TestToSpeech: PCM copy failed\n");
            return false;
        }
        committed = target;
        return emit(audio, 0, e - b, final_);
    };

    mio::SamplingParams sp;
    sp.temperature = temp, sp.seed = 42, sp.eos0 = I.eos, sp.eos1 = I.im_end;
    I.harness(options, sp);
    const auto tl0 = clk::now();
    if (mio::llm_begin(I.llm, prompt.data(), (int)prompt.size(), max_tokens, sp)) {
        fprintf(stderr, "TestToSpeech: initial decode failed: %s\n", mio::last_error());
        return false;
    }
    profile.llm_sec += secs(tl0, clk::now());
    std::vector<int32_t> toks;
    size_t consumed = 0;
    bool done = false;
    // the codec works on its own stream: each check's re-decode runs beside the LLM's next
    // kCheck steps, which are enqueued before it (same tokens, same emitted samples)
    // MIO_CSTREAM_PRIO=low|normal|high: the codec stream's priority relative to the LLM's
    // (normal) stream, for the scheduling of workgroups when both have work queued
    if (!I.cstream && hipStreamCreateWithPriority(&I.cstream, hipStreamNonBlocking, cstream_priority()) != hipSuccess) {
        fprintf(stderr, "TestToSpeech: codec stream creation failed\n");
        return false;
    }
    // the PCM buffer holds the whole stream from the start: growing it between re-decodes
    // frees the old one, and a free waits for the LLM steps queued beside the re-decode
    // (MIO_STREAM_PRESIZE=0 restores the growth, for A/B)
    const char *presize = getenv("MIO_STREAM_PRESIZE");
    if ((!presize || atoi(presize) != 0) && I.spt > 0 &&
        !I.ensure(I.d_pcm, I.pcm_cap, (size_t)max_tokens * I.spt * sizeof(float) + 64))
        return false;
    if (mio::llm_run(I.llm, kCheck)) {
        fprintf(stderr, "TestToSpeech: decode failed: %s\n", mio::last_error());
        return false;
    }
    while (!done && ok) {
        const auto ta = clk::now();
        // the next kCheck steps are enqueued before the previous ones are checked (llm_poll
        // waits for the oldest outstanding interval): the GPU never waits for this loop
        if (mio::llm_run(I.llm, kCheck) || mio::llm_poll(I.llm, toks, &done)) {
            fprintf(stderr, "TestToSpeech: decode failed: %s\n", mio::last_error());
            ok = false;
            break;
        }
        profile.llm_sec += secs(ta, clk::now());
        // consume in check-interval groups exactly as the per-token loop would
        while (consumed < toks.size() && ok) {
            const size_t upto = std::min(toks.size(), (consumed / kCheck + 1) * kCheck);
            for (; consumed < upto; ++consumed) generated += I.tok.piece(toks[consumed]);
            profile.llm_tokens = (int)consumed;
            if (consumed % kCheck == 0 && !maybe_emit(false)) ok = false;
        }
    }
    if (ok) ok = maybe_emit(true);
    profile.total_sec = secs(t0, clk::now());
    return ok;
}
