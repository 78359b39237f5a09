// `miotts-stream-compare`: non-streaming output vs concatenated streaming chunks (drop-in
// for examples/stream-compare.cpp: same flags, WAV outputs and `compare.*` stdout keys).
#include <algorithm>
#include <cmath>
#include <limits>

#include "cli_args.h"
#include "wav-writer.h"

namespace {

struct Err {
    size_t n = 0;
    double mae = 0, rmse = 0, max_abs = 0;
};

Err errors(const std::vector<float> &a, const std::vector<float> &b, size_t a0 = 0, size_t b0 = 0) {
    Err e;
    if (a0 >= a.size() || b0 >= b.size()) return e;
    e.n = std::min(a.size() - a0, b.size() - b0);
    double se = 0;
    for (size_t i = 0; i < e.n; ++i) {
        const double d = (double)a[a0 + i] - (double)b[b0 + i];
        e.mae += std::fabs(d);
        se += d * d;
        e.max_abs = std::max(e.max_abs, std::fabs(d));
    }
    if (e.n) e.mae /= (double)e.n, e.rmse = std::sqrt(se / (double)e.n);
    return e;
}

void print_errors(const char *prefix, const Err &e) {
    if (!e.n) {
        std::printf("%s.error: no overlap samples\n", prefix);
        return;
    }
    std::printf("%s.samples=%zu\n", prefix, e.n);
    std::printf("%s.mae=%.8f\n", prefix, e.mae);
    std::printf("%s.rmse=%.8f\n", prefix, e.rmse);
    std::printf("%s.max_abs=%.8f\n", prefix, e.max_abs);
}

// lag in [-max_lag, max_lag] (>= 1024 overlapping samples) minimising the RMSE of a vs b
int best_lag(const std::vector<float> &a, const std::vector<float> &b, int max_lag) {
    int best = 0;
    double best_rmse = std::numeric_limits<double>::infinity();
    for (int lag = -max_lag; lag <= max_lag; ++lag) {
        const size_t a0 = lag > 0 ? (size_t)lag : 0, b0 = lag < 0 ? (size_t)-lag : 0;
        const Err e = errors(a, b, a0, b0);
        if (e.n >= 1024 && e.rmse < best_rmse) best_rmse = e.rmse, best = lag;
    }
    return best;
}

}  // namespace

int main(int argc, char **argv) {
    std::vector<CliFlag> flags = cli_common_flags();
    flags.push_back({{"--out-offline"}, true, "Output WAV path for non-streaming audio (default: offline.wav)",
                     [](CliArgs &a, const std::string &v) { a.out_offline = v; }});
    flags.push_back({{"--out-stream"}, true, "Output WAV path for stream-concat audio (default: stream_concat.wav)",
                     [](CliArgs &a, const std::string &v) { a.out_stream = v; }});
    flags.push_back({{"--chunk-samples"}, true, "Streaming chunk size in samples (default: 4096)",
                     [](CliArgs &a, const std::string &v) { a.chunk_samples = (size_t)std::stoul(v); }});
    const char *what = "Compare non-streaming output with concatenated streaming chunks.";
    CliArgs a;
    if (!cli_parse(argc, argv, flags, a, what)) {
        cli_usage(argv[0], what, flags);
        return 1;
    }
    const std::string err = cli_check(a);
    if (!err.empty()) {
        std::fprintf(stderr, "Error: %s\n", err.c_str());
        return 1;
    }
    TestToSpeech tts(cli_config(a));
    if (!tts.is_ready()) {
        std::fprintf(stderr, "Error: failed to initialize TestToSpeech\n");
        return 1;
    }
    VoiceModel voice;
    if (!voice.load_from_file(a.voice_path)) {
        std::fprintf(stderr, "Error: failed to load voice model: %s\n", a.voice_path.c_str());
        return 1;
    }
    TestToSpeech::Options opt = cli_options(a);
    opt.apply_peak_normalization = false;
    std::string token_text;
    if (!tts.generate_token_text(a.prompt, opt, token_text)) {
        std::fprintf(stderr, "Error: failed to generate token text\n");
        return 1;
    }
    TestToSpeech::Options dec = opt;
    dec.skip_llm = true;
    std::vector<float> offline, streamed;
    if (!tts.synthesize_to_vector(voice, token_text, offline, dec)) {
        std::fprintf(stderr, "Error: synthesize_to_vector failed\n");
        return 1;
    }
    if (!tts.synthesize_stream(voice, token_text,
                               [&](const float *s, size_t n, int, bool) {
                                   if (s && n) streamed.insert(streamed.end(), s, s + n);
                                   return true;
                               },
                               a.chunk_samples, dec)) {
        std::fprintf(stderr, "Error: synthesize_stream failed\n");
        return 1;
    }
    if (!wav_write(a.out_offline, offline, tts.sample_rate())) {
        std::fprintf(stderr, "Error: failed to write %s\n", a.out_offline.c_str());
        return 1;
    }
    if (!wav_write(a.out_stream, streamed, tts.sample_rate())) {
        std::fprintf(stderr, "Error: failed to write %s\n", a.out_stream.c_str());
        return 1;
    }
    std::printf("offline_samples=%zu\n", offline.size());
    std::printf("stream_samples=%zu\n", streamed.size());
    std::printf("sample_diff=%lld\n", (long long)streamed.size() - (long long)offline.size());
    const Err e = errors(offline, streamed);
    print_errors("compare", e);
    const int lag = best_lag(offline, streamed, 4096);
    std::printf("best_lag_samples=%d\n", lag);
    if (lag != 0) {
        // the reference's "aligned" pass re-measures the same two signals (its apply_lag with
        // pad_front=false returns them unchanged), so the metrics repeat
        std::printf("aligned_metrics:\n");
        print_errors("compare", e);
    }
    return 0;
}
