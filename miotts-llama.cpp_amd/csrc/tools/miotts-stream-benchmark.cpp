// `miotts-stream-benchmark`: streaming synthesis speed, no playback (drop-in for
// examples/stream-benchmark.cpp:85-167: same flags and `stream_bench.*` stdout keys).
// Extension (parity tests): --dump-stream PREFIX writes the emitted samples (PREFIX.f32),
// the callback chunk sizes (PREFIX.chunks.i64) and the generated codes (PREFIX.codes.i32,
// from a second generate_token_text: the sampler is counter-based, so it repeats the run).
#include <cstdio>

#include "cli_args.h"
#include "token-parser.h"

namespace {
std::string g_dump;

bool write_raw(const std::string &path, const void *p, size_t bytes) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(p, 1, bytes, f) == bytes;
    return std::fclose(f) == 0 && ok;
}
}  // namespace

int main(int argc, char **argv) {
    std::vector<CliFlag> flags = cli_common_flags();
    flags.push_back({{"--chunk-samples"}, true, "Streaming chunk size in samples (default: 4096)",
                     [](CliArgs &a, const std::string &v) { a.chunk_samples = (size_t)std::stoul(v); }});
    flags.push_back({{"--dump-stream"}, true, "Write emitted samples / chunk sizes / codes to PREFIX.* (tests)",
                     [](CliArgs &, const std::string &v) { g_dump = v; }});
    const char *what = "Benchmark streaming TTS processing speed (no playback).";
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
    TestToSpeech::StreamProfile p;
    std::vector<float> emitted;
    std::vector<long long> chunks;
    const bool dump = !g_dump.empty();
    if (!tts.synthesize_stream_profiled(voice, a.prompt,
                                        [&](const float *s, size_t n, int, bool) {
                                            if (dump && s && n) {
                                                emitted.insert(emitted.end(), s, s + n);
                                                chunks.push_back((long long)n);
                                            }
                                            return true;
                                        },
                                        a.chunk_samples, cli_options(a), p)) {
        std::fprintf(stderr, "Error: streaming benchmark failed\n");
        return 1;
    }
    if (dump) {
        std::string text;
        if (!tts.generate_token_text(a.prompt, cli_options(a), text)) {
            std::fprintf(stderr, "Error: generate_token_text failed\n");
            return 1;
        }
        const std::vector<int> codes = parse_speech_tokens(text);
        if (!write_raw(g_dump + ".f32", emitted.data(), emitted.size() * 4) ||
            !write_raw(g_dump + ".chunks.i64", chunks.data(), chunks.size() * 8) ||
            !write_raw(g_dump + ".codes.i32", codes.data(), codes.size() * 4)) {
            std::fprintf(stderr, "Error: cannot write %s.*\n", g_dump.c_str());
            return 1;
        }
    }
    const double audio = p.emitted_samples ? (double)p.emitted_samples / tts.sample_rate() : 0.0;
    const double total = p.total_sec > 1e-9 ? p.total_sec : 1e-9;
    std::printf("stream_bench.total_sec=%.6f\n", p.total_sec);
    std::printf("stream_bench.audio_sec=%.6f\n", audio);
    std::printf("stream_bench.rtf=%.6f\n", audio > 0.0 ? p.total_sec / audio : 0.0);
    std::printf("stream_bench.x_realtime=%.6f\n", p.total_sec > 0.0 ? audio / p.total_sec : 0.0);
    std::printf("stream_bench.llm_tokens=%d\n", p.llm_tokens);
    std::printf("stream_bench.decode_calls=%d\n", p.decode_calls);
    std::printf("stream_bench.decoded_codes=%zu\n", p.decoded_codes);
    std::printf("stream_bench.prenet_rows_reused=%zu\n", p.prenet_rows_reused);
    std::printf("stream_bench.emitted_samples=%zu\n", p.emitted_samples);
    auto stage = [&](const char *k, double v) {
        std::printf("stream_bench.stage.%s=%.6f (%.2f%%)\n", k, v, 100.0 * v / total);
    };
    stage("llm_sec", p.llm_sec);
    stage("codec_sec", p.codec_sec);
    stage("istft_sec", p.istft_sec);
    stage("callback_sec", p.callback_sec);
    return 0;
}
