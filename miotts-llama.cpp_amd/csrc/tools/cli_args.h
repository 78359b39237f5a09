// Shared flag parsing of the MI355X CLIs. The flag set, defaults and help text follow the
// reference tools (main.cpp:24-89, examples/stream-benchmark.cpp:20-83,
// examples/stream-compare.cpp:27-98).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "test-to-speech.h"

struct CliArgs {
    std::string model_path, codec_path, voice_path, prompt;
    std::string output_path = "output.wav";
    std::string out_offline = "offline.wav", out_stream = "stream_concat.wav";
    std::string batch_file;  // miotts --batch: one prompt per line
    int gpus = 1;            // miotts --gpus: MI355Xs the batch is sharded over
    float temperature = 0.8f;
    int max_tokens = 700, n_threads = 4, n_gpu_layers = 0, device = -1;
    size_t chunk_samples = 4096;
    bool skip_llm = false, dump_tensors = false, speech_only = false, ignore_eos = false;
};

struct CliFlag {
    std::vector<std::string> names;
    bool takes_value;
    const char *help;
    std::function<void(CliArgs &, const std::string &)> set;
};

inline std::vector<CliFlag> cli_common_flags() {
    return {
        {{"-m", "--model"}, true, "MioTTS LLM GGUF model path (required unless --skip-llm)",
         [](CliArgs &a, const std::string &v) { a.model_path = v; }},
        {{"-c", "--codec"}, true, "MioCodec GGUF model path (required)",
         [](CliArgs &a, const std::string &v) { a.codec_path = v; }},
        {{"-v", "--voice"}, true, "Voice embedding .emb.gguf path (required)",
         [](CliArgs &a, const std::string &v) { a.voice_path = v; }},
        {{"-p", "--prompt"}, true, "Text to synthesize (required)",
         [](CliArgs &a, const std::string &v) { a.prompt = v; }},
        {{"-t", "--temp"}, true, "Sampling temperature (default: 0.8)",
         [](CliArgs &a, const std::string &v) { a.temperature = std::stof(v); }},
        {{"--max-tokens"}, true, "Max tokens to generate (default: 700)",
         [](CliArgs &a, const std::string &v) { a.max_tokens = std::stoi(v); }},
        {{"--threads"}, true, "Number of CPU threads (default: 4; accepted, unused: the path runs on the GPU)",
         [](CliArgs &a, const std::string &v) { a.n_threads = std::stoi(v); }},
        {{"-ngl"}, true, "Number of GPU layers (default: 0; accepted, unused: every layer runs on the GPU)",
         [](CliArgs &a, const std::string &v) { a.n_gpu_layers = std::stoi(v); }},
        {{"--device"}, true, "MI355X index (default: MIO_DEVICE, else LOCAL_RANK, else 0)",
         [](CliArgs &a, const std::string &v) { a.device = std::stoi(v); }},
        {{"--skip-llm"}, false, "Treat --prompt as raw <|s_N|> token text",
         [](CliArgs &a, const std::string &) { a.skip_llm = true; }},
        {{"--speech-only"}, false, "Benchmark harness: sample only the <|s_N|> speech ids",
         [](CliArgs &a, const std::string &) { a.speech_only = true; }},
        {{"--ignore-eos"}, false, "Benchmark harness: do not stop at <|endoftext|> / <|im_end|>",
         [](CliArgs &a, const std::string &) { a.ignore_eos = true; }},
    };
}

inline void cli_usage(const char *prog, const char *what, const std::vector<CliFlag> &flags) {
    std::fprintf(stderr, "Usage: %s [options]\n\n%s%sOptions:\n", prog, what, *what ? "\n\n" : "");
    for (const CliFlag &f : flags) {
        std::string n;
        for (const std::string &s : f.names) n += (n.empty() ? "" : ", ") + s;
        if (f.takes_value) n += f.names.back() == "-ngl" || f.names.back().rfind("--", 0) != 0 ? " N" : " VALUE";
        std::fprintf(stderr, "  %-24s %s\n", n.c_str(), f.help);
    }
    std::fprintf(stderr, "  %-24s %s\n\n", "-h, --help", "Show this help");
}

// false on an unknown flag or a missing value (the reference prints usage and exits 1)
inline bool cli_parse(int argc, char **argv, const std::vector<CliFlag> &flags, CliArgs &a, const char *what) {
    for (int i = 1; i < argc; ++i) {
        const std::string arg = argv[i];
        if (arg == "-h" || arg == "--help") {
            cli_usage(argv[0], what, flags);
            std::exit(0);
        }
        const CliFlag *hit = nullptr;
        for (const CliFlag &f : flags)
            for (const std::string &n : f.names)
                if (n == arg) hit = &f;
        if (!hit) {
            std::fprintf(stderr, "Unknown argument: %s\n", arg.c_str());
            return false;
        }
        if (hit->takes_value && ++i >= argc) return false;
        hit->set(a, hit->takes_value ? std::string(argv[i]) : std::string());
    }
    return true;
}

// the reference tools' required-argument checks; returns an error text or empty.
// path_words: main.cpp:109-121 says "--codec path is required" where the examples
// (stream-benchmark.cpp:93-105, stream-compare.cpp:174-186) say "--codec is required".
inline std::string cli_check(const CliArgs &a, bool path_words = false) {
    const std::string p = path_words ? " path" : "";
    if (a.prompt.empty()) return "--prompt is required";
    if (a.codec_path.empty()) return "--codec" + p + " is required";
    if (a.voice_path.empty()) return "--voice" + p + " is required";
    if (!a.skip_llm && a.model_path.empty()) return "--model" + p + " is required (or use --skip-llm)";
    return "";
}

inline TestToSpeech::Config cli_config(const CliArgs &a) {
    TestToSpeech::Config c;
    c.model_path = a.model_path;
    c.codec_path = a.codec_path;
    c.n_threads = a.n_threads;
    c.n_gpu_layers = a.n_gpu_layers;
    c.temperature = a.temperature;
    c.max_tokens = a.max_tokens;
    c.device = a.device;
    return c;
}

inline TestToSpeech::Options cli_options(const CliArgs &a) {
    TestToSpeech::Options o;
    o.temperature = a.temperature;
    o.max_tokens = a.max_tokens;
    o.skip_llm = a.skip_llm;
    o.speech_only = a.speech_only;
    o.ignore_eos = a.ignore_eos;
    return o;
}
