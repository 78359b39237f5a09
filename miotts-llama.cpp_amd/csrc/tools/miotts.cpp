// `miotts`: offline synthesis to a WAV file on one MI355X (drop-in for the reference CLI,
// main.cpp:91-151: same flags, checks, exit codes and messages).
// Extensions: --batch FILE synthesizes one prompt per line, their LLM
// decodes together (TestToSpeech::synthesize_batch_to_files), into OUTPUT_000.wav,
// OUTPUT_001.wav, ...; --gpus N shards those lines over N MI355Xs (one thread and one
// TestToSpeech per device, line i on device i % N; utterances are independent, no collective).
#include <fstream>
#include <thread>

#include "cli_args.h"
#include "miocodec.h"

static std::string numbered(const std::string &path, size_t i) {
    const size_t dot = path.rfind('.');
    const size_t slash = path.find_last_of('/');
    const bool ext = dot != std::string::npos && (slash == std::string::npos || dot > slash);
    char n[16];
    std::snprintf(n, sizeof(n), "_%03zu", i);
    return ext ? path.substr(0, dot) + n + path.substr(dot) : path + n;
}

static int run_batch(const CliArgs &a, const std::vector<std::string> &lines) {
    const int ng = a.gpus < 1 ? 1 : a.gpus;
    const int dev0 = a.device < 0 ? 0 : a.device;
    std::vector<int> rc((size_t)ng, 0);
    auto shard = [&](int g) {
        std::vector<std::string> texts, paths;
        for (size_t i = (size_t)g; i < lines.size(); i += (size_t)ng) {
            texts.push_back(lines[i]);
            paths.push_back(numbered(a.output_path, i));
        }
        if (texts.empty()) return;
        TestToSpeech::Config c = cli_config(a);
        c.device = dev0 + g;
        TestToSpeech tts(c);
        if (!tts.is_ready()) {
            std::fprintf(stderr, "Error: failed to initialize TestToSpeech on device %d\n", c.device);
            rc[(size_t)g] = 1;
            return;
        }
        VoiceModel voice;
        if (!voice.load_from_file(a.voice_path)) {
            std::fprintf(stderr, "Error: failed to load voice model: %s\n", a.voice_path.c_str());
            rc[(size_t)g] = 1;
            return;
        }
        if (!tts.synthesize_batch_to_files(voice, texts, paths, cli_options(a))) {
            std::fprintf(stderr, "Error: synthesis failed on device %d\n", c.device);
            rc[(size_t)g] = 1;
            return;
        }
        for (const std::string &p : paths) std::fprintf(stderr, "Saved: %s\n", p.c_str());
    };
    if (ng == 1) {
        shard(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < ng; ++g) th.emplace_back(shard, g);
        for (std::thread &t : th) t.join();
    }
    for (int r : rc)
        if (r) return 1;
    return 0;
}

int main(int argc, char **argv) {
    std::vector<CliFlag> flags = cli_common_flags();
    flags.push_back({{"-o", "--output"}, true, "Output WAV file path (default: output.wav)",
                     [](CliArgs &a, const std::string &v) { a.output_path = v; }});
    flags.push_back({{"--dump-tensors"}, false, "Print MioCodec tensor names and exit",
                     [](CliArgs &a, const std::string &) { a.dump_tensors = true; }});
    flags.push_back({{"--batch"}, true, "Synthesize every line of this file (OUTPUT_000.wav, ...), decoded together",
                     [](CliArgs &a, const std::string &v) { a.batch_file = v; }});
    flags.push_back({{"--gpus"}, true, "Shard the --batch lines over this many MI355Xs (default: 1)",
                     [](CliArgs &a, const std::string &v) { a.gpus = std::stoi(v); }});
    CliArgs a;
    if (!cli_parse(argc, argv, flags, a, "")) {
        cli_usage(argv[0], "", flags);
        return 1;
    }
    if (a.dump_tensors) {
        if (a.codec_path.empty()) {
            std::fprintf(stderr, "Error: --codec path required for --dump-tensors\n");
            return 1;
        }
        miocodec_print_tensors(a.codec_path);
        return 0;
    }
    std::vector<std::string> lines;
    if (!a.batch_file.empty()) {
        std::ifstream f(a.batch_file);
        if (!f) {
            std::fprintf(stderr, "Error: cannot read --batch file: %s\n", a.batch_file.c_str());
            return 1;
        }
        for (std::string l; std::getline(f, l);) {
            if (!l.empty() && l.back() == '\r') l.pop_back();
            if (!l.empty()) lines.push_back(l);
        }
        if (lines.empty()) {
            std::fprintf(stderr, "Error: --batch file has no prompts: %s\n", a.batch_file.c_str());
            return 1;
        }
        if (a.prompt.empty()) a.prompt = lines[0];  // the reference checks below need one
    } else if (a.gpus != 1) {
        std::fprintf(stderr, "Error: --gpus needs --batch\n");
        return 1;
    }
    const std::string err = cli_check(a, true);
    if (!err.empty()) {
        std::fprintf(stderr, "Error: %s\n", err.c_str());
        return 1;
    }
    if (!lines.empty()) return run_batch(a, lines);
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
    if (!tts.synthesize_to_file(voice, a.prompt, a.output_path, cli_options(a))) {
        std::fprintf(stderr, "Error: synthesis failed\n");
        return 1;
    }
    std::fprintf(stderr, "Saved: %s\n", a.output_path.c_str());
    return 0;
}
