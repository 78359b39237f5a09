// `miotts`: offline synthesis to a WAV file on one MI355X (drop-in for the reference CLI,
// main.cpp:91-151: same flags, checks, exit codes and messages).
#include "cli_args.h"
#include "miocodec.h"

int main(int argc, char **argv) {
    std::vector<CliFlag> flags = cli_common_flags();
    flags.push_back({{"-o", "--output"}, true, "Output WAV file path (default: output.wav)",
                     [](CliArgs &a, const std::string &v) { a.output_path = v; }});
    flags.push_back({{"--dump-tensors"}, false, "Print MioCodec tensor names and exit",
                     [](CliArgs &a, const std::string &) { a.dump_tensors = true; }});
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
    const std::string err = cli_check(a, true);
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
    if (!tts.synthesize_to_file(voice, a.prompt, a.output_path, cli_options(a))) {
        std::fprintf(stderr, "Error: synthesis failed\n");
        return 1;
    }
    std::fprintf(stderr, "Saved: %s\n", a.output_path.c_str());
    return 0;
}
