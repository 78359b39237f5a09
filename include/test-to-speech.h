// Drop-in for the reference test-to-speech.h (test-to-speech.h:11-123): the same classes,
// nested types, defaults and member functions, so callers (main.cpp, the stream examples,
// stream-to-device) compile unchanged. The implementation (csrc/host/tts.cpp) runs the
// whole path on one MI355X: GGUF tokenizer on the host, the LLM decode step as one
// hipGraph per token with on-device sampling, the MioCodec decoder and the fused iSTFT.
// Config::n_threads / n_gpu_layers are accepted and ignored (everything runs on the GPU);
// Config::device (extension, default -1) picks the GPU (-1: MIO_DEVICE, else LOCAL_RANK,
// else 0).
#pragma once

#include <cstddef>
#include <functional>
#include <memory>
#include <string>
#include <vector>

class istft_cache;

class VoiceModel {
public:
    VoiceModel() = default;

    bool load_from_file(const std::string & path);
    bool is_ready() const;

    const std::vector<float> & embedding() const;
    const std::string & path() const;

private:
    std::string path_;
    std::vector<float> embedding_;
};

class TestToSpeech {
public:
    struct StreamProfile {
        double total_sec = 0.0;
        double llm_sec = 0.0;
        double codec_sec = 0.0;
        double istft_sec = 0.0;
        double callback_sec = 0.0;
        int llm_tokens = 0;
        int decode_calls = 0;
        size_t decoded_codes = 0;
        size_t emitted_samples = 0;
        // (extension) codes whose prenet rows a re-decode took from the previous decode
        // (MIO_CODEC_INCREMENTAL) instead of recomputing them
        size_t prenet_rows_reused = 0;
    };

    struct Config {
        std::string model_path;
        std::string codec_path;
        int n_threads = 4;
        int n_gpu_layers = 0;
        float temperature = 0.8f;
        int max_tokens = 700;
        int device = -1;  // extension: GPU index (-1 = MIO_DEVICE / LOCAL_RANK / 0)
    };

    struct Options {
        float temperature = -1.0f; // negative => use Config default
        int max_tokens = -1;       // negative => use Config default
        bool skip_llm = false;     // when true, text is raw <|s_N|> token text
        bool apply_peak_normalization = true;
        // extensions for benchmark harnesses (flagged deviations): sample only the 12,800
        // speech ids / never stop at an end token
        bool speech_only = false;
        bool ignore_eos = false;
    };

    using StreamCallback = std::function<bool(const float * samples,
                                              size_t n_samples,
                                              int sample_rate,
                                              bool is_last_chunk)>;

    explicit TestToSpeech(const Config & config);
    ~TestToSpeech();

    TestToSpeech(const TestToSpeech &) = delete;
    TestToSpeech & operator=(const TestToSpeech &) = delete;

    bool is_ready() const;
    int sample_rate() const;

    bool synthesize_to_file(const VoiceModel & voice,
                            const std::string & text,
                            const std::string & output_path,
                            const Options & options);
    bool synthesize_to_file(const VoiceModel & voice,
                            const std::string & text,
                            const std::string & output_path);

    bool synthesize_to_vector(const VoiceModel & voice,
                              const std::string & text,
                              std::vector<float> & out_audio,
                              const Options & options);
    bool synthesize_to_vector(const VoiceModel & voice,
                              const std::string & text,
                              std::vector<float> & out_audio);

    bool synthesize_stream(const VoiceModel & voice,
                           const std::string & text,
                           const StreamCallback & callback,
                           size_t chunk_samples,
                           const Options & options);
    bool synthesize_stream(const VoiceModel & voice,
                           const std::string & text,
                           const StreamCallback & callback,
                           size_t chunk_samples = 4096);
    bool synthesize_stream_profiled(const VoiceModel & voice,
                                    const std::string & text,
                                    const StreamCallback & callback,
                                    size_t chunk_samples,
                                    const Options & options,
                                    StreamProfile & profile);
    bool generate_token_text(const std::string & text,
                             const Options & options,
                             std::string & out_token_text);

    // (extension) several utterances on this device: their LLM decodes run together (one
    // weight pass per step for all of them, mio_hip_llm_generate_batch, up to 16 at a time),
    // then each is written as synthesize_to_file writes it (the same bytes: every utterance
    // samples with the seed synthesize_to_file uses)
    bool synthesize_batch_to_files(const VoiceModel & voice,
                                   const std::vector<std::string> & texts,
                                   const std::vector<std::string> & output_paths,
                                   const Options & options);

    struct Impl;  // GPU handles (device, LLM runner, codec, tokenizer)

private:
    Config config_;
    std::unique_ptr<Impl> impl_;
};
