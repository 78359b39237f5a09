// Parity helper for the drop-in C++ surface: runs miocodec_decode (miocodec.h) and
// istft (istft.h) exactly as TestToSpeech::decode_tokens_to_audio does
// (test-to-speech.cpp:210-230) and writes the raw f32 results for tests/test_cli_gpu.py.
//   miotts-api-dump CODEC.gguf VOICE.emb.gguf CODES.i32 OUT_SPEC.f32 OUT_PCM.f32
#include <cstdio>
#include <fstream>
#include <vector>

#include "istft.h"
#include "miocodec.h"

int main(int argc, char **argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s codec.gguf voice.emb.gguf codes.i32 spec.f32 pcm.f32\n", argv[0]);
        return 2;
    }
    std::vector<int> codes;
    std::ifstream g(argv[3], std::ios::binary | std::ios::ate);
    const size_t nbytes = (size_t)g.tellg();
    g.seekg(0);
    codes.assign(nbytes / 4, 0);
    g.read(reinterpret_cast<char *>(codes.data()), (std::streamsize)nbytes);
    miocodec_context *ctx = miocodec_load(argv[1]);
    const std::vector<float> emb = load_voice_embedding(argv[2]);
    if (!ctx || emb.empty() || codes.empty()) return 1;
    int frames = 0;
    const std::vector<float> spec = miocodec_decode(ctx, codes.data(), (int)codes.size(), emb.data(), 0, &frames);
    if (spec.empty()) return 1;
    istft_cache cache(miocodec_n_fft(ctx), miocodec_n_fft(ctx));
    const std::vector<float> pcm = istft(spec.data(), frames, miocodec_hop_length(ctx), cache);
    if (pcm.empty()) return 1;
    std::ofstream(argv[4], std::ios::binary).write(reinterpret_cast<const char *>(spec.data()), spec.size() * 4);
    std::ofstream(argv[5], std::ios::binary).write(reinterpret_cast<const char *>(pcm.data()), pcm.size() * 4);
    std::printf("frames=%d samples=%zu sample_rate=%d spt=%d\n", frames, pcm.size(), miocodec_sample_rate(ctx),
                miocodec_samples_per_token(ctx));
    miocodec_free(ctx);
    return 0;
}
