// Synthetic GGUF generators (no real model files exist offline).
// Files use the reference's tensor names / KV keys (miocodec.cpp:448-481,
// 599-728; create_voice_emb.py:125-129) so the same loaders read them as real files.
#pragma once

#include <cstdint>
#include <string>

namespace mio {

struct SynthCodecCfg {
    int prenet_layers = 6, prenet_dim = 768, prenet_heads = 12, prenet_ff = 2048, prenet_window = 65;
    int dec_layers = 8, dec_dim = 512, dec_heads = 8, dec_ff = 1536, dec_window = 65, adaln_dim = 128;
    int resnet_blocks = 2, resnet_groups = 32, up_stages = 2;
    int factors[2] = {3, 3}, kernels[2] = {7, 7}, up_ch[2] = {256, 128};
    int n_codes = 12800, n_fft = 392, hop = 98, sample_rate = 44100;
    uint64_t seed = 1;
};

// preset 0 = MioCodec-25Hz-44.1kHz shapes, 1 = tiny test codec.
SynthCodecCfg synth_codec_preset(int preset);
bool synth_write_codec(const std::string &path, const SynthCodecCfg &cfg);
bool synth_write_voice(const std::string &path, uint64_t seed, int dim = 128);

// Deterministic N(0,1) stream: element i of stream `key` (order-independent).
float synth_normal(uint64_t key, uint64_t i);
uint64_t synth_key(uint64_t seed, const std::string &name);

}  // namespace mio
