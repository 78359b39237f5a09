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
    bool f16 = false;  // every tensor of >= 2 dims stored F16 (an F16 GGUF conversion)
    uint64_t seed = 1;
};

// preset 0 = MioCodec-25Hz-44.1kHz shapes, 1 = tiny test codec, 2 / 3 = the
// same with F16 matrices.
SynthCodecCfg synth_codec_preset(int preset);
bool synth_write_codec(const std::string &path, const SynthCodecCfg &cfg);
bool synth_write_voice(const std::string &path, uint64_t seed, int dim = 128);

// Synthetic LLM in llama.cpp GGUF conventions (arch "llama" or "qwen3"), with a
// byte-level "gpt2" vocabulary containing the chat-template specials and the 12,800
// speech tokens <|s_0|>..<|s_12799|> (test-to-speech.cpp:91; miocodec.h:16).
struct SynthLlmCfg {
    const char *name = "tiny";
    const char *arch = "llama";  // "llama" (rope NORM) | "qwen3" (rope NEOX + q/k RMSNorm) | "qwen2"
    int n_embd = 256, n_layer = 2, n_head = 4, n_head_kv = 2, head_dim = 64, n_ff = 512;
    int n_vocab = 13312, n_ctx = 4096;
    float rope_base = 10000.f, rms_eps = 1e-6f, w_std = 0.02f;
    int qtype = 8;   // 8 = all Q8_0; 15 = Q4_K_M mix (Q4_K + Q6_K); 2 = Q4_0; 30 = all BF16
    // llama-quantize's fallback for rows whose length is not a multiple of 256: Q4_K -> Q5_0,
    // Q6_K -> Q8_0 (llama-quant.cpp); Q4_K_M files of the 0.1B model (n_embd 576) carry them
    bool kq_fallback = true;
    bool tied = true;
    bool qkv_bias = false;  // attn_{q,k,v}.bias tensors (qwen2)
    // lfm2: layer i is attention when (i % attn_mod) is in attn_at, else a gated short conv
    int attn_mod = 4, attn_at0 = 2, attn_at1 = -1;
    uint64_t seed = 1;
};
// preset: 0 tiny Q8_0 (llama), 1 tiny Q4_K_M (qwen3), 2 "0.1B" Q8_0, 3 "1.7B" Q4_K_M,
//         4 "2.6B" Q8_0  (shapes sized to the published file sizes, README.md:189-196),
//         5 tiny Q8_0 qwen2 with q/k/v projection biases, 6 "2.6B" Q8_0 as lfm2 (the LFM2-2.6B
//         width, FFN, vocab and GQA; short-conv / attention layer hybrid), 7 tiny Q8_0 lfm2,
//         8 tiny Q4_K_M lfm2, 9 tiny Q4_K_M at the 0.1B width (n_embd 576: q/k/v, O, gate/up and
//         the embedding fall back to Q5_0 / Q8_0 as llama-quantize does), 10 tiny Q4_0,
//         11 tiny BF16 (qwen3), 12 "1.7B" BF16
SynthLlmCfg synth_llm_preset(int preset);
bool synth_write_llm(const std::string &path, const SynthLlmCfg &cfg);
// Token ids of the synthetic vocabulary.
constexpr int kSynthTokStartOfText = 256, kSynthTokImStart = 257, kSynthTokImEnd = 258,
              kSynthTokEndOfText = 259, kSynthTokSpeech0 = 260, kSynthNumSpeech = 12800;

// Deterministic N(0,1) stream: element i of stream `key` (order-independent).
float synth_normal(uint64_t key, uint64_t i);
// Fast approximate N(0,1) (Irwin-Hall, 4 uniforms from one hash) for large LLM tensors.
float synth_normal_fast(uint64_t key, uint64_t i);
uint64_t synth_key(uint64_t seed, const std::string &name);

}  // namespace mio
