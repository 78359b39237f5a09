// Synthetic codec / voice GGUF generators (see synth.h).
#include "synth.h"

#include <cmath>
#include <cstring>
#include <functional>
#include <vector>

#include "common.h"
#include "gguf.h"

namespace mio {

static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint64_t synth_key(uint64_t seed, const std::string &name) {
    uint64_t h = 1469598103934665603ull ^ splitmix64(seed);
    for (unsigned char c : name) h = (h ^ c) * 1099511628211ull;
    return splitmix64(h);
}

float synth_normal(uint64_t key, uint64_t i) {
    const uint64_t h = splitmix64(key ^ splitmix64(i + 0x632BE59BD9B4E019ull));
    const double u1 = ((h >> 40) + 0.5) * (1.0 / 16777216.0);          // (0,1)
    const double u2 = ((h & 0xFFFFFFull) + 0.5) * (1.0 / 16777216.0);  // (0,1)
    return (float)(std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2));
}

SynthCodecCfg synth_codec_preset(int preset) {
    SynthCodecCfg c;
    c.f16 = preset >= 2;
    if (preset == 1 || preset == 2) {  // tiny: same topology, small widths (fast parity tests)
        c.prenet_layers = 2, c.prenet_dim = 128, c.prenet_heads = 2, c.prenet_ff = 256;
        c.dec_layers = 2, c.dec_dim = 128, c.dec_heads = 2, c.dec_ff = 384;
        c.up_ch[0] = 64, c.up_ch[1] = 32;
        c.resnet_groups = 8;
    }
    return c;
}

namespace {

enum Init { NORMAL, ONES_JITTER, BIAS };

struct Spec {
    std::string name;
    uint32_t type;
    std::vector<int64_t> ne;
    Init init;
    float std;
    std::vector<int32_t> ints;  // for I32 tensors
};

}  // namespace

bool synth_write_codec(const std::string &path, const SynthCodecCfg &c) {
    std::vector<Spec> S;
    auto lin = [&](const std::string &n, int in, int out, float gain = 1.0f) {
        S.push_back({n, GGML_F32, {in, out}, NORMAL, gain / std::sqrt((float)in), {}});
    };
    auto vec = [&](const std::string &n, int d, Init init, float std = 0.02f) {
        S.push_back({n, GGML_F32, {d}, init, std, {}});
    };
    auto conv = [&](const std::string &n, int k, int cin, int cout, float gain) {
        S.push_back({n, GGML_F32, {k, cin, cout}, NORMAL, gain / std::sqrt((float)(k * cin)), {}});
    };
    auto resnet = [&](const std::string &p, int ch) {
        vec(p + "norm1.weight", ch, ONES_JITTER, 0.1f);
        vec(p + "norm1.bias", ch, BIAS, 0.05f);
        conv(p + "conv1.weight", 3, ch, ch, 1.0f);
        vec(p + "conv1.bias", ch, BIAS, 0.02f);
        vec(p + "norm2.weight", ch, ONES_JITTER, 0.1f);
        vec(p + "norm2.bias", ch, BIAS, 0.05f);
        conv(p + "conv2.weight", 3, ch, ch, 0.5f);
        vec(p + "conv2.bias", ch, BIAS, 0.02f);
    };
    const int D = c.prenet_dim, Dd = c.dec_dim;
    S.push_back({"token_embd", GGML_F32, {D, c.n_codes}, NORMAL, 0.5f, {}});
    for (int i = 0; i < c.prenet_layers; ++i) {
        std::string p = "wave_prenet.blk." + std::to_string(i) + ".";
        vec(p + "attn_norm.weight", D, ONES_JITTER, 0.1f);
        vec(p + "attn_norm.bias", D, BIAS);
        lin(p + "attn_q.weight", D, D);
        lin(p + "attn_k.weight", D, D);
        lin(p + "attn_v.weight", D, D);
        lin(p + "attn_output.weight", D, D, 0.5f);
        vec(p + "ffn_norm.weight", D, ONES_JITTER, 0.1f);
        vec(p + "ffn_norm.bias", D, BIAS);
        lin(p + "ffn_gate.weight", D, c.prenet_ff);
        lin(p + "ffn_up.weight", D, c.prenet_ff);
        lin(p + "ffn_down.weight", c.prenet_ff, D, 0.5f);
    }
    vec("wave_prenet.norm.weight", D, ONES_JITTER, 0.1f);
    vec("wave_prenet.norm.bias", D, BIAS);
    lin("wave_prenet.output.weight", D, Dd);
    vec("wave_prenet.output.bias", Dd, BIAS);
    S.push_back({"wave_upsample.weight", GGML_F32, {2, Dd, Dd}, NORMAL, 1.0f / std::sqrt((float)Dd), {}});
    vec("wave_upsample.bias", Dd, BIAS);
    for (int b = 0; b < c.resnet_blocks; ++b) resnet("wave_prior." + std::to_string(b) + ".", Dd);
    for (int i = 0; i < c.dec_layers; ++i) {
        std::string p = "wave_decoder.blk." + std::to_string(i) + ".";
        lin(p + "attn_cond.weight", c.adaln_dim, 3 * Dd, 0.3f);
        vec(p + "attn_cond.bias", 3 * Dd, BIAS, 0.05f);
        lin(p + "ffn_cond.weight", c.adaln_dim, 3 * Dd, 0.3f);
        vec(p + "ffn_cond.bias", 3 * Dd, BIAS, 0.05f);
        lin(p + "attn_q.weight", Dd, Dd);
        lin(p + "attn_k.weight", Dd, Dd);
        lin(p + "attn_v.weight", Dd, Dd);
        lin(p + "attn_output.weight", Dd, Dd, 0.5f);
        lin(p + "ffn_gate.weight", Dd, c.dec_ff);
        lin(p + "ffn_up.weight", Dd, c.dec_ff);
        lin(p + "ffn_down.weight", c.dec_ff, Dd, 0.5f);
    }
    lin("wave_decoder.norm_cond.weight", c.adaln_dim, 2 * Dd, 0.3f);
    vec("wave_decoder.norm_cond.bias", 2 * Dd, BIAS, 0.05f);
    for (int b = 0; b < c.resnet_blocks; ++b) resnet("wave_post." + std::to_string(b) + ".", Dd);
    int cin = Dd;
    for (int s = 0; s < c.up_stages; ++s) {
        const int cout = c.up_ch[s], k = c.kernels[s], f = c.factors[s];
        const std::string ss = std::to_string(s);
        S.push_back({"wave_upsampler.up." + ss + ".weight", GGML_F32, {k, cout, cin}, NORMAL,
                     1.0f / std::sqrt((float)cin * k / f), {}});
        vec("wave_upsampler.up." + ss + ".bias", cout, BIAS);
        vec("wave_upsampler.snake." + ss + ".alpha", cout, BIAS, 0.2f);
        vec("wave_upsampler.snake." + ss + ".beta", cout, BIAS, 0.2f);
        resnet("wave_upsampler.resblk." + ss + ".", cout);
        cin = cout;
    }
    lin("wave_upsampler.out_proj.weight", cin, Dd);
    vec("wave_upsampler.out_proj.bias", Dd, BIAS);
    vec("wave_upsampler.out_snake.alpha", Dd, BIAS, 0.2f);
    vec("wave_upsampler.out_snake.beta", Dd, BIAS, 0.2f);
    const int n_freq = c.n_fft / 2 + 1;
    lin("istft_head.out.weight", Dd, 2 * n_freq, 0.7f);
    vec("istft_head.out.bias", 2 * n_freq, BIAS, 0.1f);
    S.push_back({"miocodec.wave_upsampler.factors", GGML_I32, {c.up_stages}, BIAS, 0,
                 {c.factors[0], c.factors[1]}});
    S.push_back({"miocodec.wave_upsampler.kernel_sizes", GGML_I32, {c.up_stages}, BIAS, 0,
                 {c.kernels[0], c.kernels[1]}});

    GgufWriter w;
    w.kv_str("general.architecture", "miocodec");
    w.kv_str("general.name", "synthetic-miocodec");
    w.kv_u32("miocodec.sample_rate", c.sample_rate);
    w.kv_u32("miocodec.n_fft", c.n_fft);
    w.kv_u32("miocodec.hop_length", c.hop);
    int up_total = 2;
    for (int s = 0; s < c.up_stages; ++s) up_total *= c.factors[s];
    w.kv_u32("miocodec.samples_per_token", up_total * c.hop);
    w.kv_u32("embedding_length_out", 2 * n_freq);
    w.kv_u32("miocodec.prenet_layers", c.prenet_layers);
    w.kv_u32("miocodec.prenet_dim", c.prenet_dim);
    w.kv_u32("miocodec.prenet_heads", c.prenet_heads);
    w.kv_u32("miocodec.prenet_ff", c.prenet_ff);
    w.kv_u32("miocodec.prenet_window", c.prenet_window);
    w.kv_u32("miocodec.decoder_layers", c.dec_layers);
    w.kv_u32("miocodec.decoder_dim", c.dec_dim);
    w.kv_u32("miocodec.decoder_heads", c.dec_heads);
    w.kv_u32("miocodec.decoder_ff", c.dec_ff);
    w.kv_u32("miocodec.decoder_window", c.dec_window);
    w.kv_u32("miocodec.decoder_adanorm_dim", c.adaln_dim);
    w.kv_u32("miocodec.resnet_blocks", c.resnet_blocks);
    w.kv_u32("miocodec.resnet_groups", c.resnet_groups);
    w.kv_u32("miocodec.wave_upsampler_layers", c.up_stages);
    w.kv_f32("miocodec.rope_theta", 10000.0f);
    w.kv_f32("miocodec.norm_eps", 1e-5f);
    w.kv_f32("miocodec.group_norm_eps", 1e-6f);
    if (c.f16)
        for (auto &s : S)
            if (s.type == GGML_F32 && s.ne.size() >= 2) s.type = GGML_F16;
    for (auto &s : S) w.add_tensor(s.name, s.type, s.ne);
    return w.write(path, [&](size_t i, uint8_t *dst, size_t nbytes) {
        const Spec &s = S[i];
        if (s.type == GGML_I32) {
            std::memcpy(dst, s.ints.data(), nbytes);
            return;
        }
        const bool h = s.type == GGML_F16;
        const size_t n = nbytes / (h ? 2 : 4);
        const uint64_t key = synth_key(c.seed, s.name);
#pragma omp parallel for schedule(static) if (n > 65536)
        for (size_t j = 0; j < n; ++j) {
            const float z = synth_normal(key, j);
            const float v = s.init == ONES_JITTER ? 1.0f + s.std * z : s.std * z;
            if (h)
                ((_Float16 *)dst)[j] = (_Float16)v;
            else
                ((float *)dst)[j] = v;
        }
    });
}

bool synth_write_voice(const std::string &path, uint64_t seed, int dim) {
    GgufWriter w;
    w.kv_str("general.architecture", "mio-embedding");
    w.kv_u32("mio.embedding.dim", dim);
    w.add_tensor("mio.global_embedding", GGML_F32, {dim});
    const uint64_t key = synth_key(seed, "voice");
    return w.write(path, [&](size_t, uint8_t *dst, size_t nbytes) {
        float *f = (float *)dst;
        for (size_t j = 0; j < nbytes / 4; ++j) f[j] = synth_normal(key, j);
    });
}

}  // namespace mio
