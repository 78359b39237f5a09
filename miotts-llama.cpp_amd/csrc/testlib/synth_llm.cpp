// Synthetic LLM GGUF writer (see synth.h). Tensor names / KV keys follow llama.cpp's
// GGUF conventions; quant types follow llama.cpp's Q4_K_M recipe: Q4_K everywhere,
// Q6_K for attn_v / ffn_down on "use_more_bits" layers and for the (tied) output.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "gguf.h"
#include "quant.h"
#include "synth.h"

namespace mio {

static inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

float synth_normal_fast(uint64_t key, uint64_t i) {
    const uint64_t h = mix64(key ^ mix64(i));
    const float s = (float)(h & 0xFFFF) + (float)((h >> 16) & 0xFFFF) + (float)((h >> 32) & 0xFFFF) +
                    (float)(h >> 48);
    return (s * (1.0f / 65536.0f) - 2.0f) * 1.7320508f;  // var(sum of 4 U(0,1)) = 1/3
}

SynthLlmCfg synth_llm_preset(int p) {
    SynthLlmCfg c;
    switch (p) {
        case 0: break;
        case 1:
            c.name = "tiny-q4km", c.arch = "qwen3", c.n_layer = 3, c.n_ff = 768, c.qtype = 15;
            c.rope_base = 1000000.f;
            break;
        case 2:
            c.name = "MioTTS-0.1B-synthetic", c.n_embd = 576, c.n_layer = 24, c.n_head = 9,
            c.n_head_kv = 3, c.head_dim = 64, c.n_ff = 1536, c.n_vocab = 49152 + 12800;
            break;
        case 3:
            c.name = "MioTTS-1.7B-synthetic", c.arch = "qwen3", c.n_embd = 2048, c.n_layer = 28,
            c.n_head = 16, c.n_head_kv = 8, c.head_dim = 128, c.n_ff = 6144,
            c.n_vocab = 151936 + 12800, c.qtype = 15, c.rope_base = 1000000.f;
            break;
        case 5:
            c.name = "tiny-qwen2-bias", c.arch = "qwen2", c.qkv_bias = true, c.rope_base = 1000000.f;
            break;
        case 4:
            c.name = "MioTTS-2.6B-synthetic", c.n_embd = 2048, c.n_layer = 32, c.n_head = 32,
            c.n_head_kv = 8, c.head_dim = 64, c.n_ff = 10752, c.n_vocab = 65536 + 12800;
            break;
        case 6:  // LFM2-2.6B shape: 30 layers, attention on 8 of them (i % 4 == 2, and 29)
            c.name = "MioTTS-2.6B-lfm2-synthetic", c.arch = "lfm2", c.n_embd = 2048, c.n_layer = 30,
            c.n_head = 32, c.n_head_kv = 8, c.head_dim = 64, c.n_ff = 10752, c.n_vocab = 65536 + 12800;
            c.rope_base = 1000000.f, c.rms_eps = 1e-5f, c.attn_mod = 4, c.attn_at0 = 2, c.attn_at1 = -1;
            break;
        case 7:
            c.name = "tiny-lfm2", c.arch = "lfm2", c.n_layer = 5, c.attn_mod = 3, c.attn_at0 = 1;
            c.rope_base = 1000000.f, c.rms_eps = 1e-5f;
            break;
        case 8:
            c.name = "tiny-lfm2-q4km", c.arch = "lfm2", c.n_layer = 5, c.attn_mod = 3, c.attn_at0 = 1, c.qtype = 15;
            c.rope_base = 1000000.f, c.rms_eps = 1e-5f;
            break;
        case 9:
            c.name = "tiny-q4km-576", c.arch = "qwen3", c.n_embd = 576, c.n_layer = 3, c.n_head = 9,
            c.n_head_kv = 3, c.head_dim = 64, c.n_ff = 1536, c.qtype = 15, c.rope_base = 1000000.f;
            break;
        case 10:
            c.name = "tiny-q4_0", c.qtype = 2;
            break;
        case 11:
            c.name = "tiny-bf16", c.arch = "qwen3", c.n_layer = 3, c.n_ff = 768, c.qtype = 30;
            c.rope_base = 1000000.f;
            break;
        case 12:  // the 1.7B shape as the published BF16 file (README.md:196)
            c = synth_llm_preset(3);
            c.name = "MioTTS-1.7B-bf16-synthetic", c.qtype = 30;
            break;
        default: break;
    }
    return c;
}

// GPT-2 byte-level unicode for byte b (bytes_to_unicode), UTF-8 encoded
static std::string byte_token(int b) {
    int cp;
    if ((b >= 33 && b <= 126) || (b >= 161 && b <= 172) || (b >= 174 && b <= 255)) {
        cp = b;
    } else {
        int n = 0;
        for (int x = 0; x < b; ++x)
            if (!((x >= 33 && x <= 126) || (x >= 161 && x <= 172) || (x >= 174 && x <= 255))) ++n;
        cp = 256 + n;
    }
    std::string s;
    if (cp < 0x80) {
        s += (char)cp;
    } else {
        s += (char)(0xC0 | (cp >> 6));
        s += (char)(0x80 | (cp & 0x3F));
    }
    return s;
}

static bool use_more_bits(int i, int n) { return i < n / 8 || i >= 7 * n / 8 || (i - n / 8) % 3 == 2; }

bool synth_lfm2_is_attn(const SynthLlmCfg &c, int i) {
    const int r = i % c.attn_mod;
    return r == c.attn_at0 || r == c.attn_at1 || (c.n_layer == 30 && i == 29);
}

bool synth_write_llm(const std::string &path, const SynthLlmCfg &c) {
    GgufWriter w;
    const std::string a = c.arch;
    const bool lfm2 = a == "lfm2";
    w.kv_str("general.architecture", a);
    w.kv_str("general.name", c.name);
    // llama_ftype: 7 MOSTLY_Q8_0, 15 MOSTLY_Q4_K_M, 2 MOSTLY_Q4_0, 32 MOSTLY_BF16
    w.kv_u32("general.file_type", c.qtype == 15 ? 15 : (c.qtype == 2 ? 2 : (c.qtype == 30 ? 32 : 7)));
    w.kv_u32(a + ".context_length", c.n_ctx);
    w.kv_u32(a + ".embedding_length", c.n_embd);
    w.kv_u32(a + ".block_count", c.n_layer);
    w.kv_u32(a + ".feed_forward_length", c.n_ff);
    w.kv_u32(a + ".attention.head_count", c.n_head);
    if (lfm2) {
        // llama.cpp LFM2: head_count_kv per layer, 0 marks a short-conv (recurrent) layer
        std::vector<int32_t> kv;
        for (int i = 0; i < c.n_layer; ++i) kv.push_back(synth_lfm2_is_attn(c, i) ? c.n_head_kv : 0);
        w.kv_arr_i32(a + ".attention.head_count_kv", kv);
        w.kv_u32(a + ".shortconv.l_cache", 3);
    } else {
        w.kv_u32(a + ".attention.head_count_kv", c.n_head_kv);
    }
    w.kv_u32(a + ".attention.key_length", c.head_dim);
    w.kv_u32(a + ".attention.value_length", c.head_dim);
    w.kv_f32(a + ".rope.freq_base", c.rope_base);
    w.kv_f32(a + ".attention.layer_norm_rms_epsilon", c.rms_eps);
    // vocabulary
    std::vector<std::string> toks;
    std::vector<int32_t> types;
    for (int b = 0; b < 256; ++b) toks.push_back(byte_token(b)), types.push_back(1);
    for (const char *sp : {"<|startoftext|>", "<|im_start|>", "<|im_end|>", "<|endoftext|>"})
        toks.push_back(sp), types.push_back(3);
    for (int i = 0; i < kSynthNumSpeech; ++i) toks.push_back("<|s_" + std::to_string(i) + "|>"), types.push_back(4);
    for (int i = (int)toks.size(); i < c.n_vocab; ++i)
        toks.push_back("<|x_" + std::to_string(i) + "|>"), types.push_back(5);
    w.kv_str("tokenizer.ggml.model", "gpt2");
    w.kv_str("tokenizer.ggml.pre", "default");
    w.kv_arr_str("tokenizer.ggml.tokens", toks);
    w.kv_arr_i32("tokenizer.ggml.token_type", types);
    w.kv_arr_str("tokenizer.ggml.merges", {});
    w.kv_u32("tokenizer.ggml.bos_token_id", kSynthTokStartOfText);
    w.kv_u32("tokenizer.ggml.eos_token_id", kSynthTokEndOfText);
    w.kv_bool("tokenizer.ggml.add_bos_token", false);

    struct T {
        std::string name;
        uint32_t type;
        int64_t k, rows;
        int fill;  // 0 quantized N(0, w_std) rows, 1 ones, 2 f32 N(0, 0.5) (biases / conv taps)
    };
    std::vector<T> ts;
    auto pick = [&](uint32_t k_mix, uint32_t q4) -> uint32_t {
        return c.qtype == 15 ? k_mix : (c.qtype == 2 ? q4 : (c.qtype == 30 ? (uint32_t)GGML_BF16 : GGML_Q8_0));
    };
    const uint32_t base = pick(GGML_Q4_K, GGML_Q4_0), more = pick(GGML_Q6_K, GGML_Q4_0);
    const int q_dim = c.n_head * c.head_dim, kv_dim = c.n_head_kv * c.head_dim;
    const uint32_t emb = pick(GGML_Q6_K, GGML_Q4_0);
    ts.push_back({"token_embd.weight", emb, c.n_embd, c.n_vocab, false});
    for (int i = 0; i < c.n_layer; ++i) {
        const std::string p = "blk." + std::to_string(i) + ".";
        const bool mb = use_more_bits(i, c.n_layer);
        ts.push_back({p + "attn_norm.weight", GGML_F32, c.n_embd, 1, true});
        if (lfm2 && !synth_lfm2_is_attn(c, i)) {
            // gated short conv: in_proj -> B | C | X, depthwise taps [n_embd][3], out_proj
            ts.push_back({p + "shortconv.in_proj.weight", base, c.n_embd, 3 * c.n_embd, false});
            ts.push_back({p + "shortconv.conv.weight", GGML_F32, 3, c.n_embd, 2});
            ts.push_back({p + "shortconv.out_proj.weight", base, c.n_embd, c.n_embd, false});
        } else {
        ts.push_back({p + "attn_q.weight", base, c.n_embd, q_dim, false});
        ts.push_back({p + "attn_k.weight", base, c.n_embd, kv_dim, false});
        ts.push_back({p + "attn_v.weight", mb ? more : base, c.n_embd, kv_dim, false});
        ts.push_back({p + "attn_output.weight", base, q_dim, c.n_embd, false});
        if (c.qkv_bias) {
            ts.push_back({p + "attn_q.bias", GGML_F32, q_dim, 1, 2});
            ts.push_back({p + "attn_k.bias", GGML_F32, kv_dim, 1, 2});
            ts.push_back({p + "attn_v.bias", GGML_F32, kv_dim, 1, 2});
        }
        if (a == "qwen3" || lfm2) {
            ts.push_back({p + "attn_q_norm.weight", GGML_F32, c.head_dim, 1, true});
            ts.push_back({p + "attn_k_norm.weight", GGML_F32, c.head_dim, 1, true});
        }
        }
        ts.push_back({p + "ffn_norm.weight", GGML_F32, c.n_embd, 1, true});
        ts.push_back({p + "ffn_gate.weight", base, c.n_embd, c.n_ff, false});
        ts.push_back({p + "ffn_up.weight", base, c.n_embd, c.n_ff, false});
        ts.push_back({p + "ffn_down.weight", mb ? more : base, c.n_ff, c.n_embd, false});
    }
    // lfm2's final norm is token_embd_norm (llama.cpp model.tok_norm)
    ts.push_back({lfm2 ? "token_embd_norm.weight" : "output_norm.weight", GGML_F32, c.n_embd, 1, true});
    if (!c.tied) ts.push_back({"output.weight", more, c.n_embd, c.n_vocab, false});
    // llama-quantize: a K-quant needs rows of whole 256-element super-blocks
    if (c.kq_fallback)
        for (auto &t : ts)
            if (t.k % 256 != 0) {
                if (t.type == GGML_Q4_K) t.type = GGML_Q5_0;
                if (t.type == GGML_Q6_K) t.type = GGML_Q8_0;
            }
    for (auto &t : ts) {
        if (t.rows == 1)
            w.add_tensor(t.name, t.type, {t.k});
        else
            w.add_tensor(t.name, t.type, {t.k, t.rows});
    }
    return w.write(path, [&](size_t idx, uint8_t *dst, size_t nbytes) {
        const T &t = ts[idx];
        if (t.fill == 1 || t.fill == 2) {
            float *f = (float *)dst;
            const uint64_t key = synth_key(c.seed, t.name);
            for (int64_t i = 0; i < t.k * t.rows; ++i)
                f[i] = t.fill == 1 ? 1.0f : 0.5f * synth_normal_fast(key, (uint64_t)i);
            return;
        }
        const size_t rb = ggml_row_bytes(t.type, t.k);
        const uint64_t key = synth_key(c.seed, t.name);
#pragma omp parallel
        {
            std::vector<float> row(t.k);
#pragma omp for schedule(static)
            for (int64_t r = 0; r < t.rows; ++r) {
                for (int64_t j = 0; j < t.k; ++j) row[j] = c.w_std * synth_normal_fast(key, (uint64_t)r * t.k + j);
                quantize_row(t.type, row.data(), dst + (size_t)r * rb, t.k);
            }
        }
        (void)nbytes;
    });
}

}  // namespace mio
