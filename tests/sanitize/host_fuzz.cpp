// Host-parser robustness under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; built
// and run by tests/test_sanitize_host.py with g++ -fsanitize=address,undefined). The product's
// GGUF reader, BPE tokenizer, quant-block re-layout and text/WAV helpers parse user-supplied
// files by offset, as the reference's miocodec_load does (miocodec.cpp:92-135, 426-504):
//   1. valid synthetic GGUFs (tiny LLMs with a gpt2 vocabulary, the tiny codec, a voice) open,
//      tokenize, and every tensor dequantizes / re-lays out (quant.cpp to_split);
//   2. every truncation of each file's header and the first data bytes is refused with a
//      message (no read past the mapping);
//   3. seeded corruptions of header bytes and targeted out-of-range fields (tensor offsets,
//      shapes, counts, string lengths, general.alignment) either are refused or open to a file
//      whose tensors all lie inside the mapping;
//   4. random byte strings through the speech-token parser, the normaliser and the WAV writer.
// Any sanitizer report aborts the process (-fno-sanitize-recover=all); exit 0 = clean.
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "gguf.h"
#include "quant.h"
#include "synth.h"
#include "text-normalize.h"
#include "token-parser.h"
#include "tokenizer.h"
#include "wav-writer.h"

// the product library defines these in csrc/capi/device.cpp (HIP runtime); the parsers only
// need the message sink
namespace mio {
static thread_local std::string g_err;
void set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
const char *last_error() { return g_err.c_str(); }
}  // namespace mio

static std::vector<uint8_t> read_file(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
static void write_file(const std::string &p, const uint8_t *d, size_t n) {
    FILE *f = std::fopen(p.c_str(), "wb");
    if (n) std::fwrite(d, 1, n, f);
    std::fclose(f);
}

static int g_opened = 0, g_refused = 0;

// Opens path and exercises everything a loader reads; returns whether it opened.
static bool exercise(const std::string &path, bool expect_ok) {
    mio::GgufFile g;
    if (!g.open(path)) {
        if (expect_ok) {
            std::fprintf(stderr, "valid file refused: %s (%s)\n", path.c_str(), mio::last_error());
            std::exit(2);
        }
        if (!*mio::last_error()) {
            std::fprintf(stderr, "refusal without a message: %s\n", path.c_str());
            std::exit(3);
        }
        ++g_refused;
        return false;
    }
    ++g_opened;
    const uint8_t *lo = nullptr, *hi = nullptr;
    // reused across calls: ASan maps and unmaps every large allocation
    static std::vector<float> row;
    static std::vector<uint8_t> split;
    for (const auto &t : g.tensors()) {
        // every byte of every tensor is touched (ASan: inside the mapping)
        volatile uint8_t acc = 0;
        for (size_t i = 0; i < t.nbytes; i += 4096) acc ^= t.data[i];
        if (t.nbytes) acc ^= t.data[t.nbytes - 1];
        (void)acc;
        const int64_t k = t.ne[0], rows = t.nbytes / std::max<size_t>(1, mio::ggml_row_bytes(t.type, k));
        if (k <= 0 || k > (1 << 20)) continue;
        row.resize((size_t)k);
        for (int64_t r = 0; r < rows && r < 4; ++r)
            mio::dequantize_row(t.type, t.data + (size_t)r * mio::ggml_row_bytes(t.type, k), row.data(), k);
        if (rows > 0 && rows < 4096 && (t.type == mio::GGML_Q8_0 || t.type == mio::GGML_Q4_K || t.type == mio::GGML_Q6_K)) {
            split.resize(mio::split_layout(t.type, rows, k).bytes);
            mio::to_split(t.type, t.data, rows, k, split.data());
        }
        if (!lo || t.data < lo) lo = t.data;
        if (!hi || t.data + t.nbytes > hi) hi = t.data + t.nbytes;
    }
    mio::BpeTokenizer tk;
    if (tk.load(g)) {
        const char *texts[] = {"", "hello world", "こんにちは、今日はいい天気ですね。", "ＡＢＣ①ｶﾞ Café naïve [SEP]",
                               "<|im_start|>user\n12345 it's<|im_end|>\n", "\xff\xfe\x80 broken \xe3\x81",
                               "   \r\n\t  tabs and  spaces  "};
        for (const char *s : texts)
            for (int sp = 0; sp < 2; ++sp) {
                const auto ids = tk.tokenize(s, sp, sp);
                for (int32_t id : ids) (void)tk.piece(id);
            }
        for (int32_t id = -3; id < tk.n_vocab() + 3; ++id) (void)tk.piece(id);
        (void)tk.piece(tk.eos()), (void)tk.piece(tk.bos());
        (void)tk.special_id("<|im_end|>");
    }
    return true;
}

// usage: host_fuzz DIR [quick|full] [GGUF...]  (quick: the CPU suite's budget, one LLM, fewer
// mutations; further GGUFs, e.g. tokenizer-only WPM / UGM vocabularies, are fuzzed the same way)
int main(int argc, char **argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const bool quick = argc > 2 && std::string(argv[2]) == "quick";
    const int n_random = quick ? 40 : 300, trunc_mid = quick ? 8 : 64;
    const size_t head_every = quick ? 5 : 1, field_step = quick ? 8 : 4;
    std::vector<std::string> files;
    auto llm = [&](int preset) {
        mio::SynthLlmCfg c = mio::synth_llm_preset(preset);
        c.n_vocab = 13312, c.n_embd = 64, c.n_head = 2, c.n_head_kv = 1, c.head_dim = 32, c.n_ff = 128;
        const std::string p = dir + "/llm" + std::to_string(preset) + ".gguf";
        if (!mio::synth_write_llm(p, c)) std::exit(4);
        files.push_back(p);
    };
    llm(0);  // llama Q8_0
    if (!quick) llm(1), llm(7);  // qwen3 Q4_K_M, lfm2
    {
        const std::string p = dir + "/codec.gguf";
        if (!mio::synth_write_codec(p, mio::synth_codec_preset(1))) std::exit(4);
        files.push_back(p);
        const std::string v = dir + "/voice.emb.gguf";
        if (!mio::synth_write_voice(v, 7)) std::exit(4);
        files.push_back(v);
    }
    for (int a = 3; a < argc; ++a) files.push_back(argv[a]);
    std::mt19937_64 rng(1234);
    const std::string mut = dir + "/mut.gguf";
    for (const auto &f : files) {
        std::fprintf(stderr, "host_fuzz: %s\n", f.c_str());
        exercise(f, true);
        const std::vector<uint8_t> b = read_file(f);
        mio::GgufFile g;
        g.open(f);
        // a file without tensors ends inside the alignment padding its data offset counts
        const size_t hdr = std::min<size_t>(g.data_offset(), b.size());
        // the tensor-info records close the header (name, n_dims, ne[], type, offset each);
        // the KV section before them is dominated by the vocabulary strings
        size_t ti = 0;
        for (const auto &t : g.tensors()) ti += 8 + t.name.size() + 4 + 8 * (size_t)t.n_dims + 4 + 8;
        g.close();
        const size_t ti0 = hdr > ti + 32 ? hdr - ti - 32 : 0;
        // header positions worth mutating: the fixed header + the first KV records, and the
        // tensor-info records
        auto pick = [&]() -> size_t { return (rng() & 1) ? rng() % std::min<size_t>(hdr, 2048) : ti0 + rng() % (hdr - ti0); };
        // 2. truncations: every cut in the first 2 KB and in the tensor-info records, 64 cuts
        // between, cuts inside the data
        for (size_t n = 0; n < hdr; n += (n < 2048 || n >= ti0) ? head_every : std::max<size_t>(1, (ti0 - 2048) / trunc_mid)) {
            write_file(mut, b.data(), n);
            exercise(mut, false);
        }
        for (size_t n = hdr; n < b.size(); n += std::max<size_t>(1, (b.size() - hdr) / 16)) {
            write_file(mut, b.data(), n);
            exercise(mut, false);
        }
        // 3a. random corruptions: 1-4 bytes per file, 300 files
        std::vector<uint8_t> c = b;  // mutated in place, restored after each file
        for (int it = 0; it < n_random; ++it) {
            const int k = 1 + (int)(rng() % 4);
            size_t at[4];
            for (int j = 0; j < k; ++j) at[j] = pick(), c[at[j]] = (uint8_t)rng();
            write_file(mut, c.data(), c.size());
            exercise(mut, false);
            for (int j = 0; j < k; ++j) c[at[j]] = b[at[j]];
        }
        // 3b. targeted fields: every 4-byte-aligned 8-byte word of the fixed header, the first
        // KV records and the tensor-info records set to extreme values (huge counts / string
        // lengths / offsets / shapes, negative shapes, zero)
        const uint64_t vals[] = {0, 1, 0xFFFFFFFFull, 0x7FFFFFFFFFFFFFFFull, 0xFFFFFFFFFFFFFFFFull,
                                 0x8000000000000000ull, (uint64_t)b.size(), (uint64_t)-32};
        for (size_t off = 8; off + 8 <= hdr; off += field_step) {
            if (off >= 512 && off < ti0) off = ti0 & ~(size_t)3;
            for (uint64_t v : vals) {
                std::memcpy(c.data() + off, &v, 8);
                write_file(mut, c.data(), c.size());
                exercise(mut, false);
                std::memcpy(c.data() + off, b.data() + off, 8);
            }
        }
    }
    // 4. text helpers on random bytes
    std::string s;
    for (int it = 0; it < (quick ? 1000 : 3000); ++it) {
        s.clear();
        const int n = (int)(rng() % 64);
        for (int j = 0; j < n; ++j) {
            const uint64_t r = rng();
            if (r % 5 == 0)
                s += "<|s_";
            else if (r % 7 == 0)
                s += "|>";
            else if (r % 11 == 0)
                s += "。";
            else
                s += (char)(r >> 8);
        }
        (void)parse_speech_tokens(s);
        (void)normalize_tts_text(s);
    }
    std::vector<float> pcm(1000);
    for (size_t i = 0; i < pcm.size(); ++i) pcm[i] = (float)((int64_t)(rng() % 4001) - 2000) / 1000.0f;
    pcm[3] = NAN, pcm[4] = INFINITY, pcm[5] = -INFINITY;
    if (!wav_write(dir + "/out.wav", pcm, 44100)) return 5;
    std::printf("host_fuzz: clean (%d files opened, %d refused)\n", g_opened, g_refused);
    return 0;
}
