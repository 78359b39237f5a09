// GGUF byte-level BPE tokenizer (see tokenizer.h).
#include "tokenizer.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <functional>
#include <queue>
#include <set>

#include "common.h"
#include "gguf.h"
#include "unicode_ranges.h"

namespace mio {
namespace {

// ------------------------------------------------------------------ UTF-8
uint32_t utf8_decode(const std::string &s, size_t i, size_t *len) {
    const uint8_t c = (uint8_t)s[i];
    auto cont = [&](size_t k) { return i + k < s.size() ? ((uint8_t)s[i + k] & 0x3F) : 0u; };
    if (c < 0x80) return *len = 1, c;
    if ((c >> 5) == 6 && i + 1 < s.size()) return *len = 2, ((c & 0x1Fu) << 6) | cont(1);
    if ((c >> 4) == 14 && i + 2 < s.size()) return *len = 3, ((c & 0x0Fu) << 12) | (cont(1) << 6) | cont(2);
    if ((c >> 3) == 30 && i + 3 < s.size())
        return *len = 4, ((c & 0x07u) << 18) | (cont(1) << 12) | (cont(2) << 6) | cont(3);
    return *len = 1, c;  // invalid byte: passed through as its own "code point"
}

std::string utf8_encode(uint32_t cp) {
    std::string o;
    if (cp < 0x80) {
        o += (char)cp;
    } else if (cp < 0x800) {
        o += (char)(0xC0 | (cp >> 6));
        o += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
        o += (char)(0xE0 | (cp >> 12));
        o += (char)(0x80 | ((cp >> 6) & 0x3F));
        o += (char)(0x80 | (cp & 0x3F));
    } else {
        o += (char)(0xF0 | (cp >> 18));
        o += (char)(0x80 | ((cp >> 12) & 0x3F));
        o += (char)(0x80 | ((cp >> 6) & 0x3F));
        o += (char)(0x80 | (cp & 0x3F));
    }
    return o;
}

// ------------------------------------------------------------------ Unicode classes
struct R {
    uint32_t a, b;
};

bool in(const R *r, size_t n, uint32_t cp) {
    for (size_t i = 0; i < n; ++i)
        if (cp >= r[i].a && cp <= r[i].b) return true;
    return false;
}

bool is_space(uint32_t cp) {
    static const R r[] = {{0x09, 0x0D}, {0x20, 0x20}, {0x85, 0x85}, {0xA0, 0xA0}, {0x1680, 0x1680},
                          {0x2000, 0x200A}, {0x2028, 0x2029}, {0x202F, 0x202F}, {0x205F, 0x205F}, {0x3000, 0x3000}};
    return in(r, sizeof(r) / sizeof(r[0]), cp);
}

// \p{N} / \p{L}: general categories N* / L* (unicode_ranges.h, generated), binary search
bool in_sorted(const CpRange *r, size_t n, uint32_t cp) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (cp < r[mid].a)
            hi = mid;
        else if (cp > r[mid].b)
            lo = mid + 1;
        else
            return true;
    }
    return false;
}

bool is_number(uint32_t cp) { return in_sorted(kNumberRanges, kNumberRanges_n, cp); }

bool is_letter(uint32_t cp) { return cp < 0x80 ? ((cp | 32) - 'a') < 26u : in_sorted(kLetterRanges, kLetterRanges_n, cp); }

bool is_punct(uint32_t cp) { return in_sorted(kPunctRanges, kPunctRanges_n, cp); }

bool is_nl(uint32_t cp) { return cp == '\r' || cp == '\n'; }
uint32_t lower_ascii(uint32_t cp) { return cp >= 'A' && cp <= 'Z' ? cp + 32 : cp; }

// WPM classes (unicode_ranges.h): Cc / Cf / Co / Cs, the first code point of the canonical
// decomposition, the one-to-one lowercase mapping, CJK ideographs (BERT's _is_chinese_char)
bool is_control(uint32_t cp) { return in_sorted(kOtherRanges, kOtherRanges_n, cp); }
uint32_t nfd_first(uint32_t cp) {
    size_t lo = 0, hi = kNfdFirst_n;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (cp < kNfdFirst[mid].a)
            hi = mid;
        else if (cp > kNfdFirst[mid].b)
            lo = mid + 1;
        else
            return kNfdFirst[mid].v;
    }
    return cp;
}
uint32_t to_lower(uint32_t cp) {
    if (cp < 0x80) return lower_ascii(cp);
    size_t lo = 0, hi = kLowerPairs_n;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (cp < kLowerPairs[mid].a)
            hi = mid;
        else if (cp > kLowerPairs[mid].a)
            lo = mid + 1;
        else
            return kLowerPairs[mid].b;
    }
    return cp;
}
bool is_cjk(uint32_t cp) {
    return (cp >= 0x4E00 && cp <= 0x9FFF) || (cp >= 0x3400 && cp <= 0x4DBF) || (cp >= 0x20000 && cp <= 0x2A6DF) ||
           (cp >= 0x2A700 && cp <= 0x2B73F) || (cp >= 0x2B740 && cp <= 0x2B81F) || (cp >= 0x2B820 && cp <= 0x2CEAF) ||
           (cp >= 0xF900 && cp <= 0xFAFF) || (cp >= 0x2F800 && cp <= 0x2FA1F);
}
// ASCII symbols (general category S*: $ + < = > ^ ` | ~)
bool is_ascii_symbol(uint32_t cp) {
    return cp == '$' || cp == '+' || cp == '<' || cp == '=' || cp == '>' || cp == '^' || cp == '`' || cp == '|' ||
           cp == '~';
}

}  // namespace

// ------------------------------------------------------------------ load
bool BpeTokenizer::load(const GgufFile &g) {
    const std::string model = g.get_str("tokenizer.ggml.model");
    const GgufValue *tv = g.get("tokenizer.ggml.tokens");
    if (model == "llama" && tv && !tv->arr_s.empty()) return load_spm(g);
    if (model == "bert" && tv && !tv->arr_s.empty()) return load_wpm(g);
    if (model == "t5" && tv && !tv->arr_s.empty()) return load_ugm(g);
    if (model != "gpt2" || !tv || tv->arr_s.empty()) {
        set_error("tokenizer: GGUF has no gpt2 (byte-level BPE), llama (SPM), bert (WPM) or t5 (UGM) vocabulary "
                  "(model '%s')", model.c_str());
        return false;
    }
    tokens_ = tv->arr_s;
    types_.assign(tokens_.size(), 1);
    if (const GgufValue *tt = g.get("tokenizer.ggml.token_type"))
        for (size_t i = 0; i < tt->arr_i.size() && i < types_.size(); ++i) types_[i] = (int32_t)tt->arr_i[i];
    id_.reserve(tokens_.size() * 2);
    for (size_t i = 0; i < tokens_.size(); ++i) id_.emplace(tokens_[i], (int32_t)i);
    if (const GgufValue *mv = g.get("tokenizer.ggml.merges"))
        for (size_t i = 0; i < mv->arr_s.size(); ++i) merge_rank_.emplace(mv->arr_s[i], (int)i);
    std::set<size_t, std::greater<size_t>> lens;
    for (size_t i = 0; i < tokens_.size(); ++i)
        if ((types_[i] == 3 || types_[i] == 4) && !tokens_[i].empty()) {  // CONTROL, USER_DEFINED
            special_.emplace(tokens_[i], (int32_t)i);
            lens.insert(tokens_[i].size());
        }
    special_lens_.assign(lens.begin(), lens.end());
    eos_ = (int32_t)g.get_int("tokenizer.ggml.eos_token_id", -1);
    bos_ = (int32_t)g.get_int("tokenizer.ggml.bos_token_id", -1);
    const GgufValue *ab = g.get("tokenizer.ggml.add_bos_token");
    add_bos_ = ab ? ab->u != 0 : false;
    // llama.cpp's tokenizer.ggml.pre names (llama-vocab.cpp) of the families implemented here.
    // convert_hf_to_gguf.py writes "gpt-2" for the GPT-2 regex; llama-vocab.cpp maps the
    // other names below onto the same regex (its GPT2 / MPT / OLMO / JAIS pre types).
    // "gpt2" is kept for GGUFs written by hand with the tokenizer.ggml.model spelling.
    const std::string pre = g.get_str("tokenizer.ggml.pre", "default");
    static const char *const kGpt2Names[] = {"gpt-2",      "gpt2",       "phi-2",        "jina-es",  "jina-de",
                                             "jina-v1-en", "jina-v2-es", "jina-v2-de",   "jina-v2-code",
                                             "roberta-bpe", "gigachat",  "a.x-4.0",      "mellum",   "mpt",
                                             "olmo",       "jais"};
    bool gpt2_name = false;
    for (const char *n : kGpt2Names) gpt2_name = gpt2_name || pre == n;
    if (gpt2_name)
        pre_ = Pre::Gpt2;
    else if (pre == "default")
        pre_ = Pre::Default;
    else if (pre == "qwen2" || pre == "deepseek-r1-qwen" || pre == "megrez")
        pre_ = Pre::Qwen2;
    else if (pre == "llama3" || pre == "llama-v3" || pre == "llama-bpe" || pre == "falcon3" || pre == "pixtral" ||
             pre == "lfm2")
        pre_ = Pre::Llama3;
    else if (pre == "smollm" || pre == "starcoder" || pre == "refact" || pre == "command-r" || pre == "codeshell" ||
             pre == "exaone" || pre == "minerva-7b")
        pre_ = Pre::Smollm;
    else {
        set_error("tokenizer: pre-tokenizer '%s' is not implemented (gpt-2, default, qwen2, llama3 / llama-bpe / "
                  "lfm2, smollm families)", pre.c_str());
        return false;
    }
    // GPT-2 bytes_to_unicode: printable bytes map to themselves, the rest to 256 + n
    int n = 0;
    for (int b = 0; b < 256; ++b) {
        const bool keep = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || (b >= 174 && b <= 255);
        const uint32_t cp = keep ? (uint32_t)b : (uint32_t)(256 + n++);
        byte_enc_[b] = utf8_encode(cp);
        byte_dec_[cp] = (uint8_t)b;
    }
    return true;
}

void BpeTokenizer::load_vocab(const GgufFile &g) {
    tokens_ = g.get("tokenizer.ggml.tokens")->arr_s;
    const size_t n = tokens_.size();
    types_.assign(n, 1);
    if (const GgufValue *tt = g.get("tokenizer.ggml.token_type"))
        for (size_t i = 0; i < tt->arr_i.size() && i < n; ++i) types_[i] = (int32_t)tt->arr_i[i];
    id_.reserve(n * 2);
    for (size_t i = 0; i < n; ++i) id_.emplace(tokens_[i], (int32_t)i);
    std::set<size_t, std::greater<size_t>> lens;
    for (size_t i = 0; i < n; ++i)
        if ((types_[i] == 3 || types_[i] == 4) && !tokens_[i].empty()) {  // CONTROL, USER_DEFINED
            special_.emplace(tokens_[i], (int32_t)i);
            lens.insert(tokens_[i].size());
        }
    special_lens_.assign(lens.begin(), lens.end());
}

// SPM (tokenizer.ggml.model "llama"): tokens, scores, types; llama.cpp's defaults for this
// vocabulary type: BOS added, EOS not, a space prefix on the first fragment
bool BpeTokenizer::load_spm(const GgufFile &g) {
    spm_ = true;
    load_vocab(g);
    const size_t n = tokens_.size();
    scores_.assign(n, 0.0f);
    if (const GgufValue *sc = g.get("tokenizer.ggml.scores"))
        for (size_t i = 0; i < sc->arr_f.size() && i < n; ++i) scores_[i] = (float)sc->arr_f[i];
    eos_ = (int32_t)g.get_int("tokenizer.ggml.eos_token_id", -1);
    bos_ = (int32_t)g.get_int("tokenizer.ggml.bos_token_id", -1);
    unk_ = (int32_t)g.get_int("tokenizer.ggml.unknown_token_id", -1);
    const GgufValue *ab = g.get("tokenizer.ggml.add_bos_token");
    add_bos_ = ab ? ab->u != 0 : true;
    const GgufValue *ae = g.get("tokenizer.ggml.add_eos_token");
    add_eos_ = ae ? ae->u != 0 : false;
    const GgufValue *sp = g.get("tokenizer.ggml.add_space_prefix");
    add_space_prefix_ = sp ? sp->u != 0 : true;
    // byte tokens "<0xXX>", else the byte itself as a token, else unk
    static const char *hex = "0123456789ABCDEF";
    for (int b = 0; b < 256; ++b) {
        const char t[7] = {'<', '0', 'x', hex[b >> 4], hex[b & 15], '>', 0};
        auto it = id_.find(t);
        if (it == id_.end()) it = id_.find(std::string(1, (char)b));
        byte_tok_[b] = it != id_.end() ? it->second : unk_;
    }
    if (bos_ >= (int32_t)n || eos_ >= (int32_t)n || unk_ >= (int32_t)n) {
        set_error("tokenizer: SPM special token id out of range");
        return false;
    }
    return true;
}

// WPM (tokenizer.ggml.model "bert"): llama.cpp's defaults for this vocabulary type are the
// BERT ids [CLS] 101 (BOS), [UNK] 100, [SEP] 102, with BOS and SEP added around the text
bool BpeTokenizer::load_wpm(const GgufFile &g) {
    wpm_ = true;
    load_vocab(g);
    const int32_t n = (int32_t)tokens_.size();
    bos_ = (int32_t)g.get_int("tokenizer.ggml.bos_token_id", 101);
    eos_ = (int32_t)g.get_int("tokenizer.ggml.eos_token_id", -1);
    unk_ = (int32_t)g.get_int("tokenizer.ggml.unknown_token_id", 100);
    sep_ = (int32_t)g.get_int("tokenizer.ggml.seperator_token_id", 102);  // the GGUF key's spelling
    const GgufValue *ab = g.get("tokenizer.ggml.add_bos_token");
    add_bos_ = ab ? ab->u != 0 : true;
    const GgufValue *ae = g.get("tokenizer.ggml.add_eos_token");
    add_eos_ = ae ? ae->u != 0 : false;
    const GgufValue *as = g.get("tokenizer.ggml.add_sep_token");
    add_sep_ = as ? as->u != 0 : true;
    for (const std::string &t : tokens_) max_tok_len_ = std::max(max_tok_len_, t.size());
    if (bos_ >= n || eos_ >= n || unk_ >= n || sep_ >= n || unk_ < 0) {
        set_error("tokenizer: WPM special token id out of range");
        return false;
    }
    return true;
}

// ------------------------------------------------------------------ WPM
void BpeTokenizer::wpm(const std::string &text, std::vector<int32_t> &out) const {
    std::vector<std::string> words;
    std::string word;
    auto end_word = [&]() {
        if (!word.empty()) words.push_back(word);
        word.clear();
    };
    for (size_t i = 0; i < text.size();) {
        size_t l = 1;
        const uint32_t cp = nfd_first(utf8_decode(text, i, &l));
        i += l;
        if (is_space(cp)) {
            end_word();
            continue;
        }
        if (cp == 0 || cp == 0xFFFD || is_control(cp)) continue;
        const std::string c = utf8_encode(to_lower(cp));
        if (is_punct(cp) || is_ascii_symbol(cp) || is_cjk(cp)) {
            end_word();
            words.push_back(c);
        } else {
            word += c;
        }
    }
    end_word();
    for (const std::string &w : words) {
        const std::string s = "\xe2\x96\x81" + w;  // U+2581: a word-initial token
        const size_t first = out.size();
        bool ok = true;
        for (size_t i = 0; i < s.size() && ok;) {
            ok = false;
            for (size_t j = std::min(s.size(), i + max_tok_len_); j > i; --j) {
                const auto it = id_.find(s.substr(i, j - i));
                if (it != id_.end()) {
                    out.push_back(it->second);
                    i = j;
                    ok = true;
                    break;
                }
            }
        }
        if (!ok) {  // an unmatched position: the whole word is UNK
            out.resize(first);
            out.push_back(unk_);
        }
    }
}

// UGM (tokenizer.ggml.model "t5"): llama.cpp's defaults for this vocabulary type are the T5
// ids (pad 0, EOS 1, UNK 2, no BOS), EOS added after the text, a space prefix, whitespace
// escaped to U+2581 and not merged unless tokenizer.ggml.remove_extra_whitespaces
bool BpeTokenizer::load_ugm(const GgufFile &g) {
    ugm_ = true;
    load_vocab(g);
    const size_t n = tokens_.size();
    scores_.assign(n, 0.0f);
    if (const GgufValue *sc = g.get("tokenizer.ggml.scores"))
        for (size_t i = 0; i < sc->arr_f.size() && i < n; ++i) scores_[i] = (float)sc->arr_f[i];
    bos_ = (int32_t)g.get_int("tokenizer.ggml.bos_token_id", -1);
    eos_ = (int32_t)g.get_int("tokenizer.ggml.eos_token_id", 1);
    unk_ = (int32_t)g.get_int("tokenizer.ggml.unknown_token_id", 2);
    auto flag = [&](const char *k, bool def) {
        const GgufValue *v = g.get(k);
        return v ? v->u != 0 : def;
    };
    add_bos_ = flag("tokenizer.ggml.add_bos_token", false);
    add_eos_ = flag("tokenizer.ggml.add_eos_token", true);
    add_space_prefix_ = flag("tokenizer.ggml.add_space_prefix", true);
    remove_extra_ws_ = flag("tokenizer.ggml.remove_extra_whitespaces", false);
    if (bos_ >= (int32_t)n || eos_ >= (int32_t)n || unk_ >= (int32_t)n || unk_ < 0) {
        set_error("tokenizer: UGM special token id out of range");
        return false;
    }
    // the character map: u32 size of the double array, its units, then the NUL-terminated
    // replacement strings the leaves index
    if (const GgufValue *cm = g.get("tokenizer.ggml.precompiled_charsmap"); cm && !cm->arr_i.empty()) {
        std::string b(cm->arr_i.size(), '\0');
        for (size_t i = 0; i < b.size(); ++i) b[i] = (char)(uint8_t)cm->arr_i[i];
        uint32_t xs = 0;
        if (b.size() < 4 || (std::memcpy(&xs, b.data(), 4), xs % 4) || xs > b.size() - 4) {
            set_error("tokenizer: malformed precompiled_charsmap");
            return false;
        }
        xcda_.resize(xs / 4);
        std::memcpy(xcda_.data(), b.data() + 4, xs);
        repl_ = b.substr(4 + xs);
    }
    float min_score = INFINITY;
    std::set<size_t, std::greater<size_t>> ulens;
    for (size_t i = 0; i < n; ++i) {
        const int32_t t = types_[i];
        if (t == 1) min_score = std::min(min_score, scores_[i]);
        if (t == 1 || t == 4 || t == 5) ugm_tok_.emplace(tokens_[i], (int32_t)i);  // NORMAL, USER_DEFINED, UNUSED
        if (t == 4 && !tokens_[i].empty()) {
            user_def_.emplace(tokens_[i], (int32_t)i);
            ulens.insert(tokens_[i].size());
        }
        max_tok_len_ = std::max(max_tok_len_, tokens_[i].size());
    }
    user_def_lens_.assign(ulens.begin(), ulens.end());
    unk_score_ = (std::isfinite(min_score) ? min_score : 0.0f) - 10.0f;
    return true;
}

// ------------------------------------------------------------------ UGM
// One normalization step at byte i: a user-defined token is kept as it is; else the longest
// input prefix in the character map's double array (Darts-clone units: BASE = unit >> 10 shifted
// left by 8 when bit 9 is set, LCHECK = label | bit 31, LEAF = bit 8, a leaf child's VALUE =
// unit & 0x7FFFFFFF, the replacement's offset); else one UTF-8 character as it is (an invalid
// byte: U+FFFD)
std::pair<std::string, size_t> BpeTokenizer::ugm_prefix(const std::string &text, size_t i) const {
    for (size_t l : user_def_lens_)
        if (l <= text.size() - i && user_def_.count(text.substr(i, l))) return {text.substr(i, l), l};
    size_t best = 0, off = 0;
    if (!xcda_.empty()) {
        auto unit = [&](size_t k) { return k < xcda_.size() ? xcda_[k] : 0u; };
        auto base = [&](uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); };
        size_t node = base(unit(0));
        for (size_t p = i; p < text.size(); ++p) {
            const uint8_t c = (uint8_t)text[p];
            if (c == 0) break;
            node ^= c;
            const uint32_t u = unit(node);
            if ((u & ((1u << 31) | 0xFFu)) != c) break;
            const bool leaf = (u >> 8) & 1;
            node ^= base(u);
            if (leaf) {
                best = p - i + 1;
                off = unit(node) & ((1u << 31) - 1);
            }
        }
    }
    if (best > 0 && off < repl_.size()) return {std::string(repl_.c_str() + off), best};
    // a valid UTF-8 sequence is kept, anything else is one byte -> U+FFFD
    const uint8_t c = (uint8_t)text[i];
    const size_t l = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    bool ok = l > 0 && i + l <= text.size();
    for (size_t k = 1; ok && k < l; ++k) ok = ((uint8_t)text[i + k] >> 6) == 2;
    if (!ok) return {"\xef\xbf\xbd", 1};
    return {text.substr(i, l), l};
}

std::string BpeTokenizer::ugm_normalize(const std::string &text) const {
    const std::string space = escape_ws_ ? "\xe2\x96\x81" : " ";
    const bool prepend = !ws_suffix_ && add_space_prefix_, append = ws_suffix_ && add_space_prefix_;
    const bool merge = remove_extra_ws_;
    bool prepended = false, non_ws = false;
    std::string o;
    for (size_t i = 0; i < text.size();) {
        const auto r = ugm_prefix(text, i);
        for (char c : r.first) {
            if (c != ' ') {
                if (!non_ws) {
                    non_ws = true;
                    if ((prepend && !prepended) || merge) {
                        o += space;
                        prepended = true;
                    }
                }
                o += c;
            } else {
                non_ws = false;
                if (!merge) o += space;
            }
        }
        i += r.second;
    }
    if (append) o += space;
    return o;
}

// Viterbi over the normalized bytes: best[e] = the best segmentation of [0, e) (score sums in
// double, kept as float), every token starting at a code point boundary; a code point no token
// covers alone may be UNK at unk_score_; backtracked, with runs of UNK merged into one
void BpeTokenizer::ugm(const std::string &text, std::vector<int32_t> &out) const {
    const std::string s = ugm_normalize(text);
    const size_t n = s.size();
    if (n == 0) return;
    struct Best {
        int32_t id;
        size_t from;
        float score;
    };
    std::vector<Best> best(n + 1, {unk_, 0, -FLT_MAX});
    best[0] = {unk_, 0, 0.0f};
    for (size_t i = 0; i < n;) {
        const uint8_t c = (uint8_t)s[i];
        const size_t cl = std::min(n - i, (size_t)(c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1));
        bool single = false;
        const Best cur = best[i];
        for (size_t l = 1; l <= std::min(max_tok_len_, n - i); ++l) {
            const auto it = ugm_tok_.find(s.substr(i, l));
            if (it == ugm_tok_.end()) continue;
            if (l == cl) single = true;
            const double sc = (double)cur.score + (types_[it->second] == 4 ? 0.0 : (double)scores_[it->second]);
            if (sc > best[i + l].score) best[i + l] = {it->second, i, (float)sc};
        }
        if (!single) {
            const double sc = (double)cur.score + (double)unk_score_;
            if (sc > best[i + cl].score) best[i + cl] = {unk_, i, (float)sc};
        }
        i += cl;
    }
    std::vector<int32_t> rev;
    bool prev_unk = false;
    for (size_t e = n;;) {
        const Best &b = best[e];
        const bool is_unk = b.id == unk_;
        if (!(prev_unk && is_unk)) rev.push_back(b.id);
        if (b.from == 0) break;
        prev_unk = is_unk;
        e = b.from;
    }
    out.insert(out.end(), rev.rbegin(), rev.rend());
}

// ------------------------------------------------------------------ SPM
void BpeTokenizer::spm(const std::string &text, std::vector<int32_t> &out) const {
    struct Sym {
        int prev, next;
        size_t off, n;
    };
    std::vector<Sym> sym;
    for (size_t off = 0; off < text.size();) {
        size_t l = 1;
        utf8_decode(text, off, &l);
        l = std::min(l, text.size() - off);
        const int idx = (int)sym.size();
        sym.push_back({idx - 1, off + l == text.size() ? -1 : idx + 1, off, l});
        off += l;
    }
    if (sym.empty()) return;
    struct Bigram {
        int left, right;
        float score;
        size_t size;
    };
    // highest score first; equal scores: the leftmost pair
    auto worse = [](const Bigram &a, const Bigram &b) { return a.score < b.score || (a.score == b.score && a.left > b.left); };
    std::priority_queue<Bigram, std::vector<Bigram>, decltype(worse)> q(worse);
    std::unordered_map<std::string, std::pair<int, int>> rev;
    auto add = [&](int l, int r) {
        if (l < 0 || r < 0) return;
        const std::string t = text.substr(sym[l].off, sym[l].n + sym[r].n);
        const auto it = id_.find(t);
        if (it == id_.end()) return;
        q.push({l, r, scores_[it->second], t.size()});
        rev[t] = {l, r};
    };
    for (int i = 1; i < (int)sym.size(); ++i) add(i - 1, i);
    while (!q.empty()) {
        const Bigram b = q.top();
        q.pop();
        Sym &L = sym[b.left], &R = sym[b.right];
        if (L.n == 0 || R.n == 0 || L.n + R.n != b.size) continue;  // stale: a side was merged since
        L.n += R.n;
        R.n = 0;
        L.next = R.next;
        if (R.next >= 0) sym[R.next].prev = b.left;
        add(L.prev, b.left);
        add(b.left, L.next);
    }
    // a final symbol that is no token: the two symbols it was merged from (split at the right
    // one's start: symbol starts never move), recursively; characters of no token -> bytes
    std::function<void(size_t, size_t)> reseg;
    reseg = [&](size_t off, size_t n) {
        const std::string t = text.substr(off, n);
        const auto it = id_.find(t);
        if (it != id_.end()) {
            out.push_back(it->second);
            return;
        }
        const auto p = rev.find(t);
        if (p == rev.end()) {
            for (size_t j = 0; j < n; ++j) out.push_back(byte_tok_[(unsigned char)text[off + j]]);
            return;
        }
        const size_t split = sym[p->second.second].off;
        reseg(off, split - off);
        reseg(split, off + n - split);
    };
    for (int i = 0; i != -1; i = sym[i].next) reseg(sym[i].off, sym[i].n);
}

int32_t BpeTokenizer::special_id(const std::string &text) const {
    const auto it = special_.find(text);
    return it == special_.end() ? -1 : it->second;
}

// ------------------------------------------------------------------ pre-tokenizer
// llama.cpp applies a pre-type's regexes in sequence; each one splits every fragment left by
// the previous one into its matches and the unmatched runs between them (both kept), and
// lookaheads see only the fragment. The regexes, per family:
//   gpt2   : 's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
//   default: [\p{P}\$\+<=>\^~\|]+ , then the gpt2 regex, then \p{N}+ , then [0-9][0-9][0-9]
//   qwen2  : (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*
//            |\s*[\r\n]+|\s+(?!\S)|\s+
//   llama3 : the qwen2 regex with \p{N}{1,3} (and ASCII-only case-insensitive contractions)
//   smollm : \p{N} , then the gpt2 regex
namespace {

struct Cps {
    const std::vector<uint32_t> &cp;
    size_t e;  // fragment end: every class test past it is false
    bool L(size_t k) const { return k < e && is_letter(cp[k]); }
    bool N(size_t k) const { return k < e && is_number(cp[k]); }
    bool S(size_t k) const { return k < e && is_space(cp[k]); }
    bool O(size_t k) const { return k < e && !is_space(cp[k]) && !is_letter(cp[k]) && !is_number(cp[k]); }
    uint32_t at(size_t k) const { return k < e ? cp[k] : 0; }
};

// 's|'t|'re|'ve|'m|'ll|'d, optionally ASCII case-insensitive
size_t m_contraction(const Cps &c, size_t i, bool fold) {
    if (c.at(i) != '\'') return 0;
    auto f = [&](uint32_t x) { return fold ? lower_ascii(x) : x; };
    const uint32_t a = f(c.at(i + 1)), b = f(c.at(i + 2));
    if (a == 's' || a == 't' || a == 'm' || a == 'd') return 2;
    if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
    return 0;
}

// \s+(?!\S)|\s+ at a whitespace run [i, j)
size_t m_spaces(const Cps &c, size_t i) {
    size_t j = i;
    while (c.S(j)) ++j;
    if (j == i) return 0;
    return (j == c.e || j - i == 1) ? j - i : j - i - 1;
}

size_t m_gpt2(const Cps &c, size_t i) {
    if (size_t m = m_contraction(c, i, false)) return m;
    const size_t k = i + (c.at(i) == ' ' ? 1 : 0);
    size_t j = k;
    if (c.L(k)) {
        while (c.L(j)) ++j;
        return j - i;
    }
    if (c.N(k)) {
        while (c.N(j)) ++j;
        return j - i;
    }
    if (c.O(k)) {
        while (c.O(j)) ++j;
        return j - i;
    }
    return m_spaces(c, i);
}

// qwen2 (ndig 1) and llama3 (ndig 3)
size_t m_qwen(const Cps &c, size_t i, int ndig) {
    if (size_t m = m_contraction(c, i, true)) return m;
    {  // [^\r\n\p{L}\p{N}]?\p{L}+
        size_t k = i;
        if (!c.L(k) && k < c.e && !is_nl(c.cp[k]) && !c.N(k) && c.L(k + 1)) ++k;
        if (c.L(k)) {
            while (c.L(k)) ++k;
            return k - i;
        }
    }
    if (c.N(i)) {  // \p{N}{1,ndig}
        size_t k = i;
        while (c.N(k) && (int)(k - i) < ndig) ++k;
        return k - i;
    }
    {  // ' ?[^\s\p{L}\p{N}]+[\r\n]*'
        size_t k = i + (c.at(i) == ' ' ? 1 : 0);
        if (c.O(k)) {
            while (c.O(k)) ++k;
            while (k < c.e && is_nl(c.cp[k])) ++k;
            return k - i;
        }
    }
    if (c.S(i)) {  // \s*[\r\n]+ : up to the last newline of the whitespace run, else \s+(?!\S)|\s+
        size_t j = i, last = SIZE_MAX;
        while (c.S(j)) {
            if (is_nl(c.cp[j])) last = j;
            ++j;
        }
        if (last != SIZE_MAX) return last + 1 - i;
        return m_spaces(c, i);
    }
    return 0;
}

// [\p{P}\$\+<=>\^~\|]+
size_t m_punct(const Cps &c, size_t i) {
    size_t k = i;
    auto p = [&](size_t q) {
        if (q >= c.e) return false;
        const uint32_t x = c.cp[q];
        return is_punct(x) || x == '$' || x == '+' || x == '<' || x == '=' || x == '>' || x == '^' || x == '~' ||
               x == '|';
    };
    while (p(k)) ++k;
    return k - i;
}

// \p{N}+ (run = true) or \p{N}
size_t m_num(const Cps &c, size_t i, bool run) {
    size_t k = i;
    while (c.N(k) && (run || k == i)) ++k;
    return k - i;
}

// [0-9][0-9][0-9]
size_t m_dig3(const Cps &c, size_t i) {
    for (size_t k = i; k < i + 3; ++k)
        if (k >= c.e || c.cp[k] < '0' || c.cp[k] > '9') return 0;
    return 3;
}

// One regex stage over the fragment boundaries `cut` (sorted code-point offsets, first 0,
// last n): every fragment is split into its leftmost-first matches and the runs between.
template <class M>
void stage(const std::vector<uint32_t> &cp, std::vector<size_t> &cut, M &&match) {
    std::vector<size_t> out{0};
    for (size_t f = 0; f + 1 < cut.size(); ++f) {
        const Cps c{cp, cut[f + 1]};
        for (size_t i = cut[f]; i < c.e;) {
            const size_t m = match(c, i);
            if (m) {
                if (out.back() != i) out.push_back(i);
                out.push_back(i + m);
                i += m;
            } else {
                ++i;
            }
        }
        if (out.back() != c.e) out.push_back(c.e);
    }
    cut.swap(out);
}

}  // namespace

void BpeTokenizer::pretokenize(const std::string &text, std::vector<std::string> &pieces) const {
    std::vector<uint32_t> cp;
    std::vector<size_t> off;
    for (size_t i = 0; i < text.size();) {
        size_t l = 1;
        cp.push_back(utf8_decode(text, i, &l));
        off.push_back(i);
        i += l;
    }
    off.push_back(text.size());
    std::vector<size_t> cut{0, cp.size()};
    if (cp.empty()) return;
    switch (pre_) {
        case Pre::Gpt2: stage(cp, cut, m_gpt2); break;
        case Pre::Default:
            stage(cp, cut, m_punct);
            stage(cp, cut, m_gpt2);
            stage(cp, cut, [](const Cps &c, size_t i) { return m_num(c, i, true); });
            stage(cp, cut, m_dig3);
            break;
        case Pre::Qwen2: stage(cp, cut, [](const Cps &c, size_t i) { return m_qwen(c, i, 1); }); break;
        case Pre::Llama3: stage(cp, cut, [](const Cps &c, size_t i) { return m_qwen(c, i, 3); }); break;
        case Pre::Smollm:
            stage(cp, cut, [](const Cps &c, size_t i) { return m_num(c, i, false); });
            stage(cp, cut, m_gpt2);
            break;
    }
    for (size_t k = 0; k + 1 < cut.size(); ++k) pieces.emplace_back(text.substr(off[cut[k]], off[cut[k + 1]] - off[cut[k]]));
}

// ------------------------------------------------------------------ BPE
void BpeTokenizer::bpe(const std::string &piece, std::vector<int32_t> &out) const {
    std::vector<std::string> sym;
    for (unsigned char c : piece) sym.push_back(byte_enc_[c]);
    if (sym.empty()) return;
    while (sym.size() > 1 && !merge_rank_.empty()) {
        int best = INT_MAX;
        size_t at = 0;
        for (size_t k = 0; k + 1 < sym.size(); ++k) {
            const auto it = merge_rank_.find(sym[k] + " " + sym[k + 1]);
            if (it != merge_rank_.end() && it->second < best) best = it->second, at = k;
        }
        if (best == INT_MAX) break;
        sym[at] += sym[at + 1];
        sym.erase(sym.begin() + at + 1);
    }
    for (const std::string &s : sym) {
        const auto it = id_.find(s);
        if (it != id_.end()) {
            out.push_back(it->second);
            continue;
        }
        // not in the vocabulary: fall back to its single-byte symbols
        for (size_t i = 0; i < s.size();) {
            size_t l = 1;
            utf8_decode(s, i, &l);
            const auto jt = id_.find(s.substr(i, l));
            if (jt != id_.end()) out.push_back(jt->second);
            i += l;
        }
    }
}

std::vector<int32_t> BpeTokenizer::tokenize(const std::string &text, bool add_special, bool parse_special) const {
    std::vector<int32_t> out;
    if (add_special && add_bos_ && bos_ >= 0) out.push_back(bos_);
    std::string run;
    bool prev_special = true;  // SPM: the space prefix goes on a fragment that opens the text or follows a special
    auto flush = [&]() {
        if (run.empty()) return;
        if (wpm_) {
            wpm(run, out);
        } else if (ugm_) {
            ugm(run, out);
        } else if (spm_) {
            std::string t = add_space_prefix_ && prev_special ? " " + run : run;
            std::string e;
            for (char c : t) {
                if (c == ' ')
                    e += "\xe2\x96\x81";  // U+2581
                else
                    e += c;
            }
            spm(e, out);
            prev_special = false;
        } else {
            std::vector<std::string> pieces;
            pretokenize(run, pieces);
            for (const std::string &p : pieces) bpe(p, out);
        }
        run.clear();
    };
    for (size_t i = 0; i < text.size();) {
        int32_t sid = -1;
        size_t slen = 0;
        if (parse_special)
            for (size_t l : special_lens_) {
                if (l > text.size() - i) continue;
                const auto it = special_.find(text.substr(i, l));
                if (it != special_.end()) {
                    sid = it->second, slen = l;
                    break;
                }
            }
        if (sid >= 0) {
            flush();
            out.push_back(sid);
            prev_special = true;
            i += slen;
        } else {
            run += text[i++];
        }
    }
    flush();
    if ((spm_ || wpm_ || ugm_) && add_special && add_eos_ && eos_ >= 0) out.push_back(eos_);
    if (wpm_ && add_special && add_sep_ && sep_ >= 0) out.push_back(sep_);
    return out;
}

std::string BpeTokenizer::piece(int32_t id) const {
    if (id < 0 || id >= (int32_t)tokens_.size()) return "";
    const std::string &t = tokens_[id];
    if (types_[id] == 3 || types_[id] == 4) return t;  // special: rendered as text
    if (spm_ || wpm_ || ugm_) {
        // llama_token_to_piece(special = true): UNKNOWN as its text, NORMAL with U+2581 -> ' ',
        // BYTE "<0xXX>" -> the byte, other types (UNUSED) nothing
        if (types_[id] == 2) return t;
        if (types_[id] == 6) {
            if (t.size() == 6 && t.compare(0, 3, "<0x") == 0 && t[5] == '>')
                return std::string(1, (char)std::stoi(t.substr(3, 2), nullptr, 16));
            return t;
        }
        if (types_[id] != 1) return "";
        std::string o;
        for (size_t i = 0; i < t.size();) {
            if (t.compare(i, 3, "\xe2\x96\x81") == 0) {
                o += ' ';
                i += 3;
            } else {
                o += t[i++];
            }
        }
        return o;
    }
    std::string o;
    for (size_t i = 0; i < t.size();) {
        size_t l = 1;
        const uint32_t c = utf8_decode(t, i, &l);
        const auto it = byte_dec_.find(c);
        if (it != byte_dec_.end())
            o += (char)it->second;
        else
            o += t.substr(i, l);
        i += l;
    }
    return o;
}

}  // namespace mio
