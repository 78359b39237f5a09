// Host text utilities on the path between the LLM and the codec:
//   normalize_tts_text  behaviour of text-normalize.cpp:108-158 (JP-only normalisation)
//   parse_speech_tokens behaviour of token-parser.cpp:5-28
//   wav_write           byte-identical output of wav-writer.cpp:24-44
// Checked against fixtures generated from the reference sources (tests/golden/).
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "common.h"
#include "text-normalize.h"
#include "token-parser.h"
#include "wav-writer.h"
#include "wav.h"

namespace {

// Decodes one code point (lenient like the reference: malformed lead bytes count as one).
uint32_t next_cp(const std::string &s, size_t &i) {
    const unsigned char c = (unsigned char)s[i];
    int len = 1;
    uint32_t cp = c;
    if ((c >> 5) == 0x6)
        len = 2, cp = c & 0x1F;
    else if ((c >> 4) == 0xE)
        len = 3, cp = c & 0x0F;
    else if ((c >> 3) == 0x1E)
        len = 4, cp = c & 0x07;
    if (len > 1 && i + len - 1 < s.size()) {
        for (int k = 1; k < len; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
        i += len;
        return cp;
    }
    i += 1;
    return c;
}

bool japanese_ratio_ok(const std::string &t) {
    int total = 0, ja = 0;
    for (size_t i = 0; i < t.size();) {
        const uint32_t cp = next_cp(t, i);
        if (cp == ' ' || cp == '\t' || cp == '\n' || cp == '\r') continue;
        ++total;
        const bool kana = cp >= 0x3040 && cp <= 0x30FF;
        const bool han = (cp >= 0x4E00 && cp <= 0x9FFF) || (cp >= 0x3400 && cp <= 0x4DBF);
        ja += (kana || han) ? 1 : 0;
    }
    return total > 0 && (float)ja / (float)total >= 0.1f;
}

void replace_every(std::string &s, const char *from, const char *to) {
    const size_t fl = std::strlen(from), tl = std::strlen(to);
    if (!fl) return;
    for (size_t p = s.find(from); p != std::string::npos; p = s.find(from, p + tl)) s.replace(p, fl, to);
}

bool has_prefix(const std::string &s, const char *p) { return s.rfind(p, 0) == 0; }
bool has_suffix(const std::string &s, const char *x) {
    const size_t n = std::strlen(x);
    return s.size() >= n && s.compare(s.size() - n, n, x) == 0;
}

}  // namespace

std::string normalize_tts_text(const std::string &text) {
    if (!japanese_ratio_ok(text)) return text;
    std::string s = text;
    static const char *const kDrop[] = {"\t", "[n]", " ", "\xE3\x80\x80" /* U+3000 */};
    for (const char *d : kDrop) replace_every(s, d, "");
    static const char *const kMap[][2] = {
        {"\xEF\xBC\x9F", "?"},                 // ？
        {"\xEF\xBC\x81", "!"},                 // ！
        {"\xE3\x80\x9C", "\xE3\x83\xBC"},      // 〜 -> ー
        {"\xEF\xBD\x9E", "\xE3\x83\xBC"},      // ～ -> ー
        {"\xE2\x99\xA5", "\xE2\x99\xA1"},      // ♥ -> ♡
        {"\xE2\x97\x8F", "\xE2\x97\x8B"},      // ● -> ○
        {"\xE2\x97\xAF", "\xE2\x97\x8B"},      // ◯ -> ○
        {"\xE3\x80\x87", "\xE2\x97\x8B"},      // 〇 -> ○
    };
    for (auto &m : kMap) replace_every(s, m[0], m[1]);
    const char *ell3 = "\xE2\x80\xA6\xE2\x80\xA6\xE2\x80\xA6", *ell2 = "\xE2\x80\xA6\xE2\x80\xA6";
    while (s.find(ell3) != std::string::npos) replace_every(s, ell3, ell2);
    static const char *const kWrap[][2] = {
        {"\xE3\x80\x8C", "\xE3\x80\x8D"},  // 「」
        {"\xE3\x80\x8E", "\xE3\x80\x8F"},  // 『』
        {"\xEF\xBC\x88", "\xEF\xBC\x89"},  // （）
        {"\xE3\x80\x90", "\xE3\x80\x91"},  // 【】
        {"(", ")"},
    };
    for (auto &w : kWrap) {
        const size_t a = std::strlen(w[0]), b = std::strlen(w[1]);
        if (has_prefix(s, w[0]) && has_suffix(s, w[1]) && s.size() > a + b) s = s.substr(a, s.size() - a - b);
    }
    const char *maru = "\xE3\x80\x82", *ten = "\xE3\x80\x81";  // 。 、
    while (has_suffix(s, maru) || has_suffix(s, ten)) s.resize(s.size() - 3);
    return s;
}

std::vector<int> parse_speech_tokens(const std::string &text) {
    std::vector<int> codes;
    const char *p = text.c_str(), *end = p + text.size();
    while (p < end) {
        const char *hit = std::strstr(p, "<|s_");
        if (!hit) break;
        const char *digits = hit + 4;
        char *stop = nullptr;
        const long v = std::strtol(digits, &stop, 10);
        if (stop && stop > digits && stop + 1 < end && stop[0] == '|' && stop[1] == '>') {
            codes.push_back((int)v);
            p = stop + 2;
        } else {
            p = hit + 1;
        }
    }
    return codes;
}

namespace {
void put16(std::vector<uint8_t> &b, uint16_t v) { b.push_back(v & 0xFF), b.push_back(v >> 8); }
void put32(std::vector<uint8_t> &b, uint32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back((v >> (8 * i)) & 0xFF);
}
}  // namespace

namespace mio {
std::vector<uint8_t> wav_header(size_t n, int sample_rate) {
    std::vector<uint8_t> b;
    b.reserve(44 + 2 * n);
    const uint32_t data = (uint32_t)(n * 2);
    b.insert(b.end(), {'R', 'I', 'F', 'F'});
    put32(b, 36 + data);
    b.insert(b.end(), {'W', 'A', 'V', 'E', 'f', 'm', 't', ' '});
    put32(b, 16);
    put16(b, 1);
    put16(b, 1);
    put32(b, (uint32_t)sample_rate);
    put32(b, (uint32_t)sample_rate * 2);
    put16(b, 2);
    put16(b, 16);
    b.insert(b.end(), {'d', 'a', 't', 'a'});
    put32(b, data);
    return b;
}

// RIFF/WAVE PCM16 mono image: 44-byte header then int16(clamp(s * 32767)) truncated.
std::vector<uint8_t> wav_bytes(const float *s, size_t n, int sample_rate) {
    std::vector<uint8_t> b = wav_header(n, sample_rate);
    for (size_t i = 0; i < n; ++i) put16(b, (uint16_t)pcm16_sample(s[i]));
    return b;
}

bool wav_write_pcm16(const std::string &path, const int16_t *pcm, size_t n, int sample_rate) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    const std::vector<uint8_t> h = wav_header(n, sample_rate);
    f.write((const char *)h.data(), (std::streamsize)h.size());
    static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "WAV samples are little-endian");
    f.write((const char *)pcm, (std::streamsize)(n * 2));
    return f.good();
}
}  // namespace mio

bool wav_write(const std::string &path, const std::vector<float> &samples, int sample_rate) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    const std::vector<uint8_t> b = mio::wav_bytes(samples.data(), samples.size(), sample_rate);
    f.write((const char *)b.data(), (std::streamsize)b.size());
    return f.good();
}

// ---- C-ABI wrappers (tests / bench / FFI users)
extern "C" int mio_normalize_tts_text(const char *text, char *out, int cap, int *out_len) {
    MIO_REQUIRE(text && out && cap > 0, MIO_ERR_INVALID, "normalize: bad args");
    const std::string s = normalize_tts_text(text);
    if (out_len) *out_len = (int)s.size();
    MIO_REQUIRE((int)s.size() < cap, MIO_ERR_INVALID, "normalize: buffer too small (%zu)", s.size());
    std::memcpy(out, s.c_str(), s.size() + 1);
    return MIO_OK;
}

extern "C" int mio_parse_speech_tokens(const char *text, int32_t *codes, int cap, int *n) {
    MIO_REQUIRE(text && n, MIO_ERR_INVALID, "parse_speech_tokens: bad args");
    const std::vector<int> c = parse_speech_tokens(text);
    *n = (int)c.size();
    for (int i = 0; i < (int)c.size() && i < cap; ++i) codes[i] = c[i];
    return MIO_OK;
}

extern "C" int mio_wav_encode(const float *samples, int n, int sample_rate, uint8_t *out, int cap, int *out_len) {
    MIO_REQUIRE((samples || n == 0) && out_len && n >= 0, MIO_ERR_INVALID, "wav_encode: bad args");
    const std::vector<uint8_t> b = mio::wav_bytes(samples, (size_t)n, sample_rate);
    *out_len = (int)b.size();
    MIO_REQUIRE(out && (int)b.size() <= cap, MIO_ERR_INVALID, "wav_encode: buffer too small (%zu)", b.size());
    std::memcpy(out, b.data(), b.size());
    return MIO_OK;
}
