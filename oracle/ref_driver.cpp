// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// extern "C" driver over the reference's own translation units that compile in
// this container: istft.cpp, token-parser.cpp, wav-writer.cpp,
// text-normalize.cpp. They are compiled in place from /root/reference/src by
// oracle/Makefile (target `ref`) into oracle/_ref/libmioref.so. Nothing is
// copied; no header or library of the reference is stubbed. miocodec.cpp and
// test-to-speech.cpp need ggml/llama headers that are absent (F1) and are NOT
// built. Used only to (a) pin the C oracle and (b) generate tests/golden/.
#include "istft.h"
#include "text-normalize.h"
#include "token-parser.h"
#include "wav-writer.h"

#include <cstring>
#include <string>
#include <vector>

extern "C" {

// istft.h:38-42 with istft_cache(n_fft, win_length) as test-to-speech.cpp:67 builds it.
int ref_istft(const float *spec, int n_frames, int n_fft, int win_length, int hop, float *out) {
    istft_cache cache(n_fft, win_length);
    std::vector<float> y = istft(spec, n_frames, hop, cache);
    if (!y.empty()) std::memcpy(out, y.data(), y.size() * sizeof(float));
    return (int)y.size();
}

// token-parser.h:8
int ref_parse_speech_tokens(const char *text, int *out, int cap) {
    std::vector<int> c = parse_speech_tokens(std::string(text));
    int n = (int)c.size();
    for (int i = 0; i < n && i < cap; i++) out[i] = c[i];
    return n;
}

// text-normalize.h:7
int ref_normalize_tts_text(const char *text, char *out, int cap) {
    std::string s = normalize_tts_text(std::string(text));
    int n = (int)s.size();
    if (n < cap) {
        std::memcpy(out, s.data(), n);
        out[n] = 0;
    }
    return n;
}

// wav-writer.h:6
int ref_wav_write(const char *path, const float *samples, int n, int sample_rate) {
    std::vector<float> v(samples, samples + n);
    return wav_write(std::string(path), v, sample_rate) ? 1 : 0;
}
}
