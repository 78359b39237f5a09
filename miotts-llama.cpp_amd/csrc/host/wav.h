// WAV image helpers shared by wav_write (wav-writer.cpp:24-44 restated in text.cpp) and the
// device PCM epilogue path of TestToSpeech::synthesize_to_file (tts.cpp).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mio {
// 44-byte RIFF/WAVE PCM16 mono header for n samples (wav-writer.cpp:29-37).
std::vector<uint8_t> wav_header(size_t n, int sample_rate);
// Header + int16(clamp(s * 32767)) samples: the bytes wav_write produces.
std::vector<uint8_t> wav_bytes(const float *s, size_t n, int sample_rate);
// Header + already-converted PCM16 samples (mio_hip_pcm_finish output) to `path`.
bool wav_write_pcm16(const std::string &path, const int16_t *pcm, size_t n, int sample_rate);
}  // namespace mio
