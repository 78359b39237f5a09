// 16-bit mono PCM WAV writer (drop-in for the reference's wav-writer.h:6).
#pragma once

#include <string>
#include <vector>

bool wav_write(const std::string & path, const std::vector<float> & samples, int sample_rate);
