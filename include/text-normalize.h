// Japanese TTS text normalisation (drop-in for the reference's text-normalize.h:7).
#pragma once

#include <string>

// Applies the JP punctuation/whitespace normalisation when >= 10% of the non-space code
// points are Japanese (text-normalize.cpp:78-97); otherwise returns the text unchanged.
std::string normalize_tts_text(const std::string & text);
