// Speech-token parser (drop-in for the reference's token-parser.h:8).
#pragma once

#include <string>
#include <vector>

// Extracts N from every well-formed "<|s_N|>" in `text`, in order.
std::vector<int> parse_speech_tokens(const std::string & text);
