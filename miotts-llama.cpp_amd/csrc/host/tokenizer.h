// GGUF byte-level BPE tokenizer (tokenizer.ggml.model == "gpt2": Qwen2/Qwen3/Llama-3
// style vocabularies, which the MioTTS LLMs use). Replaces the llama_vocab calls of
// TestToSpeech::run_llm: llama_tokenize(text, add_special=true, parse_special=true)
// (test-to-speech.cpp:117-125), the "<|im_end|>" lookup (:150-159), llama_vocab_eos
// (:150) and llama_token_to_piece(..., special=true) (:173-176).
//
// Algorithm (the public GPT-2 / llama.cpp BPE scheme, restated):
//   1. split the text on special tokens (token_type CONTROL / USER_DEFINED), longest match;
//   2. pre-tokenize the remaining runs with the regex sequence of the vocabulary's
//      tokenizer.ggml.pre (llama.cpp's llm_tokenizer_bpe families: gpt2, default, qwen2,
//      llama3 / llama-bpe / lfm2, smollm; any other value is refused at load), evaluated on
//      code points with generated Unicode letter/number/punctuation classes;
//   3. map each piece's bytes through the GPT-2 byte->unicode table and apply the merges in
//      rank order; pieces are then looked up in the vocabulary (bytes as a fallback).
// Parity: llama.cpp is absent here; each pre-type is checked id for id against HuggingFace
// `tokenizers` with the same regex sequence (tests/test_tokenizer_hf.py).
//
// SPM vocabularies (tokenizer.ggml.model == "llama": SentencePiece pieces with scores and
// <0xXX> byte tokens, llama.cpp's llm_tokenizer_spm, restated): specials split as above; a
// text fragment gets a leading " " when tokenizer.ggml.add_space_prefix (default true) and it
// opens the text or follows a special token, every ' ' becomes U+2581; the fragment is split
// into UTF-8 characters and adjacent symbols are merged greedily, highest vocabulary score
// first (ties: leftmost), whenever their concatenation is a token; a final symbol that is not
// a token is resegmented into the two symbols it was merged from, and characters that form no
// token become their <0xXX> byte tokens. BOS is added by default (add_bos_token), EOS when
// add_eos_token. Pieces: U+2581 -> ' ', byte tokens -> the byte. Checked id for id against
// the `sentencepiece` package's BPE encoder on trained vocabularies (tests/test_tokenizer_spm.py).
//
// WPM vocabularies (tokenizer.ggml.model == "bert": WordPiece, llama.cpp's llm_tokenizer_wpm,
// restated): specials split as above; a fragment's code points are mapped to the first code
// point of their canonical decomposition (accents of precomposed letters drop) and lowercased;
// whitespace ends a word, control / format characters and U+FFFD are dropped, and punctuation,
// ASCII symbols and CJK ideographs become words of their own; each word, prefixed with U+2581,
// is split greedily into the longest vocabulary tokens (convert_hf_to_gguf writes a BERT
// vocabulary's word-initial tokens with that prefix and "##" continuations without it), and a
// word with an unmatched position becomes one UNK. [CLS] (BOS) opens and [SEP] closes the text
// by default. Checked id for id against HuggingFace `tokenizers`' BERT WordPiece
// (tests/test_tokenizer_wpm.py).
//
// UGM vocabularies (tokenizer.ggml.model == "t5": SentencePiece Unigram, llama.cpp's
// llm_tokenizer_ugm, restated): a fragment is normalized with the precompiled character map
// (tokenizer.ggml.precompiled_charsmap: sentencepiece's XOR-compressed double-array trie of
// input prefixes and their replacements, longest prefix first; user-defined tokens are kept as
// they are; invalid UTF-8 becomes U+FFFD), spaces become U+2581 with a prefix space
// (add_space_prefix) and runs merged (remove_extra_whitespaces); then the Viterbi best
// segmentation by summed token scores (user-defined tokens score 0; a code point no token
// covers is UNK at the lowest score - 10), consecutive UNKs merged. EOS added by default.
// Checked id for id against the `sentencepiece` package's Unigram encoder on vocabularies
// trained with its nmt_nfkc character map and with identity normalization
// (tests/test_tokenizer_ugm.py).
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace mio {

class GgufFile;

class BpeTokenizer {
public:
    // false + set_error when the GGUF has no usable tokenizer
    bool load(const GgufFile &g);

    std::vector<int32_t> tokenize(const std::string &text, bool add_special, bool parse_special) const;
    // token text as llama_token_to_piece(special=true) renders it (bytes for normal tokens)
    std::string piece(int32_t id) const;
    int32_t eos() const { return eos_; }
    int32_t bos() const { return bos_; }
    // id of a single-token special text, -1 when it is not one token
    int32_t special_id(const std::string &text) const;
    int n_vocab() const { return (int)tokens_.size(); }

private:
    void bpe(const std::string &piece, std::vector<int32_t> &out) const;
    void spm(const std::string &text, std::vector<int32_t> &out) const;
    bool load_spm(const GgufFile &g);
    void wpm(const std::string &text, std::vector<int32_t> &out) const;
    bool load_wpm(const GgufFile &g);
    void ugm(const std::string &text, std::vector<int32_t> &out) const;
    bool load_ugm(const GgufFile &g);
    std::string ugm_normalize(const std::string &text) const;
    // one normalization step at byte i: the replacement and the input bytes it consumes
    std::pair<std::string, size_t> ugm_prefix(const std::string &text, size_t i) const;
    // tokens, types, id map, special tokens (shared by the SPM / WPM loaders)
    void load_vocab(const GgufFile &g);
    void pretokenize(const std::string &text, std::vector<std::string> &pieces) const;

    std::vector<std::string> tokens_;
    std::vector<int32_t> types_;
    std::unordered_map<std::string, int32_t> id_;
    std::unordered_map<std::string, int> merge_rank_;  // "left right" -> rank
    std::unordered_map<std::string, int32_t> special_;  // special text -> id
    std::vector<size_t> special_lens_;                  // distinct lengths, descending
    std::string byte_enc_[256];                          // byte -> UTF-8 of its unicode stand-in
    std::unordered_map<uint32_t, uint8_t> byte_dec_;     // stand-in code point -> byte
    int32_t eos_ = -1, bos_ = -1, unk_ = -1;
    bool add_bos_ = false, add_eos_ = false;
    // SPM vocabularies
    bool spm_ = false, add_space_prefix_ = true;
    // WPM vocabularies: [SEP] after the text (add_sep), longest token in bytes
    bool wpm_ = false, add_sep_ = true;
    int32_t sep_ = -1;
    size_t max_tok_len_ = 0;
    // UGM vocabularies: the character map (double-array units, replacement strings), the
    // matchable tokens (NORMAL, USER_DEFINED, UNUSED) and user-defined lengths, UNK's score
    bool ugm_ = false, remove_extra_ws_ = false, escape_ws_ = true, ws_suffix_ = false;
    std::vector<uint32_t> xcda_;
    std::string repl_;
    std::unordered_map<std::string, int32_t> ugm_tok_;
    std::unordered_map<std::string, int32_t> user_def_;
    std::vector<size_t> user_def_lens_;  // descending
    float unk_score_ = 0.0f;
    std::vector<float> scores_;
    int32_t byte_tok_[256];
    // pre-tokenizer family (llama.cpp LLAMA_VOCAB_PRE_TYPE_*): the regex sequence of step 2
    enum class Pre { Gpt2, Default, Qwen2, Llama3, Smollm };
    Pre pre_ = Pre::Gpt2;
};

}  // namespace mio
