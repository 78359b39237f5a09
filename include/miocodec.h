// Drop-in for the reference miocodec.h (miocodec.h:10-43): same functions and semantics.
// miocodec_load uploads the decoder once to the process's default MI355X (MIO_DEVICE, else
// LOCAL_RANK, else 0); miocodec_decode runs the gfx950 codec kernels and returns the
// spectrogram in host memory. Errors: nullptr / empty vector + a message on stderr.
#pragma once

#include <string>
#include <vector>

struct miocodec_context;

// Load MioCodec model from GGUF file. Returns nullptr on failure.
miocodec_context * miocodec_load(const std::string & model_path);

// Free MioCodec context.
void miocodec_free(miocodec_context * ctx);

// Decode speech token codes (0..12799) to the spectrogram, interleaved [real, imag] per bin
// per frame: [n_frames][n_freq*2]; audio_length is informational (0 = n_codes *
// samples_per_token), as in miocodec.cpp:546-552. out_n_frames may be null.
std::vector<float> miocodec_decode(
    miocodec_context * ctx,
    const int * codes,
    int n_codes,
    const float * global_emb,
    int audio_length,
    int * out_n_frames);

// Model parameter accessors
int   miocodec_sample_rate(const miocodec_context * ctx);
int   miocodec_n_fft(const miocodec_context * ctx);
int   miocodec_hop_length(const miocodec_context * ctx);
int   miocodec_samples_per_token(const miocodec_context * ctx);

// Load a voice embedding from .emb.gguf file (first tensor, F32). Returns it, or empty.
std::vector<float> load_voice_embedding(const std::string & path);

// Print all tensor names in a GGUF file (for debugging).
void miocodec_print_tensors(const std::string & path);
