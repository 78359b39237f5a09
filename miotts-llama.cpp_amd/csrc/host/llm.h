// LLM decode runner on one MI355X (replaces the llama.cpp context used by
// TestToSpeech::run_llm, test-to-speech.cpp:94-199 / :435-614).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

struct mio_hip_device;
struct mio_hip_llm;

namespace mio {

struct LlmInfo {
    int n_vocab, n_embd, n_layer, n_head, n_kv, head_dim, n_ff, n_ctx;
};

struct SamplingParams {
    float temperature = 0.8f;
    uint64_t seed = 42;      // llama_sampler_init_dist(42), test-to-speech.cpp:130
    int allow_lo = 0, allow_hi = -1;  // restrict sampling to [lo, hi) (-1 = n_vocab)
    int eos0 = -1, eos1 = -1;
};

// Incremental generation on the device: begin() seeds the prompt, run() enqueues decode
// steps (one hipGraph replay each), poll() syncs and returns the tokens produced so far.
int llm_begin(mio_hip_llm *m, const int32_t *prompt, int n_prompt, int max_new,
              const SamplingParams &sp);
int llm_run(mio_hip_llm *m, int n_steps);
// Every remaining step, stopping (at step-graph granularity) once the device has flagged an
// end token to the host; then the flush sampler and a snapshot for llm_poll.
int llm_run_to_end(mio_hip_llm *m);
int llm_graph_steps();
// Copies generated tokens [0, *n_out) and reports whether an end token was sampled.
int llm_poll(mio_hip_llm *m, std::vector<int32_t> &out, bool *done);
LlmInfo llm_info(const mio_hip_llm *m);
uint64_t llm_step_weight_bytes(const mio_hip_llm *m);

}  // namespace mio
