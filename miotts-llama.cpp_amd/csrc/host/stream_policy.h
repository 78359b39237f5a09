// Streaming commit policy of TestToSpeech::synthesize_stream_profiled
// (test-to-speech.cpp:496-571): check every 20 generated tokens, keep the newest 32 codes
// back, decode (all codes so far) only once at least 24 new codes can be committed; the
// final check commits everything.
#pragma once

#include <cstddef>

namespace mio {

struct StreamPolicy {
    static constexpr int kCheckInterval = 20;     // stream_check_interval (:496)
    static constexpr size_t kHoldback = 32;       // holdback_codes (:497)
    static constexpr size_t kMinCommit = 24;      // min_commit_step_codes (:498)
    size_t committed = 0;

    // With n_codes parsed so far: true if this check decodes, with the new commit target in
    // *target (codes [committed, *target) are emitted, then committed = *target).
    bool plan(size_t n_codes, bool final_, size_t *target) const {
        const size_t t = final_ ? n_codes : (n_codes > kHoldback ? n_codes - kHoldback : 0);
        *target = t;
        if (t <= committed) return false;
        if (!final_ && t - committed < kMinCommit) return false;
        return true;
    }
};

}  // namespace mio
