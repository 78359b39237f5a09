// C-ABI of the GGUF tokenizer (csrc/host/tokenizer.h), for host-side callers and tests.
#include <cstring>
#include <string>

#include "common.h"
#include "gguf.h"
#include "mio_hip.h"
#include "tokenizer.h"

struct mio_tokenizer {
    mio::BpeTokenizer t;
};

extern "C" int mio_tokenizer_load(const char *gguf_path, mio_tokenizer **out) {
    MIO_REQUIRE(gguf_path && out, MIO_ERR_INVALID, "tokenizer_load: null argument");
    mio::GgufFile g;
    if (!g.open(gguf_path)) return MIO_ERR_IO;
    auto *t = new mio_tokenizer();
    if (!t->t.load(g)) {
        delete t;
        return MIO_ERR_FORMAT;
    }
    *out = t;
    return MIO_OK;
}

extern "C" void mio_tokenizer_free(mio_tokenizer *t) { delete t; }

extern "C" int mio_tokenizer_info(const mio_tokenizer *t, int *info) {
    MIO_REQUIRE(t && info, MIO_ERR_INVALID, "tokenizer_info: null argument");
    info[0] = t->t.n_vocab(), info[1] = t->t.bos(), info[2] = t->t.eos(), info[3] = t->t.special_id("<|im_end|>");
    return MIO_OK;
}

extern "C" int mio_tokenize(const mio_tokenizer *t, const char *text, int add_special, int parse_special,
                            int32_t *out, int cap, int *n) {
    MIO_REQUIRE(t && text && n && (out || cap == 0), MIO_ERR_INVALID, "tokenize: null argument");
    const std::vector<int32_t> ids = t->t.tokenize(text, add_special != 0, parse_special != 0);
    *n = (int)ids.size();
    MIO_REQUIRE((int)ids.size() <= cap, MIO_ERR_INVALID, "tokenize: %d tokens > capacity %d", (int)ids.size(), cap);
    if (!ids.empty()) std::memcpy(out, ids.data(), ids.size() * 4);
    return MIO_OK;
}

extern "C" int mio_token_piece(const mio_tokenizer *t, int32_t id, char *out, int cap, int *len) {
    MIO_REQUIRE(t && len && (out || cap == 0), MIO_ERR_INVALID, "token_piece: null argument");
    const std::string p = t->t.piece(id);
    *len = (int)p.size();
    MIO_REQUIRE((int)p.size() <= cap, MIO_ERR_INVALID, "token_piece: %d bytes > capacity %d", (int)p.size(), cap);
    if (!p.empty()) std::memcpy(out, p.data(), p.size());
    return MIO_OK;
}

// Streaming cadence of n_tokens speech tokens (one code each): decode calls and decoded
// codes of the commit policy (csrc/host/stream_policy.h), for the KAT of SURVEY 8c.
#include "stream_policy.h"

extern "C" int mio_stream_cadence(int n_tokens, int *decode_calls, int64_t *decoded_codes) {
    MIO_REQUIRE(n_tokens >= 0 && decode_calls && decoded_codes, MIO_ERR_INVALID, "stream_cadence: bad args");
    mio::StreamPolicy p;
    int calls = 0;
    int64_t codes = 0;
    auto check = [&](size_t n, bool final_) {
        size_t t = 0;
        if (n == 0 || !p.plan(n, final_, &t)) return;
        ++calls, codes += (int64_t)n;
        p.committed = t;
    };
    for (int g = 1; g <= n_tokens; ++g)
        if (g % mio::StreamPolicy::kCheckInterval == 0) check((size_t)g, false);
    check((size_t)n_tokens, true);
    *decode_calls = calls;
    *decoded_codes = codes;
    return MIO_OK;
}
