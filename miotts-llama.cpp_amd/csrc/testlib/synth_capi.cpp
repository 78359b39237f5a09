// C-ABI: synthetic model files (no real GGUFs exist offline).
#include "common.h"
#include "synth.h"

extern "C" int mio_synth_codec_gguf(const char *path, int preset, uint64_t seed) {
    MIO_REQUIRE(path && preset >= 0 && preset <= 3, MIO_ERR_INVALID, "synth_codec: bad args");
    mio::SynthCodecCfg c = mio::synth_codec_preset(preset);
    c.seed = seed;
    MIO_REQUIRE(mio::synth_write_codec(path, c), MIO_ERR_IO, "synth_codec: cannot write %s", path);
    return MIO_OK;
}

extern "C" int mio_synth_voice_gguf(const char *path, uint64_t seed) {
    MIO_REQUIRE(path, MIO_ERR_INVALID, "synth_voice: null path");
    MIO_REQUIRE(mio::synth_write_voice(path, seed), MIO_ERR_IO, "synth_voice: cannot write %s", path);
    return MIO_OK;
}

extern "C" int mio_synth_llm_gguf(const char *path, int preset, uint64_t seed) {
    MIO_REQUIRE(path && preset >= 0 && preset <= 12, MIO_ERR_INVALID, "synth_llm: bad args");
    mio::SynthLlmCfg c = mio::synth_llm_preset(preset);
    c.seed = seed;
    MIO_REQUIRE(mio::synth_write_llm(path, c), MIO_ERR_IO, "synth_llm: cannot write %s", path);
    return MIO_OK;
}
