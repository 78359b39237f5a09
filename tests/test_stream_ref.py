"""CPU: the C restatement of the streaming emission (oracle/stream_ref.c,
test-to-speech.cpp:367-417,496-571) reproduces the reference cadence (SURVEY 8c KAT 4:
100 speech tokens -> 3 full decodes of 60/100/100 codes) and emits every sample once, in
chunk_samples pieces; with no earlier piece the first emission is the decode itself."""
import numpy as np
import pytest

import miotts_amd as m
import pyoracle


@pytest.fixture(scope="module")
def tiny(tmp_path_factory):
    d = tmp_path_factory.mktemp("stream_ref")
    codec = pyoracle.Codec(m.synth_codec(str(d / "codec_tiny.gguf"), 1, 1))
    return codec, m.read_voice(m.synth_voice(str(d / "voice.emb.gguf"), 7))


def test_stream_ref_cadence_and_chunks(tiny):
    codec, emb = tiny
    codes = (np.arange(100) * 7919) % 12800
    out, chunks, n_dec = pyoracle.stream_emit(codec, emb, codes, 20, 32, 24, 4096)
    assert n_dec == 3
    assert out.size == int(chunks.sum()) == 100 * codec.samples_per_token
    assert (chunks[:-1] <= 4096).all() and chunks.max() == 4096
    # first commit: codes [0, 28) of the 60-code decode, no crossfade before it
    first = codec.decode_pcm(codes[:60], emb)
    n0 = int(round(28 * first.size / 60))
    assert np.array_equal(out[:4096], first[:4096]) and n0 == 28 * codec.samples_per_token


def test_stream_ref_small_and_empty(tiny):
    codec, emb = tiny
    out, chunks, n_dec = pyoracle.stream_emit(codec, emb, np.arange(10), 20, 32, 24, 4096)
    assert n_dec == 1 and out.size == 10 * codec.samples_per_token  # only the final check decodes
    out, chunks, n_dec = pyoracle.stream_emit(codec, emb, np.zeros(0, np.int32), 20, 32, 24, 4096)
    assert n_dec == 0 and out.size == 0 and chunks.size == 0
