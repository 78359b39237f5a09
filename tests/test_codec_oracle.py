"""CPU: synthetic codec files + the codec oracle (oracle/codec_ref.c).

The codec oracle is "parity unpinned" (ggml is absent): these tests pin
what can be pinned without ggml — file format/names, stage shapes
and lengths (miocodec.cpp:538-549), the f16 rounding helper used for ggml's conv_1d
im2col, determinism, and the 20-code fixture of compare_codec.py:50-51.
"""
import numpy as np
import pytest

import miotts_amd as m
from miotts_amd import gguf_np
import pyoracle

FIXTURE_20 = [12287, 11619, 11774, 12223, 2490, 826, 2257, 1668, 1219, 2319,
              9994, 12683, 12745, 4215, 12478, 8800, 8696, 375, 1406, 12396]


@pytest.fixture(scope="session")
def codec_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("codec")
    tiny = m.synth_codec(str(d / "codec_tiny.gguf"), preset=1, seed=1)
    full = m.synth_codec(str(d / "codec_full.gguf"), preset=0, seed=1)
    voice = m.synth_voice(str(d / "voice.emb.gguf"), seed=7)
    return {"tiny": tiny, "full": full, "voice": voice}


def test_synth_codec_format(codec_files):
    g = gguf_np.GGUFReader(codec_files["full"])
    assert g.kv["general.architecture"] == "miocodec"
    assert g.kv["miocodec.n_fft"] == 392 and g.kv["miocodec.hop_length"] == 98
    assert g.kv["embedding_length_out"] == 394
    assert g.kv["miocodec.samples_per_token"] == 1764
    assert g.tensor("token_embd").ne == [768, 12800]
    assert g.tensor("wave_prenet.blk.5.attn_q.weight").ne == [768, 768]
    assert g.tensor("wave_upsample.weight").ne == [2, 512, 512]
    assert g.tensor("wave_prior.1.conv2.weight").ne == [3, 512, 512]
    assert g.tensor("wave_decoder.blk.7.attn_cond.weight").ne == [128, 1536]
    assert g.tensor("wave_decoder.norm_cond.weight").ne == [128, 1024]
    assert g.tensor("wave_upsampler.up.0.weight").ne == [7, 256, 512]
    assert g.tensor("istft_head.out.weight").ne == [512, 394]
    assert list(g.tensor("miocodec.wave_upsampler.factors").array()) == [3, 3]
    v = m.read_voice(codec_files["voice"])
    assert v.shape == (128,) and np.isfinite(v).all()
    gv = gguf_np.GGUFReader(codec_files["voice"])
    assert gv.kv["general.architecture"] == "mio-embedding"
    assert gv.tensors[0].name == "mio.global_embedding"


def test_f16_round_matches_ieee_rne():
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.standard_normal(2000).astype(np.float32) * 10,
                         np.array([0.0, -0.0, 65504.0, 65519.0, 65520.0, 1e-8, 6.1e-5, 5.96e-8,
                                   -3.0e-6, 2049.0, 2051.0, 1.0 + 2 ** -11], np.float32)])
    o = pyoracle.oracle()
    got = np.array([o.mo_f16_round(float(x)) for x in xs], np.float32)
    want = xs.astype(np.float16).astype(np.float32)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("which", ["tiny", "full"])
def test_oracle_codec_stage_shapes(codec_files, which):
    c = pyoracle.Codec(codec_files[which])
    emb = m.read_voice(codec_files["voice"])
    T = 5
    codes = np.arange(T, dtype=np.int32) * 997 % 12800
    assert c.n_stages == 8 + c.up_stages
    shapes = []
    for st in range(c.n_stages):
        a = c.decode_stage(codes, emb, st, 18 * T * 512 + 1024)
        shapes.append(a.shape)
        assert np.isfinite(a).all(), st
    assert shapes[0][0] == T and shapes[1][0] == T
    assert shapes[2][0] == 2 * T and shapes[5][0] == 2 * T
    assert shapes[6][0] == 6 * T and shapes[7][0] == 18 * T
    assert shapes[-1] == (18 * T, 394)
    spec = c.decode(codes, emb)
    pcm = pyoracle.istft(spec)
    assert pcm.size == T * 1764  # miocodec.cpp:546-548, samples_per_token


def test_oracle_codec_fixture20_deterministic(codec_files):
    c = pyoracle.Codec(codec_files["full"])
    emb = m.read_voice(codec_files["voice"])
    a = c.decode(FIXTURE_20, emb)
    b = c.decode(FIXTURE_20, emb)
    assert a.shape == (360, 197, 2)
    assert np.array_equal(a, b)
    mag = np.hypot(a[..., 0], a[..., 1])
    assert mag.max() <= 100.0 + 1e-3  # clamp(exp(.), 0, 100), miocodec.cpp:735


def test_oracle_codec_rejects_bad_codes(codec_files):
    c = pyoracle.Codec(codec_files["tiny"])
    emb = np.zeros(128, np.float32)
    with pytest.raises(RuntimeError):
        c.decode([0, 12800], emb)
    with pytest.raises(RuntimeError):
        c.decode([-1], emb)
