"""CPU: the C codec oracle (oracle/codec_ref.c) against an independent numpy restatement of
miocodec_decode (tests/np_codec.py), stage by stage, for the F32 and the
F16 synthetic codecs (presets 1 / 2: the same tiny topology, matrices stored F32 / F16).

Both follow the reference graph (miocodec.cpp:204-420, 599-737) in ggml CPU semantics; they
share no code. numpy computes in float64, the oracle in float32, so the pure-f32 stages agree
to ~2e-7 (embedding, prenet, ConvT of the F32 codec: bound 1e-5). Where ggml rounds to f16
(conv_1d's im2col input from the first ResNet on; every F16 matrix's input in the F16 codec)
ulp-level differences flip a few f16 roundings (one f16 ulp = 4.9e-4 relative), measured
<= 1.6e-3 relative RMS at the spectrogram: bound 5e-3 per stage. A semantic error does not
hide under that: the RoPE pairing of the prenet swapped (adjacent -> NEOX halves) moves the
prenet output by > 1e-1 (last test).
"""
import numpy as np
import pytest

import miotts_amd as m
import np_codec
import pyoracle


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("npcodec")
    return {"f32": m.synth_codec(str(d / "c32.gguf"), 1, 1), "f16": m.synth_codec(str(d / "c16.gguf"), 2, 1),
            "emb": m.read_voice(m.synth_voice(str(d / "v.emb.gguf"), 7))}


@pytest.mark.parametrize("kind,T", [("f32", 1), ("f32", 9), ("f32", 40), ("f16", 1), ("f16", 9), ("f16", 40)])
def test_codec_stages_match_numpy_restatement(files, kind, T):
    path, emb = files[kind], files["emb"]
    oc, nc = pyoracle.Codec(path), np_codec.Codec(path)
    codes = (np.arange(T) * 7919 + 13) % 12800
    st = nc.stages(codes, emb)
    assert len(st) == oc.n_stages
    for i, a in enumerate(st):
        b = oc.decode_stage(codes, emb, i, 18 * T * 512 + 4096)
        assert a.shape == b.shape, (i, a.shape, b.shape)
        bound = 1e-5 if (kind == "f32" and i <= 2) else 5e-3
        assert _rel(a, b) <= bound, (kind, T, i, _rel(a, b))


def test_numpy_codec_detects_a_rope_pairing_error(files, monkeypatch):
    path, emb = files["f32"], files["emb"]
    oc, nc = pyoracle.Codec(path), np_codec.Codec(path)
    codes = (np.arange(12) * 7919 + 13) % 12800

    def neox(x, S, hd):  # the other ggml RoPE mode: pairs (i, i + hd/2)
        y = np_codec.Codec.rope(nc, np.concatenate([x[..., :hd // 2, None], x[..., hd // 2:, None]], -1)
                                .reshape(x.shape), S, hd)
        return np.concatenate([y[..., 0::2], y[..., 1::2]], -1)

    monkeypatch.setattr(nc, "rope", neox)
    assert _rel(nc.stages(codes, emb)[1], oc.decode_stage(codes, emb, 1, 12 * 512)) > 1e-1
