"""GPU parity: HIP MioCodec decoder (csrc/host/codec.cpp + csrc/hip/codec_kernels.hip)
vs the C oracle (oracle/codec_ref.c), stage by stage and end to end through the iSTFT.

Tolerances. The path is float32 except where the reference itself rounds to f16
(ggml conv_1d casts the kernel AND the im2col input to f16, miocodec.cpp:382-386).
The GPU reorders f32 sums (MFMA fma chains, tree reductions): pure-f32 stages agree to
~2e-6 relative (measured, tools/codec_err_profile.py). At each f16 rounding point an
ulp-level f32 difference flips ~0.2% of the f16 roundings (one f16 ulp = 4.9e-4), so
after the first ResNet the stage agreement is ~7e-5 and grows to ~4e-4 at the
spectrogram (exp() of the log-magnitude). Hence:
  * per stage : RMS(diff) <= 1e-3 * RMS(ref) and max|diff| <= 5e-3 * max|ref|
  * PCM       : RMS(diff) <= 1e-4 absolute (north star) and <= 1e-3 * RMS(ref)
                (measured: 5.5e-5 absolute at ref RMS 0.13, T = 20..700)
"""
import numpy as np
import pytest

import miotts_amd as m
import pyoracle

pytestmark = pytest.mark.gpu

FIXTURE_20 = [12287, 11619, 11774, 12223, 2490, 826, 2257, 1668, 1219, 2319,
              9994, 12683, 12745, 4215, 12478, 8800, 8696, 375, 1406, 12396]


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("codec_gpu")
    return {"tiny": m.synth_codec(str(d / "tiny.gguf"), 1, 1),
            "full": m.synth_codec(str(d / "full.gguf"), 0, 1),
            "voice": m.synth_voice(str(d / "voice.emb.gguf"), 7)}


@pytest.fixture(scope="module")
def emb(files):
    return m.read_voice(files["voice"])


def _stage_close(g, o, name, rms_bound=1e-3, max_bound=5e-3):
    assert g.shape == o.shape, (name, g.shape, o.shape)
    d = g.astype(np.float64) - o.astype(np.float64)
    rms_ref = np.sqrt(np.mean(o.astype(np.float64) ** 2)) + 1e-30
    rel_rms = np.sqrt(np.mean(d * d)) / rms_ref
    rel_max = np.abs(d).max() / (np.abs(o).max() + 1e-30)
    assert rel_rms <= rms_bound and rel_max <= max_bound, f"{name}: rel_rms={rel_rms:.3g} rel_max={rel_max:.3g}"


def _pcm_close(g, o):
    assert g.shape == o.shape
    d = g.astype(np.float64) - o.astype(np.float64)
    rms = np.sqrt(np.mean(d * d))
    rms_ref = np.sqrt(np.mean(o.astype(np.float64) ** 2))
    assert rms <= 1e-4 and rms <= 1e-3 * rms_ref, f"PCM rms diff {rms:.3g} (ref rms {rms_ref:.3g})"
    return rms


@pytest.mark.parametrize("T", [1, 2, 7, 33])
def test_codec_stages_tiny(device, files, emb, T):
    gc = m.Codec(device, files["tiny"])
    oc = pyoracle.Codec(files["tiny"])
    codes = (np.arange(T, dtype=np.int64) * 7919 + 13) % 12800
    cap = 18 * T * 512 + 4096
    for st in range(oc.n_stages):
        _stage_close(gc.decode_stage(codes, emb, st, cap), oc.decode_stage(codes, emb, st, cap),
                     f"T={T} stage {st}")


def test_codec_stages_full_fixture20(device, files, emb):
    gc = m.Codec(device, files["full"])
    oc = pyoracle.Codec(files["full"])
    cap = 18 * 20 * 512 + 4096
    for st in range(oc.n_stages):
        _stage_close(gc.decode_stage(FIXTURE_20, emb, st, cap),
                     oc.decode_stage(FIXTURE_20, emb, st, cap), f"stage {st}")
    spec_g = gc.decode(FIXTURE_20, emb)
    spec_o = oc.decode(FIXTURE_20, emb)
    _stage_close(spec_g, spec_o, "spec")
    pcm_g = gc.decode_pcm(FIXTURE_20, emb)
    assert pcm_g.size == 20 * 1764
    _pcm_close(pcm_g, pyoracle.istft(spec_o))


def test_codec_pcm_full_T700(device, files, emb):
    """BASELINE size: T = 700 codes -> 1,234,800 PCM samples, PCM within 1e-4 RMS."""
    gc = m.Codec(device, files["full"])
    oc = pyoracle.Codec(files["full"])
    codes = np.random.default_rng(1234).integers(0, 12800, 700).astype(np.int32)
    pcm_g = gc.decode_pcm(codes, emb)
    assert pcm_g.size == 1234800
    rms = _pcm_close(pcm_g, oc.decode_pcm(codes, emb))
    print(f"T=700 PCM rms diff {rms:.3g}")


def test_codec_device_buffers_and_repeat(device, files, emb):
    gc = m.Codec(device, files["tiny"])
    codes = np.arange(40, dtype=np.int32) * 31 % 12800
    a = gc.decode_pcm(codes, emb)
    d_codes = device.upload(codes)
    d_emb = device.upload(emb)
    d_out = device.empty((40 * 1764 + 392,), np.float32)
    n = gc.decode_pcm_device(d_codes, 40, d_emb, d_out)
    device.sync()
    assert n == 40 * 1764
    b = d_out.numpy()[:n]
    assert np.array_equal(a, b)  # deterministic: same kernels, same order


def test_codec_batch_equals_single(device, files, emb):
    """mio_hip_codec_decode_pcm_batch (the batched bench line and batch synthesis): ragged
    utterances decoded concurrently on up to 4 streams, each lane in its own workspace and
    reused for a second utterance, give each utterance's single-decode PCM bit for bit (same
    kernels, same tiling; test-to-speech.cpp:264-287 runs every utterance on its own)."""
    gc = m.Codec(device, files["full"])
    rng = np.random.default_rng(5)
    lens = [33, 7, 120, 60, 2, 95]
    codes = [rng.integers(0, 12800, n).astype(np.int32) for n in lens]
    got = gc.decode_pcm_batch(codes, emb)
    for c, g in zip(codes, got):
        want = gc.decode_pcm(c, emb)
        assert g.shape == want.shape and np.array_equal(g, want), len(c)


def test_codec_rejects_bad_codes(device, files, emb):
    gc = m.Codec(device, files["tiny"])
    with pytest.raises(m.HipError):
        gc.decode([5, 12800], emb)


def test_codec_incremental_streaming_decode(device, files, emb):
    """f3 (test-to-speech.cpp:526-529 re-decodes every committed prefix): an incremental
    decode reuses the prenet rows of the previous one whose +-192-code receptive field was
    complete (6 layers x window/2), and recomputes the prenet only from 192 codes before
    them. Its PCM equals the full decode up to f32 summation order (the recomputed window
    picks its own GEMM tiling) and the oracle within the PCM bound."""
    gc = m.Codec(device, files["full"])
    oc = pyoracle.Codec(files["full"])
    radius = 6 * (65 // 2)
    codes = np.random.default_rng(77).integers(0, 12800, 420).astype(np.int32)
    prev = 0
    for n in (60, 100, 260, 300, 420):  # the streaming cadence's growing prefixes
        inc = gc.decode_pcm(codes[:n], emb, incremental=True)
        assert gc.last_reused() == max(0, prev - radius)
        full = gc.decode_pcm(codes[:n], emb)  # a plain decode neither reads nor moves the cache
        d = inc.astype(np.float64) - full
        assert np.sqrt(np.mean(d * d)) <= 1e-5 * np.sqrt(np.mean(full.astype(np.float64) ** 2)), n
        prev = n
    _pcm_close(inc, oc.decode_pcm(codes, emb))
    # a different code at 300: rows whose receptive field reaches it are recomputed
    edited = codes.copy()
    edited[300] = (edited[300] + 1) % 12800
    inc = gc.decode_pcm(edited, emb, incremental=True)
    assert gc.last_reused() == 300 - radius
    full = gc.decode_pcm(edited, emb)
    d = inc.astype(np.float64) - full
    assert np.sqrt(np.mean(d * d)) <= 1e-5 * np.sqrt(np.mean(full.astype(np.float64) ** 2))


@pytest.mark.parametrize("preset,T", [(2, 7), (2, 33), (3, 20)])
def test_codec_f16_weights(device, tmp_path, emb, preset, T):
    """A codec GGUF whose matrices are F16 (synthetic presets 2 / 3: every tensor of >= 2 dims
    F16): ggml's mul_mat and conv_transpose_1d then convert the activation to the F16
    vec_dot_type (miocodec.cpp:205-209 linear, :624 / :685 ConvT), which the GPU GEMMs do in
    their operand staging (GemmArgs::a_f16) and the oracle before its dot products (whose F16
    path tests/test_np_codec.py checks against the numpy restatement). Every F16 linear rounds
    its input, so last-bit differences upstream that cross an f16 rounding boundary move a
    value by one f16 ulp (5e-4 relative) and the chained stages drift further than in the F32
    codec (measured 1.0e-3 rms at stage 8, T=33): stages before the spectrogram within 3e-3
    rms / 1e-2 max. The spectrogram head rounds its input to f16 and then
    exponentiates, so one-ulp input flips (last-bit differences upstream crossing an f16
    rounding boundary) grow into ~1e-3 of the output: there the GPU is checked teacher-forced
    (numpy head with f16 rounding on the GPU's own stage input: tight; without the rounding:
    measurably farther, so the rounding is proven present) and chained against the oracle
    at 5e-3; PCM at 5e-3 of its rms."""
    import np_codec
    path = m.synth_codec(str(tmp_path / f"f16_{preset}.gguf"), preset, 1)
    from miotts_amd import gguf_np
    r = gguf_np.GGUFReader(path)
    assert r.tensor("wave_prenet.blk.0.attn_q.weight").type == 1 and r.tensor("wave_upsample.weight").type == 1
    gc = m.Codec(device, path)
    oc = pyoracle.Codec(path)
    codes = (np.arange(T, dtype=np.int64) * 7919 + 13) % 12800
    cap = 18 * T * 512 + 4096
    last = oc.n_stages - 1
    for st in range(last):
        _stage_close(gc.decode_stage(codes, emb, st, cap), oc.decode_stage(codes, emb, st, cap),
                     f"f16 preset {preset} T={T} stage {st}", 3e-3, 1e-2)
    g_in = gc.decode_stage(codes, emb, last - 1, cap).astype(np.float64)
    g_spec = gc.decode_stage(codes, emb, last, cap).astype(np.float64)
    nc = np_codec.Codec(path)
    w, h16 = nc.W("istft_head.out.weight")
    assert h16
    bias = nc.W("istft_head.out.bias")[0]
    nf = nc.n_freq

    def head(x):
        y = x @ w.T + bias
        mag = np.clip(np.exp(y[:, :nf]), 0.0, 100.0)
        return np.stack([mag * np.cos(y[:, nf:]), mag * np.sin(y[:, nf:])], axis=-1).reshape(len(y), 2 * nf)

    def rel(a, b):
        return float(np.sqrt(np.mean((a - b) ** 2)) / (np.sqrt(np.mean(b * b)) + 1e-30))

    e_round = rel(g_spec, head(np_codec._h(g_in)))
    e_plain = rel(g_spec, head(g_in))
    print(f"f16 preset {preset} T={T}: spectrogram teacher-forced rel_rms {e_round:.3g} "
          f"(without the f16 input rounding {e_plain:.3g})")
    assert e_round <= 2e-5 and e_plain >= 5 * e_round, (e_round, e_plain)
    o_spec = oc.decode_stage(codes, emb, last, cap).astype(np.float64)
    assert g_spec.shape == o_spec.shape
    assert rel(g_spec, o_spec) <= 5e-3, rel(g_spec, o_spec)
    gp, op = gc.decode_pcm(codes, emb).astype(np.float64), oc.decode_pcm(codes, emb).astype(np.float64)
    assert gp.shape == op.shape and rel(gp, op) <= 5e-3, rel(gp, op)


@pytest.mark.parametrize("preset,T", [(2, 33), (3, 700)])
def test_codec_f16_teacher_forced_pcm(device, tmp_path, emb, preset, T):
    """F16 codec matrices held to the north-star bar (PCM within 1e-4 RMS of the CPU reference,
    BASELINE.json) stage by stage. ggml rounds every F16 linear's input to f16 (miocodec.cpp:
    205-209, :624, :685), so chained end to end a last-bit difference upstream that crosses an
    f16 rounding boundary moves a value by a whole f16 ulp (4.9e-4 relative) and the chain
    drifts (test_codec_f16_weights' 5e-3). Here the oracle runs each stage on the GPU's own
    input of that stage (pyoracle.Codec.stage_from, teacher forcing): every stage's arithmetic is
    checked without upstream flips, and the PCM is the oracle's head + iSTFT on the GPU's last
    stage input, which must be within 1e-4 RMS absolute of the GPU's PCM at T = 700 (the bench
    length) on the full-size F16 preset. Per-stage bound: the F32 codec's stage bar, rel-rms
    1e-3 (within-stage flips only: a stage chains up to ~10 f16-rounded linears; the tiny
    preset's prenet measured 2.6e-4)."""
    path = m.synth_codec(str(tmp_path / f"f16tf_{preset}.gguf"), preset, 1)
    gc = m.Codec(device, path)
    oc = pyoracle.Codec(path)
    codes = np.random.default_rng(700 + preset).integers(0, 12800, T).astype(np.int32)
    cap = 18 * T * 1024 + 4096
    last = oc.n_stages - 1
    prev = gc.decode_stage(codes, emb, 0, cap)
    worst = 0.0
    for st in range(1, last + 1):
        g = gc.decode_stage(codes, emb, st, cap)
        o = oc.stage_from(codes, emb, st, prev, st, cap)
        assert g.shape == o.shape, (st, g.shape, o.shape)
        d = g.astype(np.float64) - o
        rel = float(np.sqrt(np.mean(d * d)) / (np.sqrt(np.mean(o.astype(np.float64) ** 2)) + 1e-30))
        worst = max(worst, rel)
        assert rel <= 1e-3, (st, rel)
        if st < last:
            prev = g
    # PCM: the oracle's head on the GPU's out_proj output, then the reference iSTFT
    o_spec = oc.stage_from(codes, emb, last, prev, last, cap)
    o_pcm = pyoracle.istft(o_spec, oc.n_fft, oc.n_fft, oc.hop_length)
    g_pcm = gc.decode_pcm(codes, emb).astype(np.float64)
    assert g_pcm.shape == o_pcm.shape
    rms = float(np.sqrt(np.mean((g_pcm - o_pcm) ** 2)))
    print(f"f16 preset {preset} T={T}: worst stage rel-rms {worst:.3g}, teacher-forced PCM rms {rms:.3g}")
    assert rms <= 1e-4, rms
