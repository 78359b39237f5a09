"""GPU: the drop-in C++ surface (include/test-to-speech.h, miocodec.h, istft.h) and the CLIs
(build/miotts, miotts-stream-benchmark, miotts-stream-compare), driven as subprocesses
the way main.cpp / examples/stream-*.cpp are used.

* miocodec_decode + istft (host API) vs the C oracle: spectrogram within the codec stage
  tolerance, PCM within 1e-4 RMS (test_codec_gpu.py explains the bounds).
* miotts writes a 16-bit mono WAV of n_codes * samples_per_token samples, peak 0.95.
* miotts-stream-benchmark with --speech-only --ignore-eos (harness deviation)
  reproduces the reference streaming cadence (700 tokens -> 18 decode calls / 7160 codes,
  SURVEY 8c KAT 4) and prints every stream_bench.* key.
* miotts-stream-compare --skip-llm: stream concat has the offline length and differs only
  in the crossfaded splice regions.
* the samples synthesize_stream emits (holdback 32, commit step 24, llround sample mapping,
  30 ms crossfade, chunking) equal the C restatement of test-to-speech.cpp:367-417,496-571
  (oracle/stream_ref.c) driven by the oracle codec, within 1e-4 RMS.
"""
import os
import re
import subprocess
import wave

import numpy as np
import pytest

import miotts_amd as m
import pyoracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "miotts-llama.cpp_amd", "build")


def run(args, timeout=300):
    p = subprocess.run([os.path.join(BIN, args[0])] + [str(a) for a in args[1:]], capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, f"{args[0]} rc={p.returncode}\n{p.stdout}\n{p.stderr[-2000:]}"
    # a fallback the product takes must not pass a test silently (tts.cpp: a batched decode that
    # fails - a refused model or a timed-out hand-off - decodes one utterance at a time)
    assert "batched decode unavailable" not in p.stderr, p.stderr[-2000:]
    return p.stdout


def kv(out):
    return dict(re.findall(r"^([\w.]+)=([^\s]+)", out, re.M))


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    return {"llm": m.synth_llm(str(d / "llm1.gguf"), 1, 1),
            "codec": m.synth_codec(str(d / "codec.gguf"), 0, 1),
            "codec_tiny": m.synth_codec(str(d / "codec_tiny.gguf"), 1, 1),
            "voice": m.synth_voice(str(d / "voice.emb.gguf"), 7),
            "dir": d}


def test_miocodec_decode_and_istft_api(files):
    rng = np.random.default_rng(5)
    codes = rng.integers(0, 12800, 60).astype(np.int32)
    d = files["dir"]
    codes.tofile(d / "codes.i32")
    out = run(["miotts-api-dump", files["codec"], files["voice"], d / "codes.i32", d / "spec.f32", d / "pcm.f32"])
    info = kv(out)
    spec = np.fromfile(d / "spec.f32", np.float32)
    pcm = np.fromfile(d / "pcm.f32", np.float32)
    oc = pyoracle.Codec(files["codec"])
    emb = m.read_voice(files["voice"])
    ospec = oc.decode(codes, emb)
    assert int(info["frames"]) == ospec.shape[0] and spec.size == ospec.size
    dspec = spec.astype(np.float64) - ospec.reshape(-1)
    assert np.sqrt(np.mean(dspec ** 2)) <= 1e-3 * np.sqrt(np.mean(ospec.astype(np.float64) ** 2))
    opcm = pyoracle.istft(ospec, oc.n_fft, oc.n_fft, oc.hop_length)
    assert pcm.shape == opcm.shape == (60 * oc.samples_per_token,)
    assert np.sqrt(np.mean((pcm.astype(np.float64) - opcm) ** 2)) <= 1e-4


def test_miotts_cli_writes_wav(files):
    wav = files["dir"] / "out.wav"
    run(["miotts", "-m", files["llm"], "-c", files["codec"], "-v", files["voice"], "-p", "テストです。",
         "-o", wav, "--max-tokens", 48, "--speech-only", "--ignore-eos"])
    with wave.open(str(wav)) as w:
        assert w.getnchannels() == 1 and w.getsampwidth() == 2 and w.getframerate() == 44100
        x = np.frombuffer(w.readframes(w.getnframes()), np.int16)
    assert len(x) == 48 * 1764
    assert abs(np.abs(x).max() - int(0.95 * 32767)) <= 1  # peak-normalised to 0.95


def test_miotts_batch_equals_single_runs(files):
    """`miotts --batch FILE` (extension): the lines decode together on the batched engine and
    each OUTPUT_nnn.wav has the bytes a single `miotts -p LINE` run writes (every stream
    samples with the single run's seed; mio_hip_llm_generate_batch's streams equal
    mio_hip_llm_generate). --gpus 1 takes the sharding path with one device."""
    d = files["dir"]
    prompts = ["テストです。", "こんにちは。", "今日はいい天気ですね。"]
    (d / "batch.txt").write_text("\n".join(prompts) + "\n", "utf-8")
    common = ["-m", files["llm"], "-c", files["codec"], "-v", files["voice"], "--max-tokens", 40, "--speech-only",
              "--ignore-eos"]
    run(["miotts"] + common + ["--batch", d / "batch.txt", "-o", d / "b.wav", "--gpus", 1])
    for i, p in enumerate(prompts):
        run(["miotts"] + common + ["-p", p, "-o", d / f"s{i}.wav"])
        assert (d / f"b_{i:03d}.wav").read_bytes() == (d / f"s{i}.wav").read_bytes(), i


def test_miotts_usage_errors(files):
    p = subprocess.run([os.path.join(BIN, "miotts"), "-c", files["codec"]], capture_output=True, text=True)
    assert p.returncode == 1 and "--prompt is required" in p.stderr
    p = subprocess.run([os.path.join(BIN, "miotts"), "--bogus"], capture_output=True, text=True)
    assert p.returncode == 1 and "Unknown argument: --bogus" in p.stderr
    out = run(["miotts", "--dump-tensors", "-c", files["codec"]])
    assert out.startswith("Tensors in ") and "type=" in out


@pytest.mark.parametrize("n,calls,codes", [(700, 18, 7160), (100, 3, 260)])
def test_stream_benchmark_cadence(files, n, calls, codes):
    out = run(["miotts-stream-benchmark", "-m", files["llm"], "-c", files["codec"], "-v", files["voice"],
               "-p", "こんにちは、今日はいい天気ですね。", "--max-tokens", n, "--speech-only", "--ignore-eos"])
    r = kv(out)
    for k in ["total_sec", "audio_sec", "rtf", "x_realtime", "llm_tokens", "decode_calls", "decoded_codes",
              "emitted_samples", "stage.llm_sec", "stage.codec_sec", "stage.istft_sec", "stage.callback_sec"]:
        assert f"stream_bench.{k}" in r, k
    assert int(r["stream_bench.llm_tokens"]) == n
    assert int(r["stream_bench.decode_calls"]) == calls
    assert int(r["stream_bench.decoded_codes"]) == codes
    assert int(r["stream_bench.emitted_samples"]) == n * 1764


def test_stream_compare_skip_llm(files):
    rng = np.random.default_rng(11)
    text = "".join(f"<|s_{c}|>" for c in rng.integers(0, 12800, 300))
    d = files["dir"]
    out = run(["miotts-stream-compare", "-c", files["codec"], "-v", files["voice"], "-p", text, "--skip-llm",
               "--out-offline", d / "off.wav", "--out-stream", d / "str.wav"])
    r = kv(out)
    assert int(r["offline_samples"]) == int(r["stream_samples"]) == 300 * 1764
    assert int(r["sample_diff"]) == 0
    # --skip-llm streams the whole decode in one pass: identical to the offline vector
    assert float(r["compare.max_abs"]) == 0.0


def test_stream_benchmark_1p7b_700_tokens(files, synth_llm_path):
    """BASELINE configs[4] (C5): the streaming path on the 1.7B Q4_K_M preset, 700 tokens ->
    18 full re-decodes / 7160 codes (test-to-speech.cpp:496-571 cadence), every sample emitted."""
    out = run(["miotts-stream-benchmark", "-m", synth_llm_path(3), "-c", files["codec"], "-v", files["voice"],
               "-p", "こんにちは、今日はいい天気ですね。", "--max-tokens", 700, "--speech-only", "--ignore-eos"],
              timeout=600)
    r = kv(out)
    assert int(r["stream_bench.llm_tokens"]) == 700
    assert int(r["stream_bench.decode_calls"]) == 18
    assert int(r["stream_bench.decoded_codes"]) == 7160
    assert int(r["stream_bench.emitted_samples"]) == 700 * 1764
    print({k: r[k] for k in r if k.startswith("stream_bench.")})


def test_stream_benchmark_c1_0p1b_700_tokens(files, synth_llm_path):
    """BASELINE configs[0] (C1): MioTTS-0.1B Q8_0 (preset 2) through miotts-stream-benchmark,
    the reference's harness (stream-benchmark.cpp:148-166): every stream_bench.* key, the
    18 / 7160 re-decode cadence of a 700-token utterance, every sample emitted. The reference
    runs this config on its CPU path (ggml, absent here); the product has no CPU
    fallback, so this is the same workload on the GPU path (bench.py's cpu_baseline_c1 times
    the C oracle on it)."""
    out = run(["miotts-stream-benchmark", "-m", synth_llm_path(2), "-c", files["codec"], "-v", files["voice"],
               "-p", "こんにちは、今日はいい天気ですね。", "--max-tokens", 700, "--speech-only", "--ignore-eos"],
              timeout=600)
    r = kv(out)
    for k in ["total_sec", "audio_sec", "rtf", "x_realtime", "llm_tokens", "decode_calls", "decoded_codes",
              "emitted_samples", "stage.llm_sec", "stage.codec_sec", "stage.istft_sec", "stage.callback_sec"]:
        assert f"stream_bench.{k}" in r, k
    assert int(r["stream_bench.llm_tokens"]) == 700
    assert int(r["stream_bench.decode_calls"]) == 18
    assert int(r["stream_bench.decoded_codes"]) == 7160
    assert int(r["stream_bench.emitted_samples"]) == 700 * 1764
    assert float(r["stream_bench.audio_sec"]) == pytest.approx(28.0, abs=1e-3)
    print({k: r[k] for k in r if k.startswith("stream_bench.")})


@pytest.mark.parametrize("n,chunk", [(100, 4096), (141, 1000), (320, 4096)])
def test_stream_emission_matches_restatement(files, n, chunk):
    """Everything synthesize_stream hands its callback (LLM speech-only, tiny codec) against
    oracle/stream_ref.c over the same codes: identical chunk sizes, samples within 1e-4 RMS.
    At 320 tokens the later re-decodes take prenet rows from the previous decode
    (MIO_CODEC_INCREMENTAL: rows whose receptive field was complete), checked to happen."""
    prefix = str(files["dir"] / f"stream_{n}_{chunk}")
    out = run(["miotts-stream-benchmark", "-m", files["llm"], "-c", files["codec_tiny"], "-v", files["voice"],
               "-p", "こんにちは、今日はいい天気ですね。", "--max-tokens", n, "--speech-only", "--ignore-eos",
               "--chunk-samples", chunk, "--dump-stream", prefix])
    r = kv(out)
    got = np.fromfile(prefix + ".f32", np.float32)
    chunks = np.fromfile(prefix + ".chunks.i64", np.int64)
    codes = np.fromfile(prefix + ".codes.i32", np.int32)
    assert codes.size == n and int(r["stream_bench.llm_tokens"]) == n
    oc = pyoracle.Codec(files["codec_tiny"])
    ref, ref_chunks, n_dec = pyoracle.stream_emit(oc, m.read_voice(files["voice"]), codes, 20, 32, 24, chunk)
    assert int(r["stream_bench.decode_calls"]) == n_dec
    assert chunks.tolist() == ref_chunks.tolist()
    assert got.size == ref.size == n * oc.samples_per_token
    d = got.astype(np.float64) - ref
    rms = float(np.sqrt(np.mean(d * d)))
    assert rms <= 1e-4 and float(np.abs(d).max()) <= 1e-3, (rms, float(np.abs(d).max()))
    if n >= 300:
        assert int(r["stream_bench.prenet_rows_reused"]) > 0, r
