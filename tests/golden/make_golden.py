"""Generate the committed golden fixtures from the REFERENCE's own code.

Runs only in the build container (where /root/reference exists): it builds
oracle/_ref/libmioref.so from the reference translation units that compile here
(istft.cpp, token-parser.cpp, wav-writer.cpp, text-normalize.cpp) and
records inputs + the reference's outputs as small data fixtures:

  istft_cases.npz        seeded spectrograms -> reference istft() PCM   (istft.cpp:68-108)
  istft_kat.npz          DC-only / Nyquist-only known-answer spectra  (SURVEY 8c KAT 1)
  token_parser.json      strings -> parse_speech_tokens()              (token-parser.cpp:5-28)
  normalize.json         strings -> normalize_tts_text()               (text-normalize.cpp:108-158)
  wav_cases.npz          sample vectors -> exact wav_write() bytes     (wav-writer.cpp:24-44)

Usage: python tests/golden/make_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle  # noqa: E402


def main() -> None:
    if not os.path.isdir("/root/reference/src"):
        sys.exit("reference sources not present; fixtures are generated in the build container only")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    R = pyoracle.ref()

    # --- iSTFT: seeded spectra of magnitude/phase statistics like the codec head
    # (mag = clamp(exp(.), 0, 100), miocodec.cpp:735-737), several frame counts incl. edge cases.
    cases = {}
    rng = np.random.default_rng(20260227)
    for n_frames in (0, 1, 2, 3, 5, 18, 36, 90):
        logmag = rng.normal(-1.0, 1.5, size=(n_frames, 197)).astype(np.float32)
        phase = rng.uniform(-np.pi, np.pi, size=(n_frames, 197)).astype(np.float32)
        mag = np.clip(np.exp(logmag), 0, 100).astype(np.float32)
        spec = np.stack([mag * np.cos(phase), mag * np.sin(phase)], axis=-1).astype(np.float32)
        out = pyoracle.istft(spec, use_ref=True)
        cases[f"spec_{n_frames}"] = spec
        cases[f"pcm_{n_frames}"] = out
    np.savez_compressed(os.path.join(HERE, "istft_cases.npz"), **cases)

    kat = {}
    F = 40
    dc = np.zeros((F, 197, 2), np.float32)
    dc[:, 0, 0] = 392.0
    ny = np.zeros((F, 197, 2), np.float32)
    ny[:, 196, 0] = 392.0
    # imaginary parts of DC and Nyquist must be ignored (istft.cpp:52-53)
    dc_im = dc.copy()
    dc_im[:, 0, 1] = 123.0
    dc_im[:, 196, 1] = -77.0
    for name, s in (("dc", dc), ("nyq", ny), ("dc_im", dc_im)):
        kat[f"spec_{name}"] = s
        kat[f"pcm_{name}"] = pyoracle.istft(s, use_ref=True)
    np.savez_compressed(os.path.join(HERE, "istft_kat.npz"), **kat)

    # --- token parser (incl. malformed tokens, token-parser.cpp:18-24)
    strs = [
        "",
        "<|s_0|>",
        "<|s_12799|><|s_1|><|s_42|>",
        "hello <|s_5|> world <|s_6|>",
        "<|s_|><|s_7|>",
        "<|s_8",
        "<|s_9|",
        "<|s_10|><|s_x|><|s_11|>",
        "<|s_-3|><|s_+4|>",
        "<|s_ 12|>",
        "<|s_<|s_13|>",
        "<|s_1234567|>",
        "<|im_end|><|s_99|>\n",
        "".join(f"<|s_{c}|>" for c in [12287, 11619, 11774, 12223, 2490, 826, 2257, 1668,
                                         1219, 2319, 9994, 12683, 12745, 4215, 12478, 8800,
                                         8696, 375, 1406, 12396]),
    ]
    tp = []
    buf = np.zeros(4096, np.int32)
    for s in strs:
        n = R.ref_parse_speech_tokens(s.encode(), buf.ctypes.data, len(buf))
        tp.append({"text": s, "codes": buf[:n].tolist()})
    with open(os.path.join(HERE, "token_parser.json"), "w", encoding="utf-8") as f:
        json.dump(tp, f, ensure_ascii=False, indent=1)

    # --- text normaliser
    ns = [
        "こんにちは、今日はいい天気ですね。",
        "ラーメン食べますか?嫌なら食べなくていいですけど、捨てるのもったいないので持って帰ってください。",
        "The quick brown fox jumps over the lazy dog.",
        "すごい！ほんと？〜〜",
        "「こんにちは」",
        "『テスト』。、",
        "（括弧）",
        "【見出し】",
        "(あいう)",
        "あ\tい[n]う　え お",
        "♥●◯〇",
        "え………………",
        "mixed English and 日本語。",
        "abc。",
        "",
        "   ",
        "。。。",
    ]
    nr = []
    cbuf = ctypes_buf = np.zeros(8192, np.uint8)
    for s in ns:
        n = R.ref_normalize_tts_text(s.encode("utf-8"), ctypes_buf.ctypes.data, len(ctypes_buf))
        nr.append({"text": s, "normalized": bytes(ctypes_buf[:n]).decode("utf-8")})
    with open(os.path.join(HERE, "normalize.json"), "w", encoding="utf-8") as f:
        json.dump(nr, f, ensure_ascii=False, indent=1)

    # --- WAV writer bytes
    wav = {}
    rng = np.random.default_rng(7)
    vecs = {
        "empty": np.zeros(0, np.float32),
        "ramp": np.linspace(-1.2, 1.2, 257).astype(np.float32),
        "noise": (rng.standard_normal(1000) * 0.5).astype(np.float32),
        "edges": np.array([1.0, -1.0, 0.99999, -0.99999, 1.00002, -1.00004, 0.5 / 32767,
                           -0.5 / 32767, 1.5 / 32767, -1.5 / 32767, 0.0, -0.0], np.float32),
        # std::clamp passes NaN through; static_cast<int16_t> of it is the x86 cvttss2si
        # integer-indefinite 0x80000000 truncated to 16 bits = 0 (the reference's bytes)
        "nan_inf": np.array([np.nan, -np.nan, np.inf, -np.inf, 0.25, np.nan], np.float32),
    }
    with tempfile.TemporaryDirectory() as td:
        for k, v in vecs.items():
            p = os.path.join(td, k + ".wav")
            ok = R.ref_wav_write(p.encode(), v.ctypes.data if v.size else None, len(v), 44100)
            assert ok == 1
            with open(p, "rb") as f:
                wav[f"in_{k}"] = v
                wav[f"bytes_{k}"] = np.frombuffer(f.read(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "wav_cases.npz"), **wav)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
