"""CPU: host utilities vs fixtures generated from the reference's own sources
(tests/golden/make_golden.py): token parser (token-parser.cpp:5-28), normaliser
(text-normalize.cpp:108-158), WAV bytes (wav-writer.cpp:24-44) — exact equality."""
import json
import os

import numpy as np

import miotts_amd as m


def test_token_parser_matches_reference(golden_dir):
    for case in json.load(open(os.path.join(golden_dir, "token_parser.json"), encoding="utf-8")):
        assert m.parse_speech_tokens(case["text"]).tolist() == case["codes"], case["text"]


def test_normalizer_matches_reference(golden_dir):
    for case in json.load(open(os.path.join(golden_dir, "normalize.json"), encoding="utf-8")):
        assert m.normalize_text(case["text"]) == case["normalized"], case["text"]


def test_wav_bytes_match_reference(golden_dir):
    z = np.load(os.path.join(golden_dir, "wav_cases.npz"))
    for k in z.files:
        if k.startswith("in_"):
            name = k[3:]
            assert m.wav_bytes(z[k], 44100) == z[f"bytes_{name}"].tobytes(), name
