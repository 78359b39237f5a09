"""CPU: the iSTFT oracle is pinned to the reference (istft.cpp:7-108).

(1) against the committed fixtures produced by the reference's own istft.cpp
    (tests/golden/make_golden.py), bit-exact;
(2) against a live build of the reference TUs when oracle/_ref exists here;
(3) known-answer tests (SURVEY 8c KAT 1).
"""
import os

import numpy as np
import pytest

import pyoracle


def test_oracle_matches_reference_fixtures(golden_dir):
    z = np.load(os.path.join(golden_dir, "istft_cases.npz"))
    for key in z.files:
        if not key.startswith("spec_"):
            continue
        n = key.split("_")[1]
        spec, pcm = z[key], z[f"pcm_{n}"]
        out = pyoracle.istft(spec)
        assert out.shape == pcm.shape, key
        assert np.array_equal(out, pcm), f"{key}: max diff {np.abs(out - pcm).max()}"


def test_oracle_kat_fixtures(golden_dir):
    z = np.load(os.path.join(golden_dir, "istft_kat.npz"))
    for name in ("dc", "nyq", "dc_im"):
        out = pyoracle.istft(z[f"spec_{name}"])
        assert np.array_equal(out, z[f"pcm_{name}"]), name
    # interior value of DC-only input = sum(w)/sum(w^2) = 4/3 for periodic Hann at hop N/4
    dc = pyoracle.istft(z["spec_dc"])
    interior = dc[400:-400]
    assert np.allclose(interior, 4.0 / 3.0, atol=1e-5)
    assert len(dc) == 98 * 40
    ny = pyoracle.istft(z["spec_nyq"])[400:-400]
    assert np.allclose(np.abs(ny), 4.0 / 3.0, atol=1e-5)


def test_oracle_empty_and_lengths():
    assert pyoracle.istft(np.zeros((0, 197, 2), np.float32)).size == 0
    for f in (1, 2, 7):
        assert pyoracle.istft(np.zeros((f, 197, 2), np.float32)).size == 98 * f


@pytest.mark.skipif(not pyoracle.ref_available(), reason="reference TUs not built here")
def test_oracle_matches_live_reference():
    rng = np.random.default_rng(99)
    for f in (1, 4, 37, 200):
        spec = rng.standard_normal((f, 197, 2)).astype(np.float32) * 3
        a = pyoracle.istft(spec)
        b = pyoracle.istft(spec, use_ref=True)
        assert np.array_equal(a, b)
