"""GPU parity: the device PCM epilogue (mio_hip_pcm_finish, csrc/hip/pcm_finish.hip) vs the
reference's own wav_write bytes and a float32 restatement of peak_normalize.

Without normalisation the int16 samples must equal the sample bytes that the reference's
wav-writer.cpp:24-44 produced for tests/golden/wav_cases.npz (pinned, bit-exact). With it, the
gain 0.95 / max|s| of test-to-speech.cpp:232-243 is applied first; numpy float32 arithmetic
(IEEE, correctly rounded, same operation order) restates it exactly.
"""
import os

import numpy as np
import pytest

import miotts_amd as m

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "wav_cases.npz")


def _to_pcm16(s):
    """std::clamp(s * 32767, -32768, 32767) then the x86 truncating conversion: NaN -> 0."""
    t = s.astype(np.float32) * np.float32(32767.0)
    with np.errstate(invalid="ignore"):
        c = np.where(t < np.float32(-32768.0), np.float32(-32768.0), np.where(np.float32(32767.0) < t,
                                                                           np.float32(32767.0), t))
        c = np.where(np.isnan(c), np.float32(0.0), c)
    return np.trunc(c).astype(np.int32).astype(np.int16)


def _normalized(s):
    # std::max(peak, fabs(s)) from peak = 0: a NaN never replaces peak
    peak = np.float32(np.nanmax(np.abs(s), initial=0.0)) if s.size else np.float32(0.0)
    if peak > np.float32(1e-8):
        s = s * (np.float32(0.95) / peak)
    return s.astype(np.float32), float(peak)


def test_matches_reference_wav_bytes(device):
    z = np.load(GOLDEN)
    for case in ("empty", "ramp", "noise", "edges", "nan_inf"):
        s = z[f"in_{case}"].astype(np.float32)
        want = np.frombuffer(z[f"bytes_{case}"][44:].tobytes(), "<i2")
        d = device.upload(s if s.size else np.zeros(1, np.float32))
        got, peak = m.pcm_finish(device, d, s.size, False)
        assert peak == 0.0
        np.testing.assert_array_equal(got, want, err_msg=case)


@pytest.mark.parametrize("n", [1, 3, 4, 1001, 1_234_800])
def test_peak_normalize_exact(device, n):
    rng = np.random.default_rng(n)
    s = (rng.standard_normal(n) * 0.3).astype(np.float32)
    if n > 4:
        s[n // 2] = np.nan  # ignored by the peak, converts to 0 like the reference's wav_write
        s[n // 3] = -1.7    # the peak
    want_s, want_peak = _normalized(s)
    got, peak = m.pcm_finish(device, device.upload(s), n, True)
    assert peak == want_peak
    np.testing.assert_array_equal(got, _to_pcm16(want_s))


def test_silence_is_not_scaled(device):
    s = np.full(4096, 1e-9, np.float32)
    got, peak = m.pcm_finish(device, device.upload(s), s.size, True)
    assert peak == np.float32(1e-9)
    np.testing.assert_array_equal(got, _to_pcm16(s))


def test_concurrent_streams_do_not_share_scratch(device):
    """Two normalising calls in flight on different streams (the partials used to
    be one module-global array): each gets its own gain."""
    import ctypes
    lib = m.lib()
    a = np.full(1 << 20, 0.5, np.float32)
    b = np.full(1 << 20, 0.25, np.float32)
    da, db = device.upload(a), device.upload(b)
    oa, ob = device.empty((a.size,), np.int16), device.empty((b.size,), np.int16)
    s1, s2 = ctypes.c_void_p(), ctypes.c_void_p()
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s1), 1) == 0
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1) == 0
    for _ in range(4):
        m.check(lib.mio_hip_pcm_finish(device.h, da.ptr, a.size, 1, oa.ptr, None, s1))
        m.check(lib.mio_hip_pcm_finish(device.h, db.ptr, b.size, 1, ob.ptr, None, s2))
    device.sync()
    hip.hipStreamSynchronize(s1), hip.hipStreamSynchronize(s2)
    want = int(np.float32(0.95) * np.float32(32767.0))
    assert (oa.numpy() == want).all() and (ob.numpy() == want).all()
    hip.hipStreamDestroy(s1), hip.hipStreamDestroy(s2)


@pytest.mark.parametrize("n", [5, 1001, 1_234_800])
def test_normalize_in_place_exact(device, n):
    """mio_hip_pcm_normalize (TestToSpeech::synthesize_to_vector's peak normalisation on the
    device): the float samples equal the host loop of test-to-speech.cpp:232-243 bit for bit."""
    rng = np.random.default_rng(n + 1)
    s = (rng.standard_normal(n) * 0.4).astype(np.float32)
    s[n // 2] = -2.5
    want, want_peak = _normalized(s)
    d = device.upload(s)
    import ctypes
    peak = ctypes.c_float(0)
    m.check(m.lib().mio_hip_pcm_normalize(device.h, d.ptr, n, d.ptr, ctypes.byref(peak), None))
    assert peak.value == want_peak
    np.testing.assert_array_equal(d.numpy(), want)
