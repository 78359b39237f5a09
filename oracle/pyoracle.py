"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes loader for the plain-C oracle (oracle/_build/libmiooracle.so) and, where it
was built in this container, the reference-TU build (oracle/_ref/libmioref.so).
Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "libmiooracle.so")
REF_LIB = os.path.join(ORACLE_DIR, "_ref", "libmioref.so")

_o = None
_r = None
_f32p = ctypes.POINTER(ctypes.c_float)


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def oracle() -> ctypes.CDLL:
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        _o = ctypes.CDLL(ORACLE_LIB)
        _o.mo_istft.restype = ctypes.c_int
        _o.mo_istft.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p]
    return _o


def ref_available() -> bool:
    return os.path.exists(REF_LIB)


def ref() -> ctypes.CDLL:
    global _r
    if _r is None:
        _r = ctypes.CDLL(REF_LIB)
        _r.ref_istft.restype = ctypes.c_int
        _r.ref_istft.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
        _r.ref_parse_speech_tokens.restype = ctypes.c_int
        _r.ref_parse_speech_tokens.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int]
        _r.ref_normalize_tts_text.restype = ctypes.c_int
        _r.ref_normalize_tts_text.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int]
        _r.ref_wav_write.restype = ctypes.c_int
        _r.ref_wav_write.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    return _r


def istft(spec: np.ndarray, n_fft: int = 392, win: int = 392, hop: int = 98,
          use_ref: bool = False) -> np.ndarray:
    spec = np.ascontiguousarray(spec, dtype=np.float32)
    n_frames = spec.shape[0] if spec.size else 0
    out = np.zeros(max(n_frames * hop + win, 1), np.float32)
    fn = ref().ref_istft if use_ref else oracle().mo_istft
    n = fn(spec.ctypes.data if spec.size else None, n_frames, n_fft, win, hop, out.ctypes.data)
    return out[:n].copy()
