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
        vp, ci = ctypes.c_void_p, ctypes.c_int
        _o.mo_codec_load.restype = vp
        _o.mo_codec_load.argtypes = [ctypes.c_char_p]
        _o.mo_codec_free.argtypes = [vp]
        _o.mo_codec_info.argtypes = [vp, vp]
        _o.mo_codec_n_stages.argtypes = [vp]
        _o.mo_codec_decode_stage.argtypes = [vp, vp, ci, vp, ci, vp, ctypes.POINTER(ci),
                                             ctypes.POINTER(ci)]
        _o.mo_codec_decode.argtypes = [vp, vp, ci, vp, vp]
        _o.mo_f16_round.restype = ctypes.c_float
        _o.mo_f16_round.argtypes = [ctypes.c_float]
        _o.mo_llm_load.restype = vp
        _o.mo_llm_load.argtypes = [ctypes.c_char_p, ci]
        _o.mo_llm_free.argtypes = [vp]
        _o.mo_llm_info.argtypes = [vp, vp]
        _o.mo_llm_reset.argtypes = [vp]
        _o.mo_llm_eval.argtypes = [vp, ci, ci, vp]
        _o.mo_llm_embed.argtypes = [vp, ci, vp]
        _o.mo_llm_layer.argtypes = [vp, ci, ci, vp, vp]
        _o.mo_llm_head.argtypes = [vp, vp, vp]
        _o.mo_llm_kv.argtypes = [vp, ci, ci, vp, vp, ci]
        _o.mo_llm_conv.argtypes = [vp, ci, vp, ci]
        _o.mo_llm_is_conv.argtypes = [vp, ci]
        _o.mo_gumbel.restype = ctypes.c_float
        _o.mo_gumbel.argtypes = [ctypes.c_uint64, ci, ci]
        _o.mo_sample.restype = ci
        _o.mo_sample.argtypes = [vp, ctypes.c_float, ctypes.c_uint64, ci, ci, ci]
        _o.mo_dequantize_row.argtypes = [ctypes.c_uint32, vp, ctypes.c_int64, vp]
        _o.mo_set_threads.restype = ci
        _o.mo_set_threads.argtypes = [ci]
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


class Codec:
    """Oracle MioCodec forward (oracle/codec_ref.c)."""

    def __init__(self, path: str):
        self.h = oracle().mo_codec_load(path.encode())
        if not self.h:
            raise RuntimeError(f"oracle: cannot load codec {path}")
        info = np.zeros(8, np.int32)
        oracle().mo_codec_info(self.h, info.ctypes.data)
        (self.sample_rate, self.n_fft, self.hop_length, self.samples_per_token, self.n_freq,
         self.up_stages, self.frames_per_code, self.n_codes) = [int(x) for x in info]
        self.n_stages = oracle().mo_codec_n_stages(self.h)

    def __del__(self):
        try:
            if self.h:
                oracle().mo_codec_free(self.h)
                self.h = None
        except Exception:
            pass

    def decode(self, codes, emb) -> np.ndarray:
        codes = np.ascontiguousarray(codes, dtype=np.int32)
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        out = np.zeros((len(codes) * self.frames_per_code, self.n_freq, 2), np.float32)
        n = oracle().mo_codec_decode(self.h, codes.ctypes.data, len(codes), emb.ctypes.data,
                                     out.ctypes.data)
        if n < 0:
            raise RuntimeError(f"oracle codec decode failed: {n}")
        return out[:n]

    def decode_stage(self, codes, emb, stage: int, max_elems: int) -> np.ndarray:
        codes = np.ascontiguousarray(codes, dtype=np.int32)
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        out = np.zeros(max_elems, np.float32)
        r, c = ctypes.c_int(0), ctypes.c_int(0)
        rc = oracle().mo_codec_decode_stage(self.h, codes.ctypes.data, len(codes), emb.ctypes.data,
                                            stage, out.ctypes.data, ctypes.byref(r), ctypes.byref(c))
        if rc != 0:
            raise RuntimeError(f"oracle stage {stage} failed: {rc}")
        return out[: r.value * c.value].reshape(r.value, c.value)

    def stage_from(self, codes, emb, start: int, x_in, stop: int, max_elems: int) -> np.ndarray:
        """Teacher forcing: stages start .. stop run on x_in (the output of stage start - 1,
        e.g. the GPU's) instead of on the oracle's own earlier stages."""
        codes = np.ascontiguousarray(codes, dtype=np.int32)
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        x_in = np.ascontiguousarray(x_in, dtype=np.float32)
        out = np.zeros(max_elems, np.float32)
        r, c = ctypes.c_int(0), ctypes.c_int(0)
        o = oracle()
        o.mo_codec_stage_from.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int)]
        rc = o.mo_codec_stage_from(self.h, codes.ctypes.data, len(codes), emb.ctypes.data, start, x_in.ctypes.data,
                                   stop, out.ctypes.data, ctypes.byref(r), ctypes.byref(c))
        if rc != 0:
            raise RuntimeError(f"oracle stages {start}..{stop} failed: {rc}")
        return out[: r.value * c.value].reshape(r.value, c.value)

    def decode_pcm(self, codes, emb) -> np.ndarray:
        spec = self.decode(codes, emb)
        return istft(spec, self.n_fft, self.n_fft, self.hop_length)


def stream_emit(codec: "Codec", emb, codes, check_interval: int = 20, holdback: int = 32, min_commit: int = 24,
                chunk_samples: int = 4096):
    """Samples TestToSpeech::synthesize_stream emits for speech-only codes (oracle/stream_ref.c):
    (samples, chunk sizes, full decodes)."""
    codes = np.ascontiguousarray(codes, dtype=np.int32)
    emb = np.ascontiguousarray(emb, dtype=np.float32)
    cap = len(codes) * codec.samples_per_token + 16
    out = np.zeros(cap, np.float32)
    chunks = np.zeros(cap // max(1, min(chunk_samples, 64)) + 64, np.int64)
    n_chunks, n_dec = ctypes.c_long(0), ctypes.c_int(0)
    f = oracle().mo_stream_emit
    f.restype = ctypes.c_long
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
                  ctypes.c_void_p, ctypes.c_void_p]
    n = f(codec.h, emb.ctypes.data, codes.ctypes.data, len(codes), check_interval, holdback, min_commit,
          chunk_samples, out.ctypes.data, cap, chunks.ctypes.data, len(chunks), ctypes.byref(n_chunks),
          ctypes.byref(n_dec))
    if n < 0:
        raise RuntimeError("oracle stream_emit failed")
    return out[:n].copy(), chunks[:n_chunks.value].copy(), n_dec.value


class Llm:
    """Oracle decode step (oracle/llm_ref.c) + shared counter-based sampler."""

    def __init__(self, path: str, n_ctx: int = 512):
        self.h = oracle().mo_llm_load(path.encode(), n_ctx)
        if not self.h:
            raise RuntimeError(f"oracle: cannot load llm {path}")
        info = np.zeros(8, np.int32)
        oracle().mo_llm_info(self.h, info.ctypes.data)
        (self.n_vocab, self.n_embd, self.n_layer, self.n_head, self.n_kv, self.head_dim,
         self.n_ff, self.n_ctx) = [int(x) for x in info]

    def __del__(self):
        try:
            if self.h:
                oracle().mo_llm_free(self.h)
                self.h = None
        except Exception:
            pass

    def reset(self):
        oracle().mo_llm_reset(self.h)

    def eval(self, token: int, pos: int) -> np.ndarray:
        out = np.zeros(self.n_vocab, np.float32)
        rc = oracle().mo_llm_eval(self.h, token, pos, out.ctypes.data)
        if rc:
            raise RuntimeError(f"oracle eval failed {rc}")
        return out

    def embed(self, token: int) -> np.ndarray:
        x = np.zeros(self.n_embd, np.float32)
        if oracle().mo_llm_embed(self.h, token, x.ctypes.data):
            raise RuntimeError("oracle embed failed")
        return x

    def layer(self, il: int, pos: int, x) -> np.ndarray:
        """Residual after decoder layer il at pos for input x (writes the layer's K/V row)."""
        xi = np.ascontiguousarray(x, np.float32)
        out = np.zeros(self.n_embd, np.float32)
        if oracle().mo_llm_layer(self.h, il, pos, xi.ctypes.data, out.ctypes.data):
            raise RuntimeError("oracle layer failed")
        return out

    def head(self, x) -> np.ndarray:
        xi = np.ascontiguousarray(x, np.float32)
        out = np.zeros(self.n_vocab, np.float32)
        oracle().mo_llm_head(self.h, xi.ctypes.data, out.ctypes.data)
        return out

    def kv(self, il: int, n_pos: int):
        """F16 K, V rows [0, n_pos) of layer il: two [n_kv, n_pos, hd] float16 arrays."""
        k = np.zeros((self.n_kv, n_pos, self.head_dim), np.float16)
        v = np.zeros_like(k)
        oracle().mo_llm_kv(self.h, il, n_pos, k.ctypes.data, v.ctypes.data, 0)
        return k, v

    def is_conv(self, il: int) -> bool:
        """lfm2: layer il is a gated short-conv layer."""
        return bool(oracle().mo_llm_is_conv(self.h, il))

    def conv_ring(self, il: int) -> np.ndarray:
        """lfm2 short-conv ring of layer il: [4, n_embd], bx of position p in row p & 3."""
        r = np.zeros((4, self.n_embd), np.float32)
        oracle().mo_llm_conv(self.h, il, r.ctypes.data, 0)
        return r

    def set_conv_ring(self, il: int, ring):
        r = np.ascontiguousarray(ring, np.float32)
        oracle().mo_llm_conv(self.h, il, r.ctypes.data, 1)

    def set_kv(self, il: int, k, v):
        k = np.ascontiguousarray(k, np.float16)
        v = np.ascontiguousarray(v, np.float16)
        oracle().mo_llm_kv(self.h, il, k.shape[1], k.ctypes.data, v.ctypes.data, 1)

    def generate(self, prompt, max_tokens, temperature=0.8, seed=42, allow=(-1, -1), eos=(-1, -1)):
        lo = 0 if allow[0] < 0 else allow[0]
        hi = self.n_vocab if allow[1] < 0 else allow[1]
        self.reset()
        logits = None
        for i, t in enumerate(prompt):
            logits = self.eval(int(t), i)
        pos = len(prompt)
        out = []
        # step counter of the GPU sampler = decode steps so far (prefill steps included)
        step = len(prompt) - 1
        for _ in range(max_tokens):
            tok = sample(logits, temperature, seed, step, lo, hi)
            if tok in eos:
                break
            out.append(tok)
            logits = self.eval(tok, pos)
            pos += 1
            step += 1
        return np.array(out, np.int32)


def sample(logits: np.ndarray, temperature: float, seed: int, step: int, lo: int, hi: int) -> int:
    logits = np.ascontiguousarray(logits, dtype=np.float32)
    return int(oracle().mo_sample(logits.ctypes.data, temperature, seed, step, lo, hi))


def set_threads(n: int) -> int:
    """OpenMP threads of the oracle's loops; returns the previous maximum."""
    return int(oracle().mo_set_threads(int(n)))
