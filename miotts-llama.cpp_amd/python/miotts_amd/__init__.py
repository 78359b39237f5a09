"""ctypes binding over libmiotts.so's C-ABI (include/mio_hip.h).

This is the Python-side mirror used by tests/ and bench.py. The product path is the
HIP library; there is no CPU fallback here: if libmiotts.so is missing or no GPU is
visible, every call raises (the driver checks that native code is what ran).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REPO_ROOT = os.path.dirname(PKG_ROOT)
# MIO_BUILD_DIR: an alternative in-tree build (A/B experiments of compile-time variants)
BUILD_DIR = os.environ.get("MIO_BUILD_DIR") or os.path.join(PKG_ROOT, "build")
LIB_PATH = os.path.join(BUILD_DIR, "libmiotts.so")
# test-support library (include/mio_hip_test.h: synthetic GGUF writers, kernel parity entries)
TEST_LIB_PATH = os.path.join(BUILD_DIR, "libmiotts_test.so")
INCLUDE_DIR = os.path.join(REPO_ROOT, "include")

MIO_IN_DEVICE = 1
MIO_OUT_DEVICE = 2
MIO_CODEC_INCREMENTAL = 4

_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p


class HipError(RuntimeError):
    pass


class _Libs:
    """The product library and, behind it, the test-support library: an entry point is looked
    up in libmiotts.so first, then in libmiotts_test.so."""

    def __init__(self, product: ctypes.CDLL, test: Optional[ctypes.CDLL]):
        self.product, self.test = product, test

    def __getattr__(self, name):
        f = getattr(self.product, name, None)
        if f is None and self.test is not None:
            f = getattr(self.test, name, None)
        if f is None:
            raise AttributeError(name)
        return f


def lib() -> _Libs:
    """Load libmiotts.so and libmiotts_test.so (built in-tree by __graft_entry__.build /
    `make`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not built: run `make -C miotts-llama.cpp_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        T = ctypes.CDLL(TEST_LIB_PATH, mode=ctypes.RTLD_GLOBAL) if os.path.exists(TEST_LIB_PATH) else None
        _declare(L)
        if T is not None:
            _declare(T)
        _lib = _Libs(L, T)
    return _lib


def _declare(L: ctypes.CDLL) -> None:
    c_int, c_size = ctypes.c_int, ctypes.c_size_t
    sig = {
        "mio_hip_last_error": (ctypes.c_char_p, []),
        "mio_hip_device_count": (c_int, [ctypes.POINTER(c_int)]),
        "mio_hip_device_open": (c_int, [c_int, ctypes.POINTER(_vp)]),
        "mio_hip_device_close": (None, [_vp]),
        "mio_hip_device_sync": (c_int, [_vp]),
        "mio_hip_device_cu_count": (c_int, [_vp, ctypes.POINTER(c_int)]),
        "mio_hip_malloc": (c_int, [_vp, c_size, ctypes.POINTER(_vp)]),
        "mio_hip_free": (c_int, [_vp, _vp]),
        "mio_hip_memcpy_h2d": (c_int, [_vp, _vp, _vp, c_size]),
        "mio_hip_memcpy_d2h": (c_int, [_vp, _vp, _vp, c_size]),
        "mio_hip_memset": (c_int, [_vp, _vp, c_int, c_size]),
        "mio_hip_timer_mark": (c_int, [_vp, _vp, c_int]),
        "mio_hip_timer_elapsed": (c_int, [_vp, c_int, c_int, _f32p]),
        "mio_hip_pcm_finish": (c_int, [_vp, _vp, ctypes.c_int64, c_int, _vp, _f32p, _vp]),
        "mio_hip_pcm_normalize": (c_int, [_vp, _vp, ctypes.c_int64, _vp, _f32p, _vp]),
        "mio_hip_istft_create": (c_int, [_vp, c_int, c_int, ctypes.POINTER(_vp)]),
        "mio_hip_istft_destroy": (None, [_vp]),
        "mio_hip_istft_out_len": (c_int, [_vp, c_int, c_int, ctypes.POINTER(c_int)]),
        "mio_hip_istft_run": (c_int, [_vp, _vp, c_int, c_int, _vp, ctypes.POINTER(c_int),
                                      ctypes.c_uint, _vp]),
        "mio_hip_codec_load": (c_int, [_vp, ctypes.c_char_p, ctypes.POINTER(_vp)]),
        "mio_hip_codec_free": (None, [_vp]),
        "mio_hip_codec_info": (c_int, [_vp, _i32p]),
        "mio_hip_codec_decode": (c_int, [_vp, _vp, c_int, _vp, _vp, ctypes.POINTER(c_int),
                                         ctypes.c_uint, _vp]),
        "mio_hip_codec_decode_pcm": (c_int, [_vp, _vp, c_int, _vp, _vp, ctypes.POINTER(c_int),
                                             ctypes.c_uint, _vp]),
        "mio_hip_codec_decode_pcm_batch": (c_int, [_vp, _vp, _vp, c_int, _vp, _vp, _vp, ctypes.c_uint, _vp]),
        "mio_hip_codec_decode_stage": (c_int, [_vp, _vp, c_int, _vp, c_int, _vp,
                                               ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
        "mio_synth_codec_gguf": (c_int, [ctypes.c_char_p, c_int, ctypes.c_uint64]),
        "mio_synth_voice_gguf": (c_int, [ctypes.c_char_p, ctypes.c_uint64]),
        "mio_synth_llm_gguf": (c_int, [ctypes.c_char_p, c_int, ctypes.c_uint64]),
        "mio_hip_llm_load": (c_int, [_vp, ctypes.c_char_p, c_int, ctypes.POINTER(_vp)]),
        "mio_hip_llm_free": (None, [_vp]),
        "mio_normalize_tts_text": (c_int, [ctypes.c_char_p, _vp, c_int, ctypes.POINTER(c_int)]),
        "mio_parse_speech_tokens": (c_int, [ctypes.c_char_p, _vp, c_int, ctypes.POINTER(c_int)]),
        "mio_wav_encode": (c_int, [_vp, c_int, c_int, _vp, c_int, ctypes.POINTER(c_int)]),
        "mio_hip_llm_time_kernel": (c_int, [_vp, c_int, c_int, _f32p, ctypes.POINTER(ctypes.c_uint64)]),
        "mio_hip_llm_trace_kernel": (c_int, [_vp, c_int, _vp]),
        "mio_tokenizer_load": (c_int, [ctypes.c_char_p, ctypes.POINTER(_vp)]),
        "mio_stream_cadence": (c_int, [c_int, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_int64)]),
        "mio_tokenizer_free": (None, [_vp]),
        "mio_tokenizer_info": (c_int, [_vp, ctypes.POINTER(c_int)]),
        "mio_tokenize": (c_int, [_vp, ctypes.c_char_p, c_int, c_int, _vp, c_int, ctypes.POINTER(c_int)]),
        "mio_token_piece": (c_int, [_vp, ctypes.c_int32, ctypes.c_char_p, c_int, ctypes.POINTER(c_int)]),
        "mio_hip_llm_timeline": (c_int, [_vp, _vp, c_int, ctypes.POINTER(c_int)]),
        "mio_hip_codec_last_timings": (c_int, [_vp, _f32p]),
        "mio_hip_codec_last_reused": (c_int, [_vp, ctypes.POINTER(c_int)]),
        "mio_hip_codec_last_flops": (c_int, [_vp, ctypes.POINTER(ctypes.c_double)]),
        "mio_hip_llm_load_ms": (c_int, [_vp, ctypes.POINTER(ctypes.c_double)]),
        "mio_hip_llm_steps_issued": (c_int, [_vp, ctypes.POINTER(c_int)]),
        "mio_hip_llm_tail": (c_int, [_vp, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_float)]),
        "mio_hip_llm_step_kinds": (c_int, [_vp, _vp, c_int, ctypes.POINTER(c_int)]),
        "mio_hip_llm_conv_ring": (c_int, [_vp, c_int, _vp, c_int]),
        "mio_hip_llm_eval_layers": (c_int, [_vp, ctypes.c_int32, c_int, _vp, _vp]),
        "mio_hip_llm_kv_rows": (c_int, [_vp, c_int, c_int, _vp, _vp]),
        "mio_hip_debug_matvec": (c_int, [_vp, ctypes.c_uint32, _vp, c_int, c_int, _vp, _vp]),
        "mio_quantize_rows": (c_int, [ctypes.c_uint32, _vp, c_int, c_int, _vp]),
        "mio_hip_debug_mmq": (c_int, [_vp, ctypes.c_uint32, _vp, c_int, c_int, _vp, c_int, c_int, _vp, _vp]),
        "mio_hip_llm_info": (c_int, [_vp, _i32p]),
        "mio_hip_llm_weight_bytes": (c_int, [_vp, ctypes.POINTER(ctypes.c_uint64)]),
        "mio_hip_llm_eval": (c_int, [_vp, ctypes.c_int32, c_int, _vp]),
        "mio_hip_llm_prefill": (c_int, [_vp, _vp, c_int, _vp]),
        "mio_hip_llm_logits": (c_int, [_vp, _vp]),
        "mio_hip_llm_generate": (c_int, [_vp, _vp, c_int, c_int, ctypes.c_float, ctypes.c_uint64,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, _vp,
                                         ctypes.POINTER(c_int)]),
        "mio_hip_llm_generate_batch": (c_int, [_vp, _vp, _vp, c_int, c_int, ctypes.c_float, _vp,
                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, _vp, _vp]),
    }
    for name, (res, args) in sig.items():
        # a library built from an older tree (same-box A/B of MIO_BUILD_DIR builds) may lack
        # newer entry points: they stay unbound and fail when called; tests/test_capi_exports.py
        # checks that the built library exports every symbol include/mio_hip.h declares
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def check(rc: int) -> None:
    if rc != 0:
        msg = lib().mio_hip_last_error()
        raise HipError(f"rc={rc}: {msg.decode() if msg else ''}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().mio_hip_device_count(ctypes.byref(n)))
    return n.value


class Device:
    """One opened GPU (mio_hip_device)."""

    def __init__(self, dev: int = 0):
        h = _vp()
        check(lib().mio_hip_device_open(dev, ctypes.byref(h)))
        self.h = h
        self.dev = dev

    def close(self) -> None:
        if self.h:
            lib().mio_hip_device_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self) -> None:
        check(lib().mio_hip_device_sync(self.h))

    def cu_count(self) -> int:
        n = ctypes.c_int(0)
        check(lib().mio_hip_device_cu_count(self.h, ctypes.byref(n)))
        return n.value

    # --- device buffers ---
    def malloc(self, nbytes: int) -> int:
        p = _vp()
        check(lib().mio_hip_malloc(self.h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, p: int) -> None:
        check(lib().mio_hip_free(self.h, p))

    def upload(self, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        buf = DeviceArray(self, a.nbytes, a.dtype, a.shape)
        check(lib().mio_hip_memcpy_h2d(self.h, buf.ptr, _ptr(a), a.nbytes))
        return buf

    def empty(self, shape, dtype) -> "DeviceArray":
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        return DeviceArray(self, n, dtype, tuple(shape) if not isinstance(shape, int) else (shape,))

    # --- event timers ---
    def mark(self, slot: int, stream: int = 0) -> None:
        check(lib().mio_hip_timer_mark(self.h, stream or None, slot))

    def elapsed_ms(self, a: int, b: int) -> float:
        ms = ctypes.c_float(0)
        check(lib().mio_hip_timer_elapsed(self.h, a, b, ctypes.byref(ms)))
        return ms.value


class DeviceArray:
    def __init__(self, dev: Device, nbytes: int, dtype, shape):
        self.dev = dev
        self.nbytes = nbytes
        self.dtype = np.dtype(dtype)
        self.shape = tuple(shape)
        self.ptr = dev.malloc(nbytes)

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        if self.nbytes:
            check(lib().mio_hip_memcpy_d2h(self.dev.h, _ptr(out), self.ptr, self.nbytes))
        return out

    def free(self) -> None:
        if self.ptr:
            self.dev.free(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def pcm_finish(dev: "Device", samples: "DeviceArray", n: int, normalize: bool,
               out: Optional["DeviceArray"] = None):
    """Device PCM epilogue (mio_hip_pcm_finish): optional peak normalisation
    (test-to-speech.cpp:232-243) + int16(clamp(s * 32767)) of wav_write (wav-writer.cpp:24-44).
    Returns (int16 samples on the host, peak max|s| or 0.0 when not normalizing)."""
    if out is None:
        out = dev.empty((max(n, 1),), np.int16)
    peak = ctypes.c_float(0)
    check(lib().mio_hip_pcm_finish(dev.h, samples.ptr if n else None, n, 1 if normalize else 0,
                                   out.ptr if n else None, ctypes.byref(peak), None))
    return out.numpy()[:n], peak.value


class Istft:
    """HIP iSTFT: mirror of istft_cache + istft() (istft.h:6-42)."""

    def __init__(self, dev: Device, n_fft: int = 392, win_length: Optional[int] = None):
        self.dev = dev
        self.n_fft = n_fft
        self.win = n_fft if win_length is None else win_length
        h = _vp()
        check(lib().mio_hip_istft_create(dev.h, n_fft, self.win, ctypes.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().mio_hip_istft_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def out_len(self, n_frames: int, hop: int) -> int:
        n = ctypes.c_int(0)
        check(lib().mio_hip_istft_out_len(self.h, n_frames, hop, ctypes.byref(n)))
        return n.value

    def __call__(self, spec: np.ndarray, hop: int = 98) -> np.ndarray:
        """spec: [n_frames][n_freq][2] float32 (host). Returns the trimmed PCM."""
        spec = np.ascontiguousarray(spec, dtype=np.float32)
        n_frames = spec.shape[0] if spec.size else 0
        out = np.empty(max(self.out_len(n_frames, hop), 1), np.float32)
        n = ctypes.c_int(0)
        check(lib().mio_hip_istft_run(self.h, _ptr(spec) if spec.size else None, n_frames, hop,
                                      _ptr(out), ctypes.byref(n), 0, None))
        return out[: n.value]

    def run_device(self, spec: DeviceArray, n_frames: int, hop: int, out: DeviceArray,
                   stream: int = 0) -> int:
        n = ctypes.c_int(0)
        check(lib().mio_hip_istft_run(self.h, spec.ptr, n_frames, hop, out.ptr, ctypes.byref(n),
                                      MIO_IN_DEVICE | MIO_OUT_DEVICE, stream or None))
        return n.value


# ---------------------------------------------------------------- synthetic files
def synth_codec(path: str, preset: int = 0, seed: int = 1) -> str:
    check(lib().mio_synth_codec_gguf(path.encode(), preset, seed))
    return path


def synth_voice(path: str, seed: int = 7) -> str:
    check(lib().mio_synth_voice_gguf(path.encode(), seed))
    return path


def read_voice(path: str) -> np.ndarray:
    """First tensor of a .emb.gguf, F32 (mirror of load_voice_embedding, miocodec.cpp:816-853)."""
    from . import gguf_np
    g = gguf_np.GGUFReader(path)
    t = g.tensors[0]
    assert t.type == 0, "voice embedding must be F32"
    return t.array().astype(np.float32)


# ---------------------------------------------------------------- codec
class Codec:
    """HIP MioCodec decoder (mirror of miocodec.h: miocodec_load / miocodec_decode)."""

    def __init__(self, dev: Device, path: str):
        self.dev = dev
        h = _vp()
        check(lib().mio_hip_codec_load(dev.h, path.encode(), ctypes.byref(h)))
        self.h = h
        info = np.zeros(8, np.int32)
        check(lib().mio_hip_codec_info(h, info.ctypes.data_as(_i32p)))
        (self.sample_rate, self.n_fft, self.hop_length, self.samples_per_token, self.n_freq,
         self.up_stages, self.frames_per_code, self.n_codes) = [int(x) for x in info]

    def close(self):
        if self.h:
            lib().mio_hip_codec_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, codes, emb) -> np.ndarray:
        codes = np.ascontiguousarray(codes, dtype=np.int32)
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        out = np.empty((len(codes) * self.frames_per_code, self.n_freq, 2), np.float32)
        nf = ctypes.c_int(0)
        check(lib().mio_hip_codec_decode(self.h, _ptr(codes), len(codes), _ptr(emb), _ptr(out),
                                         ctypes.byref(nf), 0, None))
        return out[: nf.value]

    def decode_pcm(self, codes, emb, incremental: bool = False) -> np.ndarray:
        """incremental: reuse the prenet rows of the previous incremental decode for the shared
        code prefix (MIO_CODEC_INCREMENTAL; last_reused() reports how many rows)."""
        codes = np.ascontiguousarray(codes, dtype=np.int32)
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        out = np.empty(len(codes) * self.frames_per_code * self.hop_length + self.n_fft, np.float32)
        n = ctypes.c_int(0)
        check(lib().mio_hip_codec_decode_pcm(self.h, _ptr(codes), len(codes), _ptr(emb), _ptr(out),
                                             ctypes.byref(n), MIO_CODEC_INCREMENTAL if incremental else 0, None))
        return out[: n.value]

    def last_reused(self) -> int:
        r = ctypes.c_int(0)
        check(lib().mio_hip_codec_last_reused(self.h, ctypes.byref(r)))
        return r.value

    def last_flops(self) -> float:
        """Algorithmic FLOPs of the last decode_pcm (mio_hip_codec_last_flops)."""
        f = ctypes.c_double(0)
        check(lib().mio_hip_codec_last_flops(self.h, ctypes.byref(f)))
        return f.value

    def decode_pcm_device(self, codes: DeviceArray, n_codes: int, emb: DeviceArray,
                          out: DeviceArray, stream: int = 0) -> int:
        n = ctypes.c_int(0)
        check(lib().mio_hip_codec_decode_pcm(self.h, codes.ptr, n_codes, emb.ptr, out.ptr,
                                             ctypes.byref(n), MIO_IN_DEVICE | MIO_OUT_DEVICE,
                                             stream or None))
        return n.value

    def decode_pcm_batch_device(self, codes, n_codes, emb: DeviceArray, outs, stream: int = 0):
        """B utterances at once (mio_hip_codec_decode_pcm_batch): codes[b] / outs[b] are
        DeviceArrays, n_codes[b] their lengths; returns the PCM lengths."""
        B = len(codes)
        cp = (ctypes.c_void_p * B)(*[c.ptr for c in codes])
        op = (ctypes.c_void_p * B)(*[o.ptr for o in outs])
        nc = (ctypes.c_int * B)(*[int(n) for n in n_codes])
        ln = (ctypes.c_int * B)()
        check(lib().mio_hip_codec_decode_pcm_batch(self.h, ctypes.cast(cp, _vp), ctypes.cast(nc, _vp), B, emb.ptr,
                                                   ctypes.cast(op, _vp), ctypes.cast(ln, _vp),
                                                   MIO_IN_DEVICE | MIO_OUT_DEVICE, stream or None))
        return [int(x) for x in ln]

    def decode_pcm_batch(self, codes, emb):
        """Host convenience of decode_pcm_batch_device: list of code arrays -> list of PCM."""
        dev = self.dev
        d_codes = [dev.upload(np.ascontiguousarray(c, np.int32)) for c in codes]
        d_emb = dev.upload(np.ascontiguousarray(emb, np.float32))
        outs = [dev.empty((len(c) * self.samples_per_token + self.n_fft,), np.float32) for c in codes]
        lens = self.decode_pcm_batch_device(d_codes, [len(c) for c in codes], d_emb, outs)
        dev.sync()
        return [o.numpy()[:n] for o, n in zip(outs, lens)]

    def last_timings(self):
        ms = np.zeros(2, np.float32)
        check(lib().mio_hip_codec_last_timings(self.h, ms.ctypes.data_as(_f32p)))
        return float(ms[0]), float(ms[1])

    def decode_stage(self, codes, emb, stage: int, max_elems: int) -> np.ndarray:
        codes = np.ascontiguousarray(codes, dtype=np.int32)
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        out = np.empty(max_elems, np.float32)
        r, c = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().mio_hip_codec_decode_stage(self.h, _ptr(codes), len(codes), _ptr(emb), stage,
                                               _ptr(out), ctypes.byref(r), ctypes.byref(c)))
        return out[: r.value * c.value].reshape(r.value, c.value)


# ---------------------------------------------------------------- LLM
SYNTH_SPEECH0 = 260      # id of <|s_0|> in the synthetic vocabulary (csrc/testlib/synth.h)
SYNTH_IM_END = 258
SYNTH_EOT = 259


def synth_llm(path: str, preset: int = 0, seed: int = 1) -> str:
    check(lib().mio_synth_llm_gguf(path.encode(), preset, seed))
    return path


class Llm:
    """HIP LLM decode (mirror of the llama.cpp calls in test-to-speech.cpp:44-196)."""

    def __init__(self, dev: Device, path: str, n_ctx: int = 2048):
        self.dev = dev
        h = _vp()
        check(lib().mio_hip_llm_load(dev.h, path.encode(), n_ctx, ctypes.byref(h)))
        self.h = h
        info = np.zeros(8, np.int32)
        check(lib().mio_hip_llm_info(h, info.ctypes.data_as(_i32p)))
        (self.n_vocab, self.n_embd, self.n_layer, self.n_head, self.n_kv, self.head_dim,
         self.n_ff, self.n_ctx) = [int(x) for x in info]

    def close(self):
        if self.h:
            lib().mio_hip_llm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def weight_bytes(self) -> int:
        b = ctypes.c_uint64(0)
        check(lib().mio_hip_llm_weight_bytes(self.h, ctypes.byref(b)))
        return b.value

    def load_ms(self) -> float:
        """Wall time of the load (GGUF mmap -> pinned staging -> HBM arena)."""
        v = ctypes.c_double(0)
        check(lib().mio_hip_llm_load_ms(self.h, ctypes.byref(v)))
        return v.value

    def steps_issued(self) -> int:
        """Decode steps issued by the last generate, look-ahead past an end token included."""
        v = ctypes.c_int(0)
        check(lib().mio_hip_llm_steps_issued(self.h, ctypes.byref(v)))
        return v.value

    def tail(self):
        """(steps after the end token, whole intervals' steps timed, their GPU ms) of the last
        generate that stopped at an end token (mio_hip_llm_tail)."""
        a, b, ms = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_float(0)
        check(lib().mio_hip_llm_tail(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(ms)))
        return a.value, b.value, ms.value

    def eval(self, token: int, pos: int) -> np.ndarray:
        out = np.empty(self.n_vocab, np.float32)
        check(lib().mio_hip_llm_eval(self.h, token, pos, _ptr(out)))
        return out

    def prefill(self, tokens) -> np.ndarray:
        """Batched prefill of tokens[:-1] + one decode step of tokens[-1]: the last token's
        logits (the reference's prompt llama_decode, test-to-speech.cpp:132-148)."""
        t = np.ascontiguousarray(tokens, np.int32)
        out = np.empty(self.n_vocab, np.float32)
        check(lib().mio_hip_llm_prefill(self.h, _ptr(t), int(t.size), _ptr(out)))
        return out

    def logits(self) -> np.ndarray:
        out = np.empty(self.n_vocab, np.float32)
        check(lib().mio_hip_llm_logits(self.h, _ptr(out)))
        return out

    def time_kernel(self, which: int, iters: int = 50):
        ms = ctypes.c_float(0)
        b = ctypes.c_uint64(0)
        check(lib().mio_hip_llm_time_kernel(self.h, which, iters, ctypes.byref(ms), ctypes.byref(b)))
        return ms.value, b.value

    def trace_kernel(self, which: int) -> np.ndarray:
        """Checkpoint timestamps of one launch (diagnostic, mio_hip_llm_trace_kernel)."""
        out = np.zeros(32, np.uint64)
        check(lib().mio_hip_llm_trace_kernel(self.h, which, _ptr(out)))
        return out

    def timeline(self) -> np.ndarray:
        """Per-launch, per-workgroup [start, marks 1-6, end] (us from the step start, NaN =
        absent) of one graph-replayed step (diagnostic, mio_hip_llm_timeline; advances the
        decode state). Marks: see MIO_TL_MARK in csrc/hip/llm_device.h."""
        slots = 2048  # kTlSlots (csrc/hip/llm_kernels.h): workgroup slots per launch
        out = np.zeros(256 * slots * 8, np.uint64)
        n = ctypes.c_int(0)
        check(lib().mio_hip_llm_timeline(self.h, _ptr(out), 256, ctypes.byref(n)))
        t = out[: n.value * slots * 8].astype(np.float64).reshape(n.value, slots, 8)
        t[t == 0] = np.nan
        return (t - np.nanmin(t[0, :, 0])) * 0.01

    def eval_layers(self, token: int, pos: int):
        """One decode step: (residual before layer 0 and after each layer [n_layer + 1,
        n_embd], logits)."""
        xs = np.empty((self.n_layer + 1, self.n_embd), np.float32)
        lg = np.empty(self.n_vocab, np.float32)
        check(lib().mio_hip_llm_eval_layers(self.h, token, pos, _ptr(xs), _ptr(lg)))
        return xs, lg

    def kv_rows(self, il: int, n_pos: int):
        """F16 K, V cache rows [0, n_pos) of layer il: two [n_kv, n_pos, head_dim] arrays."""
        k = np.empty((self.n_kv, n_pos, self.head_dim), np.float16)
        v = np.empty_like(k)
        check(lib().mio_hip_llm_kv_rows(self.h, il, n_pos, _ptr(k), _ptr(v)))
        return k, v

    def step_kinds(self) -> list:
        """The decode step's launches in order, as time_kernel's `which` (0 attn_in,
        1 attention, 2 attn_out, 3 ffn_in, 4 ffn_down, 8 conv_in, 9 conv_out; 6 lm_head)."""
        n = ctypes.c_int(0)
        check(lib().mio_hip_llm_step_kinds(self.h, None, 0, ctypes.byref(n)))
        k = np.zeros(n.value, np.int32)
        check(lib().mio_hip_llm_step_kinds(self.h, _ptr(k), n.value, ctypes.byref(n)))
        return [int(v) for v in k]

    def conv_ring(self, il: int, ring=None):
        """lfm2 short-conv state of layer il, [4, n_embd] (slot p & 3 = B*X of position p);
        with `ring`: sets it."""
        if ring is None:
            r = np.empty((4, self.n_embd), np.float32)
            check(lib().mio_hip_llm_conv_ring(self.h, il, _ptr(r), 0))
            return r
        r = np.ascontiguousarray(ring, np.float32)
        check(lib().mio_hip_llm_conv_ring(self.h, il, _ptr(r), 1))

    def generate(self, prompt, max_tokens: int, temperature: float = 0.8, seed: int = 42,
                 allow=(-1, -1), eos=(-1, -1), check_interval: int = 20) -> np.ndarray:
        prompt = np.ascontiguousarray(prompt, dtype=np.int32)
        out = np.empty(max_tokens, np.int32)
        n = ctypes.c_int(0)
        check(lib().mio_hip_llm_generate(self.h, _ptr(prompt), len(prompt), max_tokens,
                                         temperature, seed, allow[0], allow[1], eos[0], eos[1],
                                         check_interval, _ptr(out), ctypes.byref(n)))
        return out[: n.value]

    def generate_batch(self, prompts, max_tokens: int, temperature: float = 0.8, seeds=None,
                       allow=(-1, -1), eos=(-1, -1), check_interval: int = 32):
        """B utterances decoded together (mio_hip_llm_generate_batch): one weight pass per
        step for all of them; stream b's tokens equal generate(prompts[b], seed=seeds[b])."""
        B = len(prompts)
        seeds = [42 + b for b in range(B)] if seeds is None else list(seeds)
        lens = np.array([len(p) for p in prompts], np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(p, np.int32) for p in prompts]), np.int32)
        sd = np.array(seeds, np.uint64)
        out = np.empty((B, max_tokens), np.int32)
        n = np.zeros(B, np.int32)
        check(lib().mio_hip_llm_generate_batch(self.h, _ptr(flat), _ptr(lens), B, max_tokens, temperature,
                                               _ptr(sd), allow[0], allow[1], eos[0], eos[1],
                                               check_interval, _ptr(out), _ptr(n)))
        return [out[b, : n[b]].copy() for b in range(B)]


GGML_BLOCK = {2: (32, 18), 6: (32, 22), 8: (32, 34), 12: (256, 144), 14: (256, 210), 30: (1, 2)}


def quantize_rows(qtype: int, x: np.ndarray) -> np.ndarray:
    """Host quantizer (csrc/host/quant.cpp) -> GGUF block bytes [rows][row_bytes]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    rows, k = x.shape
    be, bb = GGML_BLOCK[qtype]
    out = np.zeros((rows, k // be * bb), np.uint8)
    check(lib().mio_quantize_rows(qtype, _ptr(x), rows, k, _ptr(out)))
    return out


def debug_matvec(dev: Device, qtype: int, w_rows: np.ndarray, k: int, x: np.ndarray) -> np.ndarray:
    w_rows = np.ascontiguousarray(w_rows)
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty(w_rows.shape[0], np.float32)
    check(lib().mio_hip_debug_matvec(dev.h, qtype, _ptr(w_rows), w_rows.shape[0], k, _ptr(x), _ptr(y)))
    return y


def debug_mmq(dev: Device, qtype: int, w_rows: np.ndarray, k: int, x: np.ndarray, mode: int = 0,
              y_in: Optional[np.ndarray] = None, up_rows: Optional[np.ndarray] = None) -> np.ndarray:
    """x: [nt][k] -> y [nt][rows] on the int8-MFMA batched matmul (mio_hip_debug_mmq); mode 1
    adds y_in, mode 2 returns silu(W x) * (up x)."""
    w_rows = np.ascontiguousarray(w_rows)
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros((x.shape[0], w_rows.shape[0]), np.float32) if y_in is None else np.array(y_in, np.float32)
    up = np.ascontiguousarray(up_rows) if up_rows is not None else None
    check(lib().mio_hip_debug_mmq(dev.h, qtype, _ptr(w_rows), w_rows.shape[0], k, _ptr(x), x.shape[0], mode,
                                  _ptr(up) if up is not None else None, _ptr(y)))
    return y


# ---------------------------------------------------------------- tokenizer
class Tokenizer:
    """GGUF byte-level BPE tokenizer (csrc/host/tokenizer.h) through the C-ABI: llama_tokenize /
    llama_token_to_piece / llama_vocab_eos equivalents (test-to-speech.cpp:117-176)."""

    def __init__(self, gguf_path: str):
        h = _vp()
        check(lib().mio_tokenizer_load(gguf_path.encode(), ctypes.byref(h)))
        self.h = h
        info = (ctypes.c_int * 4)()
        check(lib().mio_tokenizer_info(self.h, info))
        self.n_vocab, self.bos, self.eos, self.im_end = list(info)

    def __del__(self):
        if getattr(self, "h", None):
            lib().mio_tokenizer_free(self.h)
            self.h = None

    def tokenize(self, text: str, add_special: bool = True, parse_special: bool = True) -> list:
        b = text.encode("utf-8")
        cap = len(b) + 16
        out = np.zeros(cap, np.int32)
        n = ctypes.c_int(0)
        check(lib().mio_tokenize(self.h, b, int(add_special), int(parse_special), _ptr(out), cap, ctypes.byref(n)))
        return out[: n.value].tolist()

    def piece(self, tok: int) -> bytes:
        cap = 1024
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_int(0)
        check(lib().mio_token_piece(self.h, int(tok), buf, cap, ctypes.byref(n)))
        return buf.raw[: n.value]

    def detokenize(self, toks) -> str:
        return b"".join(self.piece(t) for t in toks).decode("utf-8", errors="replace")


def stream_cadence(n_tokens: int):
    """(decode_calls, decoded_codes) of the streaming commit policy for n_tokens codes."""
    c, k = ctypes.c_int(0), ctypes.c_int64(0)
    check(lib().mio_stream_cadence(int(n_tokens), ctypes.byref(c), ctypes.byref(k)))
    return c.value, k.value


# ---------------------------------------------------------------- host text utilities
def normalize_text(text: str) -> str:
    """normalize_tts_text (text-normalize.h:7) via the C-ABI."""
    b = text.encode("utf-8")
    cap = 4 * len(b) + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_int(0)
    check(lib().mio_normalize_tts_text(b, out, cap, ctypes.byref(n)))
    return out.raw[: n.value].decode("utf-8")


def parse_speech_tokens(text: str) -> np.ndarray:
    b = text.encode("utf-8")
    n = ctypes.c_int(0)
    check(lib().mio_parse_speech_tokens(b, None, 0, ctypes.byref(n)))
    out = np.zeros(max(n.value, 1), np.int32)
    check(lib().mio_parse_speech_tokens(b, _ptr(out), len(out), ctypes.byref(n)))
    return out[: n.value]


def wav_bytes(samples: np.ndarray, sample_rate: int = 44100) -> bytes:
    s = np.ascontiguousarray(samples, dtype=np.float32)
    cap = 44 + 2 * len(s)
    out = np.zeros(cap, np.uint8)
    n = ctypes.c_int(0)
    check(lib().mio_wav_encode(_ptr(s) if len(s) else None, len(s), sample_rate, _ptr(out), cap,
                               ctypes.byref(n)))
    return out[: n.value].tobytes()
