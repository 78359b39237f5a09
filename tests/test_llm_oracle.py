"""CPU: LLM oracle (oracle/llm_ref.c, quant_ref.c), quantizers and the shared sampler.

The decode-step oracle is "parity unpinned" (llama.cpp/ggml absent). What is
pinned here without ggml: the public block layouts (quantize -> dequantize round trips
within the format's resolution), the activation quantizers against a numpy restatement
of quantize_row_q8_K_ref / quantize_row_q8_0_ref, and the sampler's distribution
(temperature + Gumbel-max draws from softmax(logits / T), the distribution llama.cpp's
temp -> dist chain samples, test-to-speech.cpp:127-130).
"""
import ctypes

import numpy as np
import pytest

import miotts_amd as m
from miotts_amd import gguf_np
import pyoracle


def _dequant(qtype, rows_bytes, k):
    o = pyoracle.oracle()
    out = np.zeros((rows_bytes.shape[0], k), np.float32)
    for r in range(rows_bytes.shape[0]):
        rb = np.ascontiguousarray(rows_bytes[r])
        assert o.mo_dequantize_row(qtype, rb.ctypes.data, k, out[r].ctypes.data) == 0
    return out


@pytest.mark.parametrize("qtype,tol", [(8, 1.0 / 127), (12, 1.0 / 15 * 1.2), (14, 1.0 / 31 * 1.2)])
def test_quantize_dequantize_roundtrip(qtype, tol):
    rng = np.random.default_rng(qtype)
    x = (rng.standard_normal((6, 512)) * 0.02).astype(np.float32)
    q = m.quantize_rows(qtype, x)
    y = _dequant(qtype, q, 512)
    # error bounded by the format's step relative to the (sub)block range
    assert np.abs(y - x).max() <= tol * np.abs(x).max() + 1e-6


def _np_q8k(x):
    """numpy restatement of ggml quantize_row_q8_K_ref."""
    nb = len(x) // 256
    d = np.zeros(nb, np.float32)
    qs = np.zeros(len(x), np.int8)
    bs = np.zeros(nb * 16, np.int16)
    for i in range(nb):
        blk = x[i * 256:(i + 1) * 256]
        j = int(np.argmax(np.abs(blk)))
        if blk[j] == 0:
            continue
        iscale = np.float32(-127.0) / blk[j]
        q = np.rint((iscale * blk).astype(np.float32)).astype(np.int32)
        q = np.minimum(q, 127)
        qs[i * 256:(i + 1) * 256] = q
        bs[i * 16:(i + 1) * 16] = q.reshape(16, 16).sum(1)
        d[i] = np.float32(1.0) / iscale
    return d, qs, bs


def test_q8k_activation_quantizer_matches_numpy():
    o = pyoracle.oracle()
    o.mo_quantize_q8_K.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    rng = np.random.default_rng(1)
    x = rng.standard_normal(2048).astype(np.float32)
    x[5] = -7.5  # signed max
    d = np.zeros(8, np.float32)
    qs = np.zeros(2048, np.int8)
    bs = np.zeros(128, np.int16)
    o.mo_quantize_q8_K(x.ctypes.data, 2048, d.ctypes.data, qs.ctypes.data, bs.ctypes.data)
    d2, qs2, bs2 = _np_q8k(x)
    assert np.array_equal(qs, qs2) and np.array_equal(bs, bs2) and np.array_equal(d, d2)


@pytest.fixture(scope="module")
def tiny_llms(tmp_path_factory):
    d = tmp_path_factory.mktemp("llm")
    return {p: m.synth_llm(str(d / f"llm{p}.gguf"), p, 1) for p in (0, 1)}


def test_synth_llm_format(tiny_llms):
    g = gguf_np.GGUFReader(tiny_llms[1])
    assert g.kv["general.architecture"] == "qwen3"
    toks = g.kv["tokenizer.ggml.tokens"]
    assert toks[256] == "<|startoftext|>" and toks[258] == "<|im_end|>"
    assert toks[m.SYNTH_SPEECH0] == "<|s_0|>" and toks[m.SYNTH_SPEECH0 + 12799] == "<|s_12799|>"
    types = {t.name: t.type for t in g.tensors}
    assert types["blk.0.attn_q.weight"] == 12 and types["token_embd.weight"] == 14
    assert types["blk.2.ffn_down.weight"] == 14  # use_more_bits layer (Q4_K_M recipe)
    assert types["blk.0.attn_q_norm.weight"] == 0


@pytest.mark.parametrize("preset", [0, 1])
def test_oracle_llm_deterministic_and_in_range(tiny_llms, preset):
    o = pyoracle.Llm(tiny_llms[preset], 128)
    prompt = [256, 257, 72, 105, 258, 257]
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    a = o.generate(prompt, 24, 0.8, 42, allow=allow)
    b = o.generate(prompt, 24, 0.8, 42, allow=allow)
    assert np.array_equal(a, b) and len(a) == 24
    assert ((a >= allow[0]) & (a < allow[1])).all()
    g = o.generate(prompt, 8, 0.0, 0)  # greedy
    o.reset()
    for i, t in enumerate(prompt):
        lg = o.eval(t, i)
    assert g[0] == int(np.argmax(lg))


def test_sampler_distribution_matches_softmax():
    """Gumbel-max with temperature samples softmax(logits/T) (llama.cpp temp -> dist)."""
    logits = np.array([1.0, 2.0, 0.5, -1.0, 1.5], np.float32)
    T = 0.8
    n = 20000
    counts = np.zeros(5)
    for step in range(n):
        counts[pyoracle.sample(logits, T, 42, step, 0, 5)] += 1
    p = np.exp(logits / T - (logits / T).max())
    p /= p.sum()
    assert np.abs(counts / n - p).max() < 0.015
    assert pyoracle.sample(logits, 0.0, 42, 0, 0, 5) == 1
    assert pyoracle.sample(logits, 0.8, 42, 3, 2, 4) in (2, 3)


def test_qwen2_bias_oracle_and_rewrite(tmp_path):
    """Synthetic qwen2 (preset 5) carries attn_{q,k,v}.bias; the oracle adds them before RoPE
    (llama.cpp build_qwen2: Qcur = ggml_add(ggml_mul_mat(wq, cur), bq)), so logits move when
    the biases are dropped (gguf_np.rewrite, the GPU loader tests' file patcher)."""
    src = m.synth_llm(str(tmp_path / "q2.gguf"), 5, 1)
    r = gguf_np.GGUFReader(src)
    assert r.kv["general.architecture"] == "qwen2"
    assert {"blk.0.attn_q.bias", "blk.0.attn_k.bias", "blk.0.attn_v.bias"} <= set(r.by_name)
    nob = str(tmp_path / "nobias.gguf")
    gguf_np.rewrite(src, nob, drop_suffix=".bias")
    r2 = gguf_np.GGUFReader(nob)
    assert not any(t.name.endswith(".bias") for t in r2.tensors)
    assert np.array_equal(r2.tensor("blk.1.ffn_up.weight").raw(), r.tensor("blk.1.ffn_up.weight").raw())
    a = pyoracle.Llm(src, 32).eval(300, 0)
    b = pyoracle.Llm(nob, 32).eval(300, 0)
    assert np.sqrt(np.mean((a - b).astype(np.float64) ** 2)) >= 0.2 * np.sqrt(np.mean(b.astype(np.float64) ** 2))
    lf = str(tmp_path / "lfm2.gguf")
    gguf_np.rewrite(src, lf, arch="lfm2")
    assert gguf_np.GGUFReader(lf).kv["general.architecture"] == "lfm2"


def _np_q45_codes(qtype, blocks):
    """numpy restatement of ggml dequantize_row_q4_0 / _q5_0 codes (before * d): blocks
    [n][18 | 22] bytes -> [n][32] int codes and the f16 scales."""
    d = blocks[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
    if qtype == 2:
        qs = blocks[:, 2:18].astype(np.int32)
        lo, hi = (qs & 0x0F) - 8, (qs >> 4) - 8
    else:
        qh = blocks[:, 2:6].copy().view(np.uint32)[:, 0].astype(np.int64)
        qs = blocks[:, 6:22].astype(np.int32)
        j = np.arange(16)
        lo = (qs & 0x0F) | ((((qh[:, None] >> j) << 4) & 0x10)).astype(np.int32)
        hi = (qs >> 4) | ((qh[:, None] >> (j + 12)) & 0x10).astype(np.int32)
        lo, hi = lo - 16, hi - 16
    return np.concatenate([lo, hi], axis=1), d


@pytest.mark.parametrize("qtype", [2, 6])
def test_q4_0_q5_0_rows(qtype):
    """llama-quantize's Q4_K fallback (Q5_0) and Q4_0: the host quantizer's blocks decode to
    the same values in the oracle (mo_dequantize_row) and in a numpy restatement of ggml's
    dequantizer, within the format's step of the input; the oracle's vec_dot_q5_0_q8_0 /
    q4_0_q8_0 equals the numpy block sum over Q8_0 activations (the GPU runs these rows as
    the equal Q8_0 rows, tests/test_llm_gpu.py)."""
    rng = np.random.default_rng(40 + qtype)
    k = 576
    x = (rng.standard_normal((5, k)) * 0.02).astype(np.float32)
    x[1, 7] = 0.3  # a positive block max (d < 0)
    q = m.quantize_rows(qtype, x)
    bb = 18 if qtype == 2 else 22
    codes, d = _np_q45_codes(qtype, q.reshape(-1, bb))
    lo = -8 if qtype == 2 else -16
    assert codes.min() >= lo and codes.max() <= -lo - 1
    want = (codes.astype(np.float32) * d[:, None]).reshape(5, k)
    got = _dequant(qtype, q, k)
    assert np.array_equal(got, want)
    step = 1.0 / (8 if qtype == 2 else 16)
    blk = np.abs(x.reshape(-1, 32)).max(1, keepdims=True)
    assert (np.abs(got - x).reshape(-1, 32) <= step * blk * 1.01 + 1e-7).all()
    # vec_dot against Q8_0 activations (ggml vec_dot_type)
    a = rng.standard_normal(k).astype(np.float32)
    o = pyoracle.oracle()
    o.mo_matvec.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                            ctypes.c_void_p]
    y = np.zeros(5, np.float32)
    assert o.mo_matvec(qtype, q.ctypes.data, 5, k, a.ctypes.data, y.ctypes.data) == 0
    aq = a.reshape(-1, 32)
    da = (np.abs(aq).max(1) / 127).astype(np.float16).astype(np.float32)
    ida = np.where(da > 0, 1.0 / (np.abs(aq).max(1) / 127), 0).astype(np.float32)
    qa = np.round(aq * ida[:, None]).astype(np.int32)
    c = codes.reshape(5, -1, 32)
    ref = ((d.reshape(5, -1) * da[None]) * (c * qa[None]).sum(2)).sum(1)
    assert np.allclose(y, ref, rtol=1e-5, atol=1e-6)


def test_bf16_rows_and_vec_dot():
    """BF16 weights (the published MioTTS BF16 GGUFs): the host quantizer rounds to nearest
    even (ggml_compute_fp32_to_bf16, checked on a tie and a NaN), the oracle decodes the
    rows exactly, and its vec_dot_bf16 equals a numpy sum (double) of the f32 products of the
    weights with the bf16-rounded activation."""
    def bf16(x):
        u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
        r = ((u + (0x7FFF + ((u >> 16) & 1))) >> 16).astype(np.uint16)
        nan = (u & 0x7FFFFFFF) > 0x7F800000
        return np.where(nan, ((u >> 16) | 64).astype(np.uint16), r)
    rng = np.random.default_rng(30)
    k = 576
    x = (rng.standard_normal((4, k)) * 0.05).astype(np.float32)
    x[0, 0] = np.float32(1.0 + 2.0 ** -8)  # a tie: rounds to even (1.0)
    x[0, 1] = np.float32(1.0 + 3 * 2.0 ** -8)  # a tie: rounds up to even
    q = m.quantize_rows(30, x)
    h = q.view(np.uint16).reshape(4, k)
    assert np.array_equal(h, bf16(x))
    assert h[0, 0] == 0x3F80 and h[0, 1] == 0x3F82
    got = _dequant(30, q, k)
    assert np.array_equal(got, (h.astype(np.uint32) << 16).view(np.float32))
    a = rng.standard_normal(k).astype(np.float32)
    o = pyoracle.oracle()
    o.mo_matvec.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                            ctypes.c_void_p]
    y = np.zeros(4, np.float32)
    assert o.mo_matvec(30, q.ctypes.data, 4, k, a.ctypes.data, y.ctypes.data) == 0
    ab = (bf16(a).astype(np.uint32) << 16).view(np.float32)
    ref = np.array([np.sum((got[r] * ab).astype(np.float64)) for r in range(4)], np.float32)
    assert np.array_equal(y, ref)
