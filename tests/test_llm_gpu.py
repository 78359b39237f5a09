"""GPU parity: HIP LLM decode step (csrc/hip/llm_kernels.hip) vs the oracle.

1. Single matvec per quant type (Q8_0 / Q4_K / Q6_K) on random data: the GPU's per-
   superblock integer sums are exact, only the float sum over superblocks is reordered:
   |y_gpu - y_ref| <= 1e-5 * sum_b |partial_b| (bounded here by 2e-5 * max|y| + 1e-6).
2. Teacher-forced logits over 80 positions (crosses the 64-position attention split):
   exact while no activation re-quantization code flips (measured 0.0 / 2e-7 at pos 0-1);
   beyond that, int8 re-quantization (the reference's own semantics) turns ulp-level f32
   differences into single-code flips, measured <= 1.3e-2 of max|logit| on the tiny models
   and ~4e-2 RMS after the 28 layers of the 1.7B model. Bounds: tiny max rel <= 5e-2,
   argmax agreement >= 95%; 1.7B RMS(diff) <= 0.1 * RMS(logits), top-1 equal.
3. Free-running sampling (temperature 0.8, seed 42, speech ids only): sampled ids equal the
   oracle's (shared counter-based Gumbel-max sampler) for >= 95% of 40 tokens (measured 100%).
"""
import numpy as np
import pytest

import miotts_amd as m
import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def llm_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("llm_gpu")
    return {p: m.synth_llm(str(d / f"llm{p}.gguf"), p, 1) for p in (0, 1)}


@pytest.mark.parametrize("qtype,k", [(8, 576), (8, 2048), (12, 2048), (12, 6144), (14, 2048), (14, 768)])
def test_matvec_exact_per_type(device, qtype, k):
    rng = np.random.default_rng(qtype * 1000 + k)
    rows = 37
    w = (rng.standard_normal((rows, k)) * 0.05).astype(np.float32)
    wq = m.quantize_rows(qtype, w)
    x = rng.standard_normal(k).astype(np.float32)
    x[3] = -9.0
    y = m.debug_matvec(device, qtype, wq, k, x)
    yo = np.zeros(rows, np.float32)
    o = pyoracle.oracle()
    o.mo_matvec.argtypes = [pyoracle.ctypes.c_uint32, pyoracle.ctypes.c_void_p, pyoracle.ctypes.c_int,
                            pyoracle.ctypes.c_int64, pyoracle.ctypes.c_void_p, pyoracle.ctypes.c_void_p]
    assert o.mo_matvec(qtype, wq.ctypes.data, rows, k, x.ctypes.data, yo.ctypes.data) == 0
    assert np.abs(y - yo).max() <= 2e-5 * np.abs(yo).max() + 1e-6, np.abs(y - yo).max()


@pytest.mark.parametrize("preset", [0, 1])
def test_teacher_forced_logits_tiny(device, llm_files, preset):
    g = m.Llm(device, llm_files[preset], 256)
    o = pyoracle.Llm(llm_files[preset], 256)
    rng = np.random.default_rng(preset)
    toks = rng.integers(0, g.n_vocab, 80)
    agree = 0
    for pos, t in enumerate(toks):
        lg, lo = g.eval(int(t), pos), o.eval(int(t), pos)
        rel = np.abs(lg - lo).max() / np.abs(lo).max()
        if pos < 2:
            assert rel <= 1e-5, (pos, rel)
        assert rel <= 5e-2, (pos, rel)
        agree += int(lg.argmax() == lo.argmax())
    assert agree >= 76


@pytest.mark.parametrize("preset", [0, 1])
def test_generate_matches_oracle(device, llm_files, preset):
    g = m.Llm(device, llm_files[preset], 256)
    o = pyoracle.Llm(llm_files[preset], 256)
    prompt = [256, 257, 84, 101, 115, 116, 258, 257]
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    tg = g.generate(prompt, 40, 0.8, 42, allow=allow)
    to = o.generate(prompt, 40, 0.8, 42, allow=allow)
    assert len(tg) == 40 and ((tg >= allow[0]) & (tg < allow[1])).all()
    assert (tg == to).sum() >= 38
    # reproducible run to run
    assert np.array_equal(tg, g.generate(prompt, 40, 0.8, 42, allow=allow))


def test_generate_stops_at_eos(device, llm_files):
    g = m.Llm(device, llm_files[0], 256)
    prompt = [256, 257, 65, 258, 257]
    # allow only [SPEECH0 - 1, SPEECH0 + 3) where SPEECH0 - 1 = <|endoftext|> is the eos
    toks = g.generate(prompt, 200, 2.0, 7, allow=(m.SYNTH_EOT, m.SYNTH_SPEECH0 + 3),
                      eos=(m.SYNTH_EOT, m.SYNTH_IM_END), check_interval=20)
    assert len(toks) < 200 and (toks != m.SYNTH_EOT).all()


def test_logits_1p7b_q4km(device, tmp_path):
    path = m.synth_llm(str(tmp_path / "llm17.gguf"), 3, 1)
    g = m.Llm(device, path, 256)
    assert g.n_layer == 28 and g.n_vocab == 164736
    o = pyoracle.Llm(path, 256)
    toks = [256, 257, 1000, 5000]
    for pos, t in enumerate(toks):
        lg, lo = g.eval(t, pos), o.eval(t, pos)
        d = lg.astype(np.float64) - lo
        assert np.sqrt(np.mean(d * d)) <= 0.1 * np.sqrt(np.mean(lo.astype(np.float64) ** 2))
        assert lg.argmax() == lo.argmax()


# --- batched prompt prefill (csrc/hip/llm_prefill.hip; reference prefill llama_decode,
# test-to-speech.cpp:132-148). The batched kernels run the decode step's arithmetic token by
# token in the same order, so the last token's logits (and therefore the KV cache rows they
# read) equal a token-by-token decode BIT FOR BIT; vs the oracle the teacher-forced bound
# above applies.
@pytest.mark.parametrize("preset,n", [(0, 2), (0, 17), (1, 40), (0, 150)])
def test_batched_prefill_matches_sequential(device, llm_files, preset, n):
    g = m.Llm(device, llm_files[preset], 256)
    toks = np.random.default_rng(100 + n).integers(0, g.n_vocab, n)
    batched = g.prefill(toks)
    seq = None
    for pos, t in enumerate(toks):
        seq = g.eval(int(t), pos)
    assert np.array_equal(batched, seq), float(np.abs(batched - seq).max())
    o = pyoracle.Llm(llm_files[preset], 256)
    for pos, t in enumerate(toks):
        lo = o.eval(int(t), pos)
    assert np.abs(batched - lo).max() <= 5e-2 * np.abs(lo).max()


def test_batched_prefill_then_generate(device, llm_files):
    """generate() prefills in batches; the sampled ids still follow the oracle's decode."""
    g = m.Llm(device, llm_files[1], 256)
    o = pyoracle.Llm(llm_files[1], 256)
    prompt = list(range(256, 259)) + list(b"batched prefill of a longer prompt, 40 tokens") + [257]
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    tg = g.generate(prompt, 24, 0.8, 42, allow=allow)
    to = o.generate(prompt, 24, 0.8, 42, allow=allow)
    assert len(tg) == 24 and (tg == to).sum() >= 22


def test_batched_prefill_1p7b_q4km(device, tmp_path):
    """1.7B Q4_K_M, 68-token prompt (the bench prompt length: 5 chunks of 16, Q4_K + Q6_K)."""
    path = m.synth_llm(str(tmp_path / "llm17.gguf"), 3, 1)
    g = m.Llm(device, path, 256)
    toks = np.random.default_rng(68).integers(0, 151936, 68)
    batched = g.prefill(toks)
    for pos, t in enumerate(toks):
        seq = g.eval(int(t), pos)
    assert np.array_equal(batched, seq), float(np.abs(batched - seq).max())
