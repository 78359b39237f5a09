"""GPU parity: HIP LLM decode step (csrc/hip/llm_kernels.hip) vs the oracle.

1. Single matvec per quant type (Q8_0 / Q4_K / Q6_K, and Q5_0 / Q4_0, which run as the Q8_0
   rows they equal exactly; BF16 within the same bound, its f32 sums reordered) on random
   data: the GPU's per-
   superblock integer sums are exact, only the float sum over superblocks is reordered:
   |y_gpu - y_ref| <= 1e-5 * sum_b |partial_b| (bounded here by 2e-5 * max|y| + 1e-6).
2. Teacher-forced logits: tiny models over 80 positions, the 1.7B model over 300 positions
   and the 0.1B (G = 3, hd 64) / 2.6B (G = 4, hd 64) models over 160 positions, i.e. across
   the 128-position attention chunks (kAttChunk, csrc/hip/llm_kernels.h) whose partial records
   k_attn_out merges. Exact while no activation re-quantization code flips (measured 0.0 /
   2e-7 at pos 0-1); beyond that, int8 re-quantization (the reference's own semantics, ggml
   quantizes every matvec input to the weight's vec_dot_type) turns ulp-level f32 differences
   into single-code flips, measured <= 1.3e-2 of max|logit| on the tiny models and 1-8e-2
   RMS after the 24-32 layers of the large models. That error does not depend on the
   position, so one bound holds at every position: tiny max rel <= 5e-2, argmax agreement
   >= 95%; large models RMS(diff) <= 0.1 * RMS(logits) per position, argmax agreement >= 75%
   and the oracle's argmax in the GPU's top 5 at >= 90% (near-flat synthetic logits). A wrong
   chunk merge or mask at a chunk boundary moves every later position's logits by
   O(RMS(logits)).
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
    return {p: m.synth_llm(str(d / f"llm{p}.gguf"), p, 1) for p in (0, 1, 9, 10, 11)}


@pytest.mark.parametrize("qtype,k", [(8, 576), (8, 2048), (12, 2048), (12, 6144), (14, 2048), (14, 768),
                                     (6, 576), (6, 2048), (2, 2048), (30, 576), (30, 2048), (30, 6144)])
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


def _bf16_round(x):
    """ggml_compute_fp32_to_bf16: round to nearest even (finite inputs)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32) << 16
    return r.astype(np.uint32).view(np.float32)


@pytest.mark.parametrize("k", [576, 2048, 6144])
def test_bf16_matvec_derived_bound(device, k):
    """BF16 rows (ggml vec_dot_bf16: the activation rounded to bf16, products of two bf16 exact
    in f32, f32 sums): the GPU's v_dot2 matvec against the exact (float64) dot of the same
    bf16 operands, within the f32 summation bound of its order — each lane sums its k / 64
    products in sequence, then a 6-level lane tree and the pass sum: |err| <= (k / 64 + 8) *
    2^-24 * sum_i |w_i x_i| per row (about 1e-6 of that sum at k = 2048). An f32 (unrounded)
    activation breaks it by ~2^-9: checked to exceed the bound (teeth)."""
    rng = np.random.default_rng(k + 30)
    rows = 41
    w = (rng.standard_normal((rows, k)) * 0.05).astype(np.float32)
    wq = m.quantize_rows(30, w)  # bf16 bit patterns, ggml row layout
    wb = (wq.view(np.uint16).reshape(rows, k).astype(np.uint32) << 16).view(np.float32)
    x = rng.standard_normal(k).astype(np.float32)
    y = m.debug_matvec(device, 30, wq, k, x).astype(np.float64)
    xb = _bf16_round(x)
    exact = wb.astype(np.float64) @ xb.astype(np.float64)
    sabs = np.abs(wb.astype(np.float64)) @ np.abs(xb.astype(np.float64))
    bound = (k / 64 + 8) * 2.0 ** -24 * sabs
    err = np.abs(y - exact)
    assert np.all(err <= bound), (float((err / sabs).max()), float((bound / sabs).max()))
    unrounded = wb.astype(np.float64) @ x.astype(np.float64)
    assert np.any(np.abs(y - unrounded) > bound), "bf16 rounding of the activation not observable"


# 9: Q4_K_M at the 0.1B width, whose q/k/v, O, gate/up and embedding rows (576 long) are
# llama-quantize's Q5_0 / Q8_0 fallbacks; 10: Q4_0 (Q5_0 and Q4_0 run as the equal Q8_0 rows);
# 11: BF16 (v_dot2 over the bf16-rounded activation, ggml's vec_dot_bf16)
@pytest.mark.parametrize("preset", [0, 1, 9, 10, 11])
def test_teacher_forced_logits_tiny(device, llm_files, preset):
    g = m.Llm(device, llm_files[preset], 256)
    o = pyoracle.Llm(llm_files[preset], 256)
    rng = np.random.default_rng(preset)
    toks = rng.integers(0, g.n_vocab, 80)
    agree = 0
    for pos, t in enumerate(toks):
        lg, lo = g.eval(int(t), pos), o.eval(int(t), pos)
        rel = np.abs(lg - lo).max() / np.abs(lo).max()
        # preset 9's 576-wide rows re-quantize to Q8_0 blocks (Q5_0 / Q8_0 fallbacks) with G = 3
        # heads per kv head, like the 0.1B model, whose flips start at position 0-1 too
        # (test_teacher_forced_large_models); BF16 (11) rounds every matvec input to 8
        # mantissa bits, so an f32-ulp difference of a sum flips a rounding much sooner. The
        # per-layer test (test_llm_layers_gpu.py) pins both presets' layers.
        if pos < {9: 1, 11: 0}.get(preset, 2):
            assert rel <= 1e-5, (pos, rel)
        assert rel <= 5e-2, (pos, rel)
        agree += int(lg.argmax() == lo.argmax())
    assert agree >= 76


@pytest.mark.parametrize("preset", [0, 1, 9, 11])
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
    # steps past the end token: the sampler stores it to the host's mapped word, the host stops
    # issuing step graphs (8 steps each, at most 2 queued ahead): the rest of the end token's
    # graph plus at most one more
    wasted = g.steps_issued() - len(toks) - 1
    assert 0 <= wasted <= 2 * 8 - 1, wasted
    assert g.tail()[0] == wasted
    # a run that stops at max_tokens issues exactly max_tokens steps
    toks = g.generate(prompt, 50, 0.8, 7, allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 3), check_interval=20)
    assert len(toks) == 50 and g.steps_issued() == 50 and g.tail() == (0, 0, 0.0)


# After an end token every decode launch returns at entry (StepState.done; the reference breaks
# before the next llama_decode, test-to-speech.cpp:168-170): a step queued past it costs about
# its launch boundaries (~1.5 us each) instead of streaming the weights. 1.7B Q4_K_M: 141
# launches per step, 0.77 ms per real step = 5.4 us per launch.
@pytest.mark.parametrize("preset", [3, 2])
def test_steps_after_eos_return_at_entry(device, synth_llm_path, preset):
    g = m.Llm(device, synth_llm_path(preset), 512)
    prompt = [256, 257, 65, 258, 257]
    toks = g.generate(prompt, 400, 2.0, 11, allow=(m.SYNTH_EOT, m.SYNTH_SPEECH0 + 3),
                      eos=(m.SYNTH_EOT, m.SYNTH_IM_END), check_interval=20)
    assert len(toks) < 20, len(toks)  # 1 in 4 allowed ids ends the run
    wasted, timed, ms = g.tail()
    # timed: the step graphs queued after the one that sampled the end token (0 or 8 steps)
    assert wasted == g.steps_issued() - len(toks) - 1 and wasted <= 15 and timed in (0, 8), (wasted, timed)
    if not timed:
        pytest.skip("the host saw the end token before queueing another graph: no step to time")
    us_per_launch = ms * 1e3 / timed / len(g.step_kinds())
    print(f"preset {preset}: {wasted} steps after the end token, {ms * 1e3 / timed:.1f} us per step "
          f"({us_per_launch:.2f} us per launch)")
    # measured 2.63 us per launch (370 us per step) on the 1.7B model against 5.4 us while decoding:
    # each exiting launch still waits for its first weight group and x (the flag is read behind
    # them so that decoding steps do not wait for it)
    assert us_per_launch <= 3.5, us_per_launch
    g.close()


def _teacher_forced(device, path, n_pos, seed):
    """Per-position (rel RMS diff, argmax equal) of GPU vs oracle logits over n_pos positions."""
    g = m.Llm(device, path, 512)
    o = pyoracle.Llm(path, 512)
    toks = np.random.default_rng(seed).integers(0, g.n_vocab, n_pos)
    rel, agree, top5 = [], [], []
    for pos, t in enumerate(toks):
        lg, lo = g.eval(int(t), pos), o.eval(int(t), pos)
        d = lg.astype(np.float64) - lo
        rel.append(np.sqrt(np.mean(d * d)) / np.sqrt(np.mean(lo.astype(np.float64) ** 2)))
        agree.append(lg.argmax() == lo.argmax())
        top5.append(lo.argmax() in np.argpartition(lg, -5)[-5:])
    g.close()
    _teacher_forced.top5 = np.array(top5)
    return np.array(rel), np.array(agree)


@pytest.mark.parametrize("preset,n_pos", [(3, 300), (2, 160), (4, 160)])
def test_teacher_forced_large_models(device, synth_llm_path, preset, n_pos):
    """1.7B Q4_K_M (G = 2, hd 128, qwen3 q/k norm), 0.1B Q8_0 (G = 3) and 2.6B Q8_0 (G = 4):
    every position within the bound, through chunk boundaries 128 and 256."""
    rel, agree = _teacher_forced(device, synth_llm_path(preset), n_pos, 300 + preset)
    top5 = _teacher_forced.top5
    print(f"preset {preset}: rel RMS max {rel.max():.3g} at pos {int(rel.argmax())}, "
          f"median {np.median(rel):.3g}, argmax agree {agree.sum()}/{n_pos}, oracle argmax in GPU top-5 "
          f"{top5.sum()}/{n_pos}")
    # the flip noise appears from position 0 on in the 24-32-layer models (measured 1.8e-7 at
    # position 0 of the 1.7B model, 1.1e-2 for the 0.1B Q8_0 one), so one bound holds at every
    # position
    assert rel.max() <= 0.1, (int(rel.argmax()), rel.max())
    # random synthetic weights give near-flat logits over 65k-165k ids: the top two are often
    # within the re-quantization noise, so the exact argmax flips at some positions (measured
    # 81-97%); the oracle's argmax must still be among the GPU's top five almost everywhere
    assert agree.sum() >= 0.75 * n_pos
    assert top5.sum() >= 0.9 * n_pos


def _free_run_agreement(device, path, preset, temp, n):
    g = m.Llm(device, path, 512)
    o = pyoracle.Llm(path, 512)
    prompt = [256, 257] + list(b"free run of the synthetic model") + [258, 257]
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    tg = g.generate(prompt, n, temp, 42 + preset, allow=allow)
    to = o.generate(prompt, n, temp, 42 + preset, allow=allow)
    g.close()
    assert len(tg) == len(to) == n
    same = tg == to
    first = int(np.argmin(same)) if not same.all() else n
    return tg, to, first


@pytest.mark.parametrize("preset", [2, 4])
def test_free_run_64_tokens_large_models(device, synth_llm_path, preset):
    """64 sampled ids (temperature 0.8, shared counter-based Gumbel-max), free-running on the GPU
    and in the oracle, against the same steps teacher-forced on the oracle's ids.
    Derived bound (no fitted step count): while the two free runs agree, the GPU's prefix IS the
    oracle's, so its step-k logits are bit for bit its teacher-forced step-k logits (batched
    prefill == sequential decode, one graph step == one eval); its id is then the teacher-forced
    GPU id. The free runs must therefore agree up to, and part exactly at, the first step whose
    teacher-forced ids differ (a Gumbel-perturbed top two within the logits' re-quantization
    flip noise). Every step is checked teacher-forced: the same noise gives the same id at
    >= 90% of the 64 steps (the flip noise of test_teacher_forced_large_models)."""
    path = synth_llm_path(preset)
    tg, to, first = _free_run_agreement(device, path, preset, 0.8, 64)
    g = m.Llm(device, path, 512)
    o = pyoracle.Llm(path, 512)
    prompt = [256, 257] + list(b"free run of the synthetic model") + [258, 257]
    seq = prompt + [int(t) for t in to]
    lo_, hi_ = m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800
    tf = []  # per generated step k: teacher-forced GPU id == oracle id
    gpu_ids = []
    for pos, t in enumerate(seq[:-1]):
        lg, lo = g.eval(int(t), pos), o.eval(int(t), pos)
        if pos >= len(prompt) - 1:
            step = pos  # the generate() step counter = position
            a, b = pyoracle.sample(lg, 0.8, 42 + preset, step, lo_, hi_), pyoracle.sample(lo, 0.8, 42 + preset,
                                                                                          step, lo_, hi_)
            assert b == to[pos - len(prompt) + 1]  # the oracle's teacher-forced id is its free-run id
            tf.append(a == b)
            gpu_ids.append(a)
    g.close()
    tf = np.array(tf)
    first_tf = int(np.argmin(tf)) if not tf.all() else 64
    print(f"preset {preset}: free-run first divergence at {first} of 64, first teacher-forced flip at {first_tf}; "
          f"teacher-forced sampled ids equal {int(tf.sum())}/64")
    assert first == first_tf, (first, first_tf, tg, to)
    if first < 64:
        assert tg[first] == gpu_ids[first]  # the GPU's free run took its teacher-forced id there
    assert tf.sum() >= 0.9 * 64


@pytest.mark.parametrize("preset", [0, 1, 2, 5])
def test_greedy_token_equality(device, synth_llm_path, preset):
    """Greedy decoding (-t 0: temperature <= 0 takes the argmax): the id
    stream equals the oracle's. A divergence is accepted only at a near-tie of the oracle's
    top two logits (within the 5e-2 teacher-forced bound); everything before it must match."""
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 256)
    o = pyoracle.Llm(path, 256)
    prompt = [256, 257] + list(b"greedy") + [258, 257]
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    n = 48
    tg = g.generate(prompt, n, 0.0, 1, allow=allow)
    assert len(tg) == n
    # oracle greedy loop with its logits kept, to judge a divergence
    for i, t in enumerate(prompt):
        lo = o.eval(int(t), i)
    for j in range(n):
        sub = lo[allow[0]:allow[1]]
        want = allow[0] + int(sub.argmax())
        if tg[j] != want:
            top2 = np.sort(sub)[-2:]
            gap = float(top2[1] - top2[0])
            assert gap <= 5e-2 * float(np.abs(sub).max()), (j, tg[j], want, gap)
            break
        lo = o.eval(int(tg[j]), len(prompt) + j)
    g.close()


def test_qwen2_bias_logits_and_generate(device, synth_llm_path, tmp_path):
    """qwen2 (RoPE NEOX + attn_{q,k,v}.bias added before RoPE, llama.cpp build_qwen2): the
    biases reach the logits (they differ from the same file read without them by far more
    than the bound) and GPU == oracle within the teacher-forced bound."""
    from miotts_amd import gguf_np
    rel, agree = _teacher_forced(device, synth_llm_path(5), 140, 5)
    assert rel[:2].max() <= 1e-4 and rel.max() <= 5e-2 and agree.sum() >= 133
    nob = str(tmp_path / "nobias.gguf")
    gguf_np.rewrite(synth_llm_path(5), nob, drop_suffix=".bias")
    g, g0 = m.Llm(device, synth_llm_path(5), 64), m.Llm(device, nob, 64)
    a, b = g.eval(300, 0), g0.eval(300, 0)
    assert np.sqrt(np.mean((a - b).astype(np.float64) ** 2)) >= 0.2 * np.sqrt(np.mean(b.astype(np.float64) ** 2))
    g.close(), g0.close()
    tg, to, first = _free_run_agreement(device, synth_llm_path(5), 5, 0.8, 40)
    assert first >= 38


def test_loader_rejects_unknown_biases_and_incomplete_lfm2(device, tmp_path):
    """A bias tensor other than attn_{q,k,v}.bias is refused rather than silently dropped; an
    lfm2 file whose attention layers lack their q norm is refused by the tensor's name."""
    from miotts_amd import gguf_np
    src = m.synth_llm(str(tmp_path / "q2.gguf"), 5, 1)
    dst = str(tmp_path / "patched.gguf")
    gguf_np.rewrite(src, dst, extra_f32="blk.0.ffn_down.bias")
    with pytest.raises(m.HipError, match="bias tensor"):
        m.Llm(device, dst, 128)
    lf = m.synth_llm(str(tmp_path / "lfm2.gguf"), 7, 1)
    gguf_np.rewrite(lf, dst, drop_suffix="attn_q_norm.weight")
    with pytest.raises(m.HipError, match="attn_q_norm"):
        m.Llm(device, dst, 128)


# --- batched prompt prefill (csrc/hip/llm_prefill.hip; reference prefill llama_decode,
# test-to-speech.cpp:132-148). The batched kernels run the decode step's arithmetic token by
# token in the same order, so the last token's logits (and therefore the KV cache rows they
# read) equal a token-by-token decode BIT FOR BIT; vs the oracle the teacher-forced bound
# above applies.
@pytest.mark.parametrize("preset,n", [(0, 2), (0, 17), (1, 40), (0, 150), (9, 70), (11, 30), (11, 150)])
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


@pytest.mark.parametrize("preset", [3, 12])
def test_batched_prefill_1p7b(device, synth_llm_path, preset):
    """1.7B, 68-token prompt (the bench prompt length: one chunk): Q4_K_M (Q4_K + Q6_K on the
    int8 matrix cores) and BF16 (the streaming dot engine with bf16 records)."""
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 256)
    toks = np.random.default_rng(68).integers(0, 151936, 68)
    batched = g.prefill(toks)
    for pos, t in enumerate(toks):
        seq = g.eval(int(t), pos)
    assert np.array_equal(batched, seq), float(np.abs(batched - seq).max())


@pytest.mark.parametrize("qtype,k,rows,nt", [(8, 256, 40, 1), (8, 576, 37, 5), (8, 2048, 64, 33), (8, 10752, 33, 17),
                                           (12, 256, 50, 3), (14, 768, 33, 2),
                                           (12, 2048, 70, 32), (12, 6144, 32, 64), (14, 2048, 45, 9),
                                           (14, 6144, 96, 40),
                                           # <= 16 tokens: the 16 x 16 tiles (k_mmq16)
                                           (8, 2048, 70, 8), (8, 10752, 40, 16), (12, 2048, 70, 8),
                                           (12, 6144, 33, 16), (14, 2048, 45, 8), (14, 6144, 37, 12)])
def test_mmq_equals_single_token_matvec(device, qtype, k, rows, nt):
    """The batched matmul on the int8 matrix cores (llm_mmq.hip: prefill and batched decode)
    returns, for every token, the single-token decode matvec's value BIT FOR BIT (same exact
    integer group sums, same float terms, summed in the decode's lane/tree order)."""
    rng = np.random.default_rng(qtype * 7 + k + nt)
    w = (rng.standard_normal((rows, k)) * 0.05).astype(np.float32)
    wq = m.quantize_rows(qtype, w)
    x = rng.standard_normal((nt, k)).astype(np.float32)
    x[:, 3] = -9.0
    y = m.debug_mmq(device, qtype, wq, k, x)
    refs = [m.debug_matvec(device, qtype, wq, k, x[t]) for t in range(nt)]
    for t in range(nt):
        assert np.array_equal(y[t], refs[t]), (t, float(np.abs(y[t] - refs[t]).max()))
    # residual epilogue (attn_out / ffn_down): v + r
    r0 = rng.standard_normal((nt, rows)).astype(np.float32)
    y = m.debug_mmq(device, qtype, wq, k, x, mode=1, y_in=r0)
    for t in range(nt):
        assert np.array_equal(y[t], refs[t] + r0[t]), t
    # SwiGLU epilogue (gate|up): silu(g) * u, u from a second matrix of the same type
    wu = m.quantize_rows(qtype, (rng.standard_normal((rows, k)) * 0.05).astype(np.float32))
    y = m.debug_mmq(device, qtype, wq, k, x, mode=2, up_rows=wu)
    for t in range(nt):
        # expf differs from numpy's exp by an ulp: the model-level tests pin this epilogue
        # bit-exactly against the decode step (test_batched_prefill_matches_sequential)
        u = m.debug_matvec(device, qtype, wu, k, x[t])
        g = refs[t].astype(np.float64)
        want = g / (1.0 + np.exp(-g)) * u
        err = float(np.abs(y[t] - want).max())
        assert err <= 1e-5 * float(np.abs(want).max()) + 1e-6, (t, err)


_FUSION_SCRIPT = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[2])
import miotts_amd as m
dev = m.Device(0)
g = m.Llm(dev, sys.argv[1], 512)
prompt = np.array([256, 257, 65, 258, 257, 300, 301], np.int32)
toks = g.generate(prompt, 80, 0.8, 5, allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800), check_interval=16)
h = hashlib.sha256(toks.tobytes())
for pos in (3, 70, 129):
    h.update(g.eval(int(toks[0]), pos).tobytes())
k = g.step_kinds()
print(k.count(11), k.count(10), k.count(12), k.count(13), h.hexdigest())
"""


@pytest.mark.parametrize("preset", [2, 3, 4])
def test_fused_attention_launches_bit_identical(synth_llm_path, tmp_path, preset):
    """The whole layer as one launch (k_layer, layers >= 1, r06, opt-in), the attention block as one
    launch (k_layer_att) + the FFN pair as one launch (k_ffn), attention + O as one launch
    (k_att_o) and the separate launches run the same arithmetic: 80 free-run tokens and the
    logits of three later evaluations are bit-identical across MIO_LAYER_FUSE / MIO_LAYER_GATE /
    MIO_LAYER_ATT / MIO_ATT_FUSE_O / MIO_FFN_FUSE (each variant is a fresh process: the switches
    are read once). k_layer is instantiated for the 1.7B Q4_K_M shapes (preset 3)."""
    import os
    import subprocess
    import sys
    path = synth_llm_path(preset)
    script = tmp_path / "fusion.py"
    script.write_text(_FUSION_SCRIPT)
    pkg = os.path.dirname(os.path.dirname(m.__file__))
    outs = {}
    for name, env in (("layer", {"MIO_LAYER_FUSE": "1"}), ("layer_gate", {"MIO_LAYER_FUSE": "1", "MIO_LAYER_GATE": "2"}),
                      ("layer_att", {"MIO_LAYER_FUSE": "0", "MIO_LAYER_ATT": "1"}),
                      ("att_o", {"MIO_LAYER_FUSE": "0", "MIO_LAYER_ATT": "0"}),
                      ("separate", {"MIO_ATT_FUSE_O": "0", "MIO_FFN_FUSE": "0"})):
        p = subprocess.run([sys.executable, str(script), path, pkg], capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, **env))
        assert p.returncode == 0, p.stderr[-2000:]
        outs[name] = p.stdout.split()
    print(outs)
    if preset == 3:
        assert int(outs["layer"][3]) == 27 and int(outs["layer_gate"][3]) == 27  # layers 1..27 as k_layer
    assert int(outs["layer_att"][0]) > 0 and int(outs["layer_att"][3]) == 0
    assert int(outs["att_o"][0]) == 0 and int(outs["att_o"][1]) > 0
    assert int(outs["separate"][0]) == int(outs["separate"][1]) == int(outs["separate"][2]) == 0
    assert int(outs["separate"][3]) == 0
    assert int(outs["layer_att"][2]) > 0  # the FFN pairs ran fused
    digests = {k: v[4] for k, v in outs.items()}
    assert len(set(digests.values())) == 1, digests
