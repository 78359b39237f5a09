"""GPU parity of the lfm2 short-conv hybrid (llama.cpp build_lfm2: attention layers with NEOX
RoPE and q/k RMSNorm interleaved with gated short-conv layers, build_shortconv_block +
ggml_ssm_conv) against the oracle (oracle/llm_ref.c, whose lfm2 path tests/test_np_crosscheck.py
pins against the independent numpy restatement; upstream llama.cpp itself is not in the
reference tree, so the lfm2 semantics are "parity unpinned" beyond that cross-check).

GPU side (csrc/hip): a short-conv layer is k_attn_in over in_proj (B | C | X rows) and
k_conv_out (bx = B*X, the 3-tap window over a 4-slot ring of earlier positions, y = C*conv,
out_proj); prefill and the batched step run in_proj / out_proj on the int8 matrix cores with
k_bt_conv (window from the chunk's own earlier tokens or the sequence's ring) and
k_bt_conv_state (ring update). Synthetic presets: 7 tiny Q8_0, 8 tiny Q4_K_M (5 layers,
attention at 1 and 4), 6 the LFM2-2.6B shape (30 layers, attention on 8).

Bounds are test_llm_gpu.py's (same re-quantization flip noise); the per-layer comparison is in
test_llm_layers_gpu.py (presets 7, 8, 6).
"""
import numpy as np
import pytest

import miotts_amd as m
import pyoracle

pytestmark = pytest.mark.gpu

ALLOW = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)


@pytest.mark.parametrize("preset", [7, 8])
def test_lfm2_teacher_forced_logits_tiny(device, synth_llm_path, preset):
    """150 positions: through the attention layers' first 128-position chunk boundary and the
    conv rings' slot wrap-around; exact at positions 0-1, flip-bounded after."""
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 256)
    o = pyoracle.Llm(path, 256)
    toks = np.random.default_rng(preset).integers(0, g.n_vocab, 150)
    agree, rels = 0, []
    for pos, t in enumerate(toks):
        lg, lo = g.eval(int(t), pos), o.eval(int(t), pos)
        rel = float(np.abs(lg - lo).max() / np.abs(lo).max())
        rels.append(rel)
        if pos < 2:
            assert rel <= 1e-5, (pos, rel)
        assert rel <= 5e-2, (pos, rel)
        agree += int(lg.argmax() == lo.argmax())
    g.close()
    print(f"preset {preset}: max rel {max(rels):.3g}, median {np.median(rels):.3g}, argmax agree {agree}/150")
    assert agree >= 0.95 * 150


@pytest.mark.parametrize("preset", [7, 8])
def test_lfm2_generate_matches_oracle(device, synth_llm_path, preset):
    """Sampled ids (temperature 0.8, shared counter-based Gumbel-max) and greedy ids follow
    the oracle's decode; run-to-run reproducible."""
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 256)
    o = pyoracle.Llm(path, 256)
    prompt = [256, 257] + list(b"short conv hybrid") + [258, 257]
    tg = g.generate(prompt, 40, 0.8, 42, allow=ALLOW)
    to = o.generate(prompt, 40, 0.8, 42, allow=ALLOW)
    same = tg == to
    assert len(tg) == 40 and same.sum() >= 38, (int(np.argmin(same)), tg.tolist(), to.tolist())
    assert np.array_equal(tg, g.generate(prompt, 40, 0.8, 42, allow=ALLOW))
    gg = g.generate(prompt, 24, 0.0, 1, allow=ALLOW)
    og = o.generate(prompt, 24, 0.0, 1, allow=ALLOW)
    assert (gg == og).sum() >= 22, (gg, og)
    g.close()


@pytest.mark.parametrize("preset,n", [(7, 2), (7, 3), (7, 17), (8, 40), (7, 150), (8, 200)])
def test_lfm2_batched_prefill_matches_sequential(device, synth_llm_path, preset, n):
    """The batched prefill (matrix-core in_proj / out_proj, the conv window from the chunk's
    own rows, ring handed from one 128-token chunk to the next at n = 150 / 200) leaves the
    state a token-by-token decode leaves: the last token's logits are equal BIT FOR BIT."""
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 256)
    toks = np.random.default_rng(100 + n).integers(0, g.n_vocab, n)
    batched = g.prefill(toks)
    seq = None
    for pos, t in enumerate(toks):
        seq = g.eval(int(t), pos)
    assert np.array_equal(batched, seq), float(np.abs(batched - seq).max())
    o = pyoracle.Llm(path, 256)
    for pos, t in enumerate(toks):
        lo = o.eval(int(t), pos)
    assert np.abs(batched - lo).max() <= 5e-2 * np.abs(lo).max()
    g.close()


def _prompts(B, seed, lo=3, hi=40):
    rng = np.random.default_rng(seed)
    lens = [1 if b == 1 else int(rng.integers(lo, hi)) for b in range(B)]
    return [list(rng.integers(0, 256, n)) for n in lens]


@pytest.mark.parametrize("preset,B", [(7, 3), (8, 5), (7, 12)])
def test_lfm2_batch_equals_single_streams(device, synth_llm_path, preset, B):
    """B utterances decoded together (per-stream conv rings) equal their single-stream decodes
    exactly; the flattened prompt prefill splits streams across 128-token chunks at B = 12."""
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 256)
    prompts = _prompts(B, 10 * preset + B, 3, 40 if B < 10 else 60)
    seeds = [1000 + 17 * b for b in range(B)]
    got = g.generate_batch(prompts, 24, 0.8, seeds, allow=ALLOW)
    for b in range(B):
        ref = g.generate(prompts[b], 24, 0.8, seeds[b], allow=ALLOW)
        assert np.array_equal(got[b], ref), (b, got[b], ref)
    g.close()


def test_lfm2_2p6b_shape(device, synth_llm_path):
    """The LFM2-2.6B shape (30 layers, 22 short-conv, Q8_0, GQA 32/8 at head dim 64, 78336
    vocab): teacher-forced logits over 140 positions within the large-model bound of
    test_llm_gpu.py, and 4 utterances decoded together equal their single-stream decodes."""
    path = synth_llm_path(6)
    g = m.Llm(device, path, 512)
    o = pyoracle.Llm(path, 512)
    kinds = g.step_kinds()
    # attention layers: attn_in (+ attention + attn_out, or the fused k_att_o), or the whole block
    # as one launch (11) on layers >= 1
    assert kinds.count(8) == 22 and kinds.count(9) == 22 and kinds.count(0) + kinds.count(11) == 8
    toks = np.random.default_rng(26).integers(0, g.n_vocab, 140)
    rel, top5 = [], []
    for pos, t in enumerate(toks):
        lg, lo = g.eval(int(t), pos), o.eval(int(t), pos)
        d = lg.astype(np.float64) - lo
        rel.append(np.sqrt(np.mean(d * d)) / np.sqrt(np.mean(lo.astype(np.float64) ** 2)))
        top5.append(lo.argmax() in np.argpartition(lg, -5)[-5:])
    rel = np.array(rel)
    print(f"lfm2 2.6B: rel RMS max {rel.max():.3g} (pos {int(rel.argmax())}), median {np.median(rel):.3g}, "
          f"oracle argmax in GPU top-5 {sum(top5)}/140")
    assert rel.max() <= 0.1 and sum(top5) >= 0.9 * 140
    prompts = _prompts(4, 266)
    seeds = [77 + b for b in range(4)]
    got = g.generate_batch(prompts, 32, 0.8, seeds, allow=ALLOW)
    for b in range(4):
        assert np.array_equal(got[b], g.generate(prompts[b], 32, 0.8, seeds[b], allow=ALLOW)), b
    g.close()


def test_lfm2_kernel_timing_and_ring_api(device, synth_llm_path):
    """time_kernel reaches the short-conv launches (8 conv_in, 9 conv_out) with their
    algorithmic bytes; the conv ring getter refuses an attention layer."""
    g = m.Llm(device, synth_llm_path(7), 128)
    g.eval(300, 0)
    for which in (8, 9, 0, 1, 2, 3, 4, 6):
        ms, by = g.time_kernel(which, 3)
        assert ms > 0 and by > 0, which
    with pytest.raises(m.HipError):
        g.conv_ring(1)  # layer 1 is an attention layer in preset 7
    assert g.conv_ring(0).shape == (4, g.n_embd)
    g.close()
