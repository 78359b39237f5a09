"""CPU: the C oracle (oracle/llm_ref.c) against an independent numpy restatement of the
decode step (tests/np_ref.py), layer by layer.

Both restate llama.cpp's graph in ggml CPU semantics (parity unpinned: ggml is absent). They
share no code, so agreement pins the op semantics the C oracle and the HIP kernels are
checked against: block dequantization, activation re-quantization, RMSNorm, q/k norm, RoPE
pairing (NORM / NEOX) and cache, qwen2 biases, GQA head mapping, softmax, SwiGLU, lm_head,
and lfm2's gated short-conv layers (presets 7 / 8: its ring of earlier bx rows handed over
like the K/V rows).

Layer by layer, teacher-forced: at every checked position the numpy layer gets the oracle's
layer input and the oracle's F16 K/V rows of the earlier positions, so a rounding flip in
one restatement (a Q8 activation code or an f16 cache value on the other side of a rounding
boundary, which then persists in the cache) cannot accumulate. The two differ only in float
summation order, so a layer output agrees to ~1e-7 relative RMS (bound: 2e-5), except where
a last-ulp difference crosses a rounding boundary: an f16 rounding of q, or the signed
largest |x| of a Q8_K block, whose change re-rounds all 256 codes of the block (measured:
q off by 1 f32 ulp -> one head's attention 5e-5 -> layer output 1e-2, preset 1, position 16).
Such a flip is ggml's own arithmetic, not a semantic difference: at most 2 of the layer
evaluations may exceed 2e-5, none 3e-2 (a semantic error, e.g. the NEOX / NORM RoPE pairing
swapped, is off on every layer output from position 1 on: last test).
"""
import numpy as np
import pytest

import miotts_amd as m
import np_ref
import pyoracle


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


@pytest.fixture(scope="module")
def llms(tmp_path_factory):
    d = tmp_path_factory.mktemp("npllm")
    return {p: m.synth_llm(str(d / f"llm{p}.gguf"), p, 1) for p in (0, 1, 5, 7, 8, 9, 10, 11)}


def _sweep(o, n, toks):
    """Layer-by-layer comparison over toks: (number of layer outputs off by > 2e-5, worst)."""
    worst, flips = 0.0, 0
    for pos, t in enumerate(toks):
        x = o.embed(t)
        assert np.array_equal(x, n.embed(t).astype(np.float32))
        for il in range(o.n_layer):
            if o.is_conv(il):  # lfm2 short conv: the oracle's earlier bx rows
                ring = o.conv_ring(il)
                for p in (pos - 1, pos - 2):
                    if p >= 0:
                        n.bx[il, p] = ring[p & 3]
            else:
                k, v = o.kv(il, pos)
                n.kc[il, :, :pos], n.vc[il, :, :pos] = k, v
            y_o = o.layer(il, pos, x)
            e = _rel(n.layer(il, x, pos), y_o)
            worst = max(worst, e)
            flips += e > 2e-5
            x = y_o
        if pos % 8 == 7:
            lo, ln = o.head(x), n.out @ np_ref.rms_norm(x, n.out_norm, n.eps)
            assert _rel(ln, lo) < 2e-5, (pos, _rel(ln, lo))
    return flips, worst


@pytest.mark.parametrize("preset", [0, 1, 5, 7, 8, 9, 10, 11])
def test_layers_match_numpy_restatement(llms, preset):
    path = llms[preset]
    n_pos = 40
    o = pyoracle.Llm(path, n_pos)
    n = np_ref.DecodeStep(path, n_pos)
    rng = np.random.default_rng(preset)
    toks = [256, 257] + [int(t) for t in rng.integers(260, 13060, n_pos - 2)]
    flips, worst = _sweep(o, n, toks)
    # rare rounding-boundary flips are the only admissible outliers (module docstring)
    assert flips <= 2 and worst < 3e-2, (flips, worst)


def test_numpy_restatement_detects_a_rope_pairing_error(llms):
    """The criterion has teeth: the llama (NORM, adjacent-pair) model evaluated with NEOX
    pairs is off on every layer output from position 1 on."""
    path = llms[0]
    o = pyoracle.Llm(path, 8)
    n = np_ref.DecodeStep(path, 8)
    n.neox = True
    flips, worst = _sweep(o, n, [256, 257, 300, 301, 302, 303, 304, 305])
    assert flips >= 7 * o.n_layer and worst > 1e-2, (flips, worst)
