"""GPU parity, layer by layer: every decoder layer of the HIP decode step against the oracle
layer (oracle/llm_ref.c mo_llm_layer) on the GPU's own layer input and K/V rows.

The end-to-end teacher-forced test (test_llm_gpu.py) has to accept 10% RMS on the logits of
the 24-32-layer models: re-quantization flips (ggml's own arithmetic: the Q8 activation
codes and f16 roundings of the reference's CPU path) accumulate through the layers and the
K/V cache. Here nothing accumulates. The decode runs teacher-forced on the GPU up to each
checked position P (positions 0..699, across the 128-position attention chunks), then one
step records the residual before layer 0 and after every layer (mio_hip_llm_eval_layers);
for each layer the oracle gets the GPU's layer input and the GPU's F16 K/V rows of positions
< P, runs that one layer (writing its own row P) and the outputs are compared. The GPU and
the oracle differ only in float summation order (matvec partial sums per superblock,
chunked online softmax, RMSNorm reductions), so a layer output agrees to ~1e-6 relative RMS
unless a last-ulp difference crosses a rounding boundary (an f16 q value, the signed max of
a Q8_K block: the whole block re-rounds), which moves that one layer by up to ~1e-2
(tests/test_np_crosscheck.py shows the same between the two CPU restatements; measured on
the 1.7B model: median 9e-8, 6% of the evaluations above 1e-4, max 1.2e-2). Flips fall on
random (position, layer) pairs; a structural error in a few heads or one layer (RoPE pairing,
q/k norm, GQA mapping, a chunk merge at a boundary position) shows at EVERY position of that
layer, or at every layer of that position. Bounds (written below): the median over the
checked positions of every layer, and over the layers of every position, <= 1e-5; at most
12% of all evaluations above 1e-4 and none above 5e-2; the K/V row the GPU appended at P
within one f16 ulp of the oracle's but in at most 12% of the evaluations; the logits of the
GPU's final residual through the oracle's head within 1e-4 (median) / 5e-2 (max).

lfm2 (presets 7, 8 tiny Q8_0 / Q4_K_M, 6 the LFM2-2.6B shape): a short-conv layer gets the
GPU's conv state instead of K/V rows (mio_hip_llm_conv_ring: the B*X rows of positions P-1,
P-2 its window reads), and the B*X row the GPU stored for P is compared with the oracle's like
an appended K/V row (relative RMS above 1e-5 counts as off).
"""
import numpy as np
import pytest

import miotts_amd as m
import pyoracle

pytestmark = pytest.mark.gpu

POSITIONS = (0, 5, 127, 128, 129, 255, 256, 257, 511, 512, 699)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


@pytest.mark.parametrize("preset", [3, 4, 2, 7, 8, 6, 9, 11, 12])
def test_layers_match_oracle_on_gpu_inputs(device, synth_llm_path, preset):
    path = synth_llm_path(preset)
    g = m.Llm(device, path, 2048)
    o = pyoracle.Llm(path, POSITIONS[-1] + 8)
    rng = np.random.default_rng(700 + preset)
    toks = [256, 257] + [int(t) for t in rng.integers(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800, POSITIONS[-1])]
    errs, kv_bad, head_errs = [], [], []
    for pos in range(POSITIONS[-1] + 1):
        if pos not in POSITIONS:
            g.eval(toks[pos], pos)
            continue
        xs, lg = g.eval_layers(toks[pos], pos)
        assert np.array_equal(xs[0], o.embed(toks[pos]))  # the same dequantized embedding row
        for il in range(g.n_layer):
            if o.is_conv(il):
                # the GPU's state after the step: slots of P-1, P-2 as the step read them, slot P
                # its own B*X row (the oracle overwrites that one with its own)
                ring = g.conv_ring(il)
                o.set_conv_ring(il, ring)
                y = o.layer(il, pos, xs[il])
                errs.append((_rel(xs[il + 1], y), pos, il))
                kv_bad.append(int(_rel(ring[pos & 3], o.conv_ring(il)[pos & 3]) > 1e-5))
                continue
            if pos:
                k, v = g.kv_rows(il, pos)
                o.set_kv(il, k, v)
            y = o.layer(il, pos, xs[il])
            errs.append((_rel(xs[il + 1], y), pos, il))
            # the row the GPU appended at pos vs the oracle's (same input): f16 values
            kg, vg = g.kv_rows(il, pos + 1)
            ko, vo = o.kv(il, pos + 1)
            off = 0
            for a, b in ((kg[:, pos], ko[:, pos]), (vg[:, pos], vo[:, pos])):
                ulp = np.abs(np.spacing(b)).astype(np.float64)
                off += int((np.abs(a.astype(np.float64) - b.astype(np.float64)) > ulp + 1e-12).sum())
            kv_bad.append(off)
        head_errs.append(_rel(lg, o.head(xs[-1])))
    g.close()
    e = np.array([x[0] for x in errs])
    worst = max(errs)
    print(f"preset {preset}: {len(e)} layer evaluations, median {np.median(e):.3g}, "
          f"p95 {np.quantile(e, 0.95):.3g}, max {worst[0]:.3g} (pos {worst[1]}, layer {worst[2]}), "
          f"> 1e-4: {(e > 1e-4).sum()}, K/V rows off by > 1 ulp: {sum(1 for b in kv_bad if b)}, "
          f"logits max {max(head_errs):.3g}")
    by_layer = {}
    by_pos = {}
    for v, pos, il in errs:
        by_layer.setdefault(il, []).append(v)
        by_pos.setdefault(pos, []).append(v)
    worst_layer = max((np.median(v), il) for il, v in by_layer.items())
    worst_pos = max((np.median(v), pos) for pos, v in by_pos.items())
    print(f"  worst per-layer median {worst_layer[0]:.3g} (layer {worst_layer[1]}), worst per-position median "
          f"{worst_pos[0]:.3g} (pos {worst_pos[1]})")
    # BF16 weights (11, 12) round every matvec input to bf16 (8-bit mantissa): an f32-ulp
    # difference of the GPU's summation order crosses a bf16 rounding midpoint far more often
    # than it flips an int8 code, and each such flip moves the layer output by ~1e-4, so the
    # flip evaluations are denser (1.7B BF16 measured: median 9.7e-8, 11.7% above 1e-4, worst
    # per-layer median 1.5e-5, max 1.8e-3). A structural error still shows at >= 1e-2 in every
    # evaluation of its layer or position, far above either bound.
    bf16 = preset in (11, 12)
    med_bound, frac_bound = (1e-4, 0.2) if bf16 else (1e-5, 0.12)
    assert worst_layer[0] <= med_bound and worst_pos[0] <= med_bound, (worst_layer, worst_pos)
    assert (e > 1e-4).sum() <= frac_bound * len(e)
    assert worst[0] <= 5e-2, worst
    # the appended K/V row: within one f16 ulp everywhere but in the flip evaluations
    assert sum(1 for b in kv_bad if b) <= frac_bound * len(kv_bad), kv_bad
    assert np.median(head_errs) <= 1e-4 and max(head_errs) <= 5e-2
