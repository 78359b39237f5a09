"""GPU: the persistent decode launch (csrc/hip/llm_persist.hip) against the per-step hipGraph
path (csrc/hip/llm_kernels.hip), which the other LLM tests pin to the oracle.

Both engines run the same arithmetic in the same order (same quantizers, integer block dots,
attention chunk decomposition and merge order); only where values travel differs (in-launch
write-through hand-offs instead of kernel boundaries). So sampled ids AND the last step's
logits must be equal BIT FOR BIT over long generations: any stale read in a hand-off (an L1
or L2 line from before the producer's store) would show up as a difference. Cases cover the
two weight families, chunk boundaries of the attention (positions past 128 and 256), launches
of 1 / 7 / 64 steps (check_interval), and the 1.7B Q4_K_M preset (Q4_K + Q6_K layers).
"""
import numpy as np
import pytest

import miotts_amd as m

pytestmark = pytest.mark.gpu

ALLOW = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)


@pytest.fixture(scope="module")
def tiny_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("llm_persist")
    return {p: m.synth_llm(str(d / f"llm{p}.gguf"), p, 1) for p in (0, 1)}


def _run(g, persistent, prompt, n, interval, temp=0.8, seed=42):
    g.set_decode_mode(persistent)
    toks = g.generate(prompt, n, temp, seed, allow=ALLOW, check_interval=interval)
    return toks, g.logits()


@pytest.mark.parametrize("preset", [0, 1])
@pytest.mark.parametrize("interval", [1, 7, 64])
def test_persistent_matches_graph_tiny(device, tiny_files, preset, interval):
    g = m.Llm(device, tiny_files[preset], 512)
    prompt = [256, 257, 84, 101, 115, 116, 258, 257]
    tp, lp = _run(g, True, prompt, 70, interval)
    assert g.persistent_active() == 1, "persistent launch did not run"
    tg, lg = _run(g, False, prompt, 70, interval)
    assert len(tp) == 70 and np.array_equal(tp, tg), (tp, tg)
    assert np.array_equal(lp, lg), float(np.abs(lp - lg).max())


@pytest.mark.parametrize("preset", [0, 1])
def test_persistent_long_generation(device, tiny_files, preset):
    """300 generated tokens: the attention crosses the 128- and 256-position chunk
    boundaries inside one launch (a chunk's K/V rows appended and re-read by its workgroup)."""
    g = m.Llm(device, tiny_files[preset], 512)
    prompt = [256, 257] + list(b"long generation") + [258, 257]
    tp, lp = _run(g, True, prompt, 300, 300)
    tg, lg = _run(g, False, prompt, 300, 300)
    assert np.array_equal(tp, tg)
    assert np.array_equal(lp, lg), float(np.abs(lp - lg).max())


def test_persistent_greedy_and_eos(device, tiny_files):
    g = m.Llm(device, tiny_files[0], 256)
    prompt = [256, 257, 65, 258, 257]
    g.set_decode_mode(True)
    a = g.generate(prompt, 40, 0.0, 1, allow=ALLOW, check_interval=40)
    g.set_decode_mode(False)
    b = g.generate(prompt, 40, 0.0, 1, allow=ALLOW, check_interval=40)
    assert np.array_equal(a, b)
    # end token inside a launch: the run stops before it (test-to-speech.cpp:168-170)
    for mode in (True, False):
        g.set_decode_mode(mode)
        toks = g.generate(prompt, 200, 2.0, 7, allow=(m.SYNTH_EOT, m.SYNTH_SPEECH0 + 3),
                          eos=(m.SYNTH_EOT, m.SYNTH_IM_END), check_interval=50)
        assert len(toks) < 200 and (toks != m.SYNTH_EOT).all()
        if mode:
            first = toks
    assert np.array_equal(first, toks)


def test_persistent_matches_graph_1p7b(device, tmp_path):
    path = m.synth_llm(str(tmp_path / "llm17.gguf"), 3, 1)
    g = m.Llm(device, path, 512)
    prompt = [256, 257] + list(b"persistent 1.7B") + [258, 257]
    tp, lp = _run(g, True, prompt, 40, 16)
    assert g.persistent_active() == 1
    tg, lg = _run(g, False, prompt, 40, 16)
    assert np.array_equal(tp, tg)
    assert np.array_equal(lp, lg), float(np.abs(lp - lg).max())
