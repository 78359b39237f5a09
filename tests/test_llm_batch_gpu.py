"""GPU parity: batched decode of B utterances (mio_hip_llm_generate_batch, csrc/hip/llm_prefill.hip
k_bt_* + the multi-token layer engine) vs single-utterance decode (mio_hip_llm_generate).

The reference decodes utterances one after another, one llama_context each
(test-to-speech.cpp:94-199 per call). Batching B of them into one weight pass per step must not
change any of them: every stream's per-token arithmetic is the single-stream decode's (same
quantizers, same per-superblock integer sums in the same order, same attention sweep, same
counter-based Gumbel noise gumbel(seed_b, step, id)), so stream b's tokens equal
generate(prompt_b, seed_b) EXACTLY. Single-stream generate is itself checked against the C
oracle in test_llm_gpu.py (>= 95% of ids, measured 100%); the first test re-checks one stream
against the oracle directly.
"""
import numpy as np
import pytest

import miotts_amd as m
import pyoracle

pytestmark = pytest.mark.gpu

ALLOW = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)


@pytest.fixture(scope="module")
def llm_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("llm_batch")
    return {p: m.synth_llm(str(d / f"llm{p}.gguf"), p, 1) for p in (0, 1)}


def _prompts(B, seed):
    rng = np.random.default_rng(seed)
    # ragged lengths, including a 1-token prompt (nothing to prefill for that stream)
    lens = [1 if b == 1 else int(rng.integers(3, 40)) for b in range(B)]
    return [list(rng.integers(0, 256, n)) for n in lens]


@pytest.mark.parametrize("preset,B", [(0, 3), (1, 4), (0, 16)])
def test_batch_equals_single_streams(device, llm_files, preset, B):
    g = m.Llm(device, llm_files[preset], 256)
    prompts = _prompts(B, 10 * preset + B)
    seeds = [1000 + 17 * b for b in range(B)]
    got = g.generate_batch(prompts, 24, 0.8, seeds, allow=ALLOW)
    for b in range(B):
        ref = g.generate(prompts[b], 24, 0.8, seeds[b], allow=ALLOW)
        assert np.array_equal(got[b], ref), (b, got[b], ref)
    if B == 3:
        o = pyoracle.Llm(llm_files[preset], 256)
        to = o.generate(prompts[0], 24, 0.8, seeds[0], allow=ALLOW)
        assert (got[0] == to).sum() >= 22


def test_batch_greedy_and_identical_streams(device, llm_files):
    """temperature 0 = greedy; two streams with the same prompt and seed stay identical."""
    g = m.Llm(device, llm_files[1], 256)
    p = [256, 257, 84, 101, 115, 116, 258, 257]
    got = g.generate_batch([p, p, p[:5]], 16, 0.0, [5, 5, 9], allow=ALLOW)
    assert np.array_equal(got[0], got[1])
    assert np.array_equal(got[0], g.generate(p, 16, 0.0, 123, allow=ALLOW))
    assert np.array_equal(got[2], g.generate(p[:5], 16, 0.0, 9, allow=ALLOW))


def test_batch_stops_at_eos(device, llm_files):
    """End tokens end each stream where its single-stream decode ends (the token itself is not
    returned, test-to-speech.cpp:168-170); the batch returns when every stream has ended."""
    g = m.Llm(device, llm_files[0], 256)
    prompts = [[256, 257, 65, 258, 257], [256, 257, 66, 67, 258, 257], [256, 257, 68, 258, 257]]
    allow = (m.SYNTH_EOT, m.SYNTH_SPEECH0 + 3)
    eos = (m.SYNTH_EOT, m.SYNTH_IM_END)
    got = g.generate_batch(prompts, 200, 2.0, [7, 8, 9], allow=allow, eos=eos, check_interval=20)
    for b, p in enumerate(prompts):
        ref = g.generate(p, 200, 2.0, 7 + b, allow=allow, eos=eos, check_interval=20)
        assert np.array_equal(got[b], ref)
        assert len(got[b]) < 200 and (got[b] != m.SYNTH_EOT).all()


@pytest.mark.parametrize("preset,B,n", [(11, 3, 24), (12, 4, 16)])
def test_batch_bf16_equals_single(device, synth_llm_path, preset, B, n):
    """BF16 weights (README.md:196 ships every size in BF16) on the multi-token engine: the
    streaming dot engine with bf16 act records (v_dot2 over the bf16-rounded activation in the
    decode's lane order and row-total tree), so every stream equals its single-stream decode
    bit for bit; 11 = tiny, 12 = the 1.7B shape."""
    g = m.Llm(device, synth_llm_path(preset), 256)
    prompts = _prompts(B, 90 + preset)
    seeds = [77 + 5 * b for b in range(B)]
    got = g.generate_batch(prompts, n, 0.8, seeds, allow=ALLOW)
    for b in range(B):
        ref = g.generate(prompts[b], n, 0.8, seeds[b], allow=ALLOW)
        assert np.array_equal(got[b], ref), (b, got[b], ref)
    g.close()


def test_batch_rejects_bad_shapes(device, llm_files):
    g = m.Llm(device, llm_files[0], 64)
    with pytest.raises(m.HipError):
        g.generate_batch([[256, 257]] * 17, 4, 0.8)
    with pytest.raises(m.HipError):
        g.generate_batch([[256] * 65], 4, 0.8)  # prompt longer than n_ctx 64


def test_context_full_ends_generation(device, llm_files):
    """40 prompt + 30 new > n_ctx 64: like the reference (test-to-speech.cpp:163-187, decode
    fails at a full context and the last sampled token is kept), generation stops after
    n_ctx - 40 + 1 = 25 tokens instead of failing; single and batched streams agree."""
    g = m.Llm(device, llm_files[0], 64)
    p = [256] + [65 + i % 20 for i in range(39)]
    single = g.generate(p, 30, 0.8, 5, allow=ALLOW)
    assert len(single) == 25
    both = g.generate_batch([p, p[:10]], 30, 0.8, [5, 6], allow=ALLOW)
    assert np.array_equal(both[0], single) and len(both[1]) == 30


def test_batch_1p7b_q4km(device, tmp_path):
    """The bench model (1.7B Q4_K_M: Q4_K + Q6_K matrices, 28 layers, GQA 16/8, 164736 vocab),
    4 streams x 16 tokens, each equal to its single-stream decode."""
    path = m.synth_llm(str(tmp_path / "llm17.gguf"), 3, 1)
    g = m.Llm(device, path, 512)
    prompts = _prompts(4, 17)
    got = g.generate_batch(prompts, 16, 0.8, [42, 43, 44, 45], allow=ALLOW)
    for b in range(4):
        assert np.array_equal(got[b], g.generate(prompts[b], 16, 0.8, 42 + b, allow=ALLOW)), b


def test_batch_c4_2p6b_q8_b8(device, synth_llm_path):
    """BASELINE config C4's per-GPU workload: the 2.6B Q8_0 model (32 layers, GQA 32/8 at head
    dim 64, n_ff 10752, 78336 vocab), 8 utterances decoded together, 48 tokens each: every
    stream equals its single-stream decode bit for bit (the single-stream decode of this model
    against the oracle: test_llm_gpu.py::test_free_run_64_tokens_large_models[4])."""
    path = synth_llm_path(4)
    g = m.Llm(device, path, 512)
    prompts = _prompts(8, 44)
    seeds = [4200 + 3 * b for b in range(8)]
    got = g.generate_batch(prompts, 48, 0.8, seeds, allow=ALLOW)
    for b in range(8):
        ref = g.generate(prompts[b], 48, 0.8, seeds[b], allow=ALLOW)
        assert np.array_equal(got[b], ref), b
    g.close()


CLI_PROMPTS = ["テストです。", "こんにちは。", "今日はいい天気ですね。"]


def test_batch_cli_prompt_set_repeated(device, llm_files):
    """Regression for round 5's intermittent `miotts --batch` mismatch (the third, longest
    prompt's WAV differed from its single run in 1 of 3 CLI runs; the batched step's in-launch
    quantization consumers read their producers' act records with plain loads). The exact CLI
    workload through the C-ABI: the three prompts in the chat template, tokenized as
    TestToSpeech::prompt_tokens does (tts.cpp:258-266), preset 1, n_ctx 2048, 40 speech-only
    tokens at the config temperature 0.8 with the single run's seed 42 for every stream, polls
    every 32 steps. Repeated 12 times (the first run of a fresh batch width captures its graphs,
    the later ones replay them): every stream equals its single-stream decode every time."""
    path = llm_files[1]
    tok = m.Tokenizer(path)
    prompts = [tok.tokenize("<|startoftext|><|im_start|>user\n" + m.normalize_text(p) +
                            "<|im_end|>\n<|im_start|>assistant\n", True, True) for p in CLI_PROMPTS]
    assert len(prompts[2]) > len(prompts[0]) > 8
    g = m.Llm(device, path, 2048)
    refs = [g.generate(p, 40, 0.8, 42, allow=ALLOW, check_interval=32) for p in prompts]
    assert all(len(r) == 40 for r in refs)
    bad = []
    for rep in range(12):
        got = g.generate_batch(prompts, 40, 0.8, [42, 42, 42], allow=ALLOW, check_interval=32)
        bad += [(rep, b, int(np.argmax(got[b] != refs[b]))) for b in range(3) if not np.array_equal(got[b], refs[b])]
    assert not bad, f"(repeat, stream, first differing token): {bad}"
    g.close()


_ENGINE_SCRIPT = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[2])
import miotts_amd as m
dev = m.Device(0)
g = m.Llm(dev, sys.argv[1], 512)
rng = np.random.default_rng(7)
prompts = [list(rng.integers(0, 256, int(n))) for n in (5, 1, 17, 9, 30, 3, 12, 8)]
got = g.generate_batch(prompts, 24, 0.8, [900 + b for b in range(8)],
                       allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800))
h = hashlib.sha256()
for t in got:
    h.update(np.asarray(t, np.int32).tobytes())
print(h.hexdigest())
"""


@pytest.mark.parametrize("preset,variants", [
    (3, [{"MIO_BT_LM_MMQ": "0"}, {"MIO_MMQ_LOOP_KQ": "0"}, {"MIO_KQ_EARLY": "0"}, {"MIO_BT_QCHUNK": "0"},
         {"MIO_BT_IQ": "1"}]),
    (4, [{"MIO_BT_DQ": "0"}, {"MIO_BT_FQ": "1"}, {"MIO_BT_LM_MMQ": "0"}, {"MIO_MMQ_LOOP": "0"}]),
])
def test_batch_engine_switches_bit_identical(synth_llm_path, tmp_path, preset, variants):
    """The round-5 batched-step engines run the arithmetic of the ones they replace: 8 streams x
    24 tokens are identical with each switched back (a fresh process per variant; the switches
    are read once). 1.7B Q4_K_M: the lm_head on the matrix cores vs k_bt_lm_head's dot4, the
    K-quant tile loops vs one workgroup per tile, weight loads before vs after the in-launch
    producers' wait, chunked vs per-token producers, the gate|up walk quantizing its tokens in
    its own prologue (r06, opt-in MIO_BT_IQ=1) vs producer workgroups. 2.6B Q8_0: the dot4 down quantizing h in
    its launch vs behind k_bt_quant_split, q|k|v on the matrix cores vs the dot4 in-launch path,
    the lm_head engines, the Q8_0 tile loops."""
    import os
    import subprocess
    import sys
    path = synth_llm_path(preset)
    script = tmp_path / "engines.py"
    script.write_text(_ENGINE_SCRIPT)
    pkg = os.path.dirname(os.path.dirname(m.__file__))
    outs = []
    for env in [{}] + variants:
        p = subprocess.run([sys.executable, str(script), path, pkg], capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, **env))
        assert p.returncode == 0, (env, p.stderr[-2000:])
        outs.append((env, p.stdout.strip()))
    print(outs)
    assert all(o == outs[0][1] for _, o in outs), outs
