"""CPU: GGUF byte-level BPE tokenizer (csrc/host/tokenizer.cpp) behind TestToSpeech::run_llm.

The llama.cpp tokenizer is absent here, so parity is unpinned; what is checked:
the chat-template prompt of test-to-speech.cpp:90-92 tokenizes on the synthetic vocabulary
exactly as bench.py's reference construction (specials split out, bytes -> byte tokens),
the piece() inverse round-trips text, <|s_N|> pieces feed parse_speech_tokens, merges are
applied in rank order, and the qwen2 / gpt2 pre-tokenizer splits follow their regexes.
"""
import os

import numpy as np
import pytest

import miotts_amd as m
from miotts_amd import gguf_np


@pytest.fixture(scope="module")
def synth_vocab(tmp_path_factory):
    d = tmp_path_factory.mktemp("tok")
    return m.synth_llm(str(d / "llm0.gguf"), 0, 1)


def _byte_tokens(s):
    return list(s.encode("utf-8"))


def test_prompt_template_tokens(synth_vocab):
    t = m.Tokenizer(synth_vocab)
    assert t.eos == m.SYNTH_EOT and t.im_end == m.SYNTH_IM_END
    text = m.normalize_text("こんにちは、今日はいい天気ですね。")
    prompt = "<|startoftext|><|im_start|>user\n" + text + "<|im_end|>\n<|im_start|>assistant\n"
    want = [256, 257] + _byte_tokens("user\n" + text) + [258] + _byte_tokens("\n") + [257] + _byte_tokens("assistant\n")
    assert t.tokenize(prompt) == want
    # parse_special=False keeps the special text as bytes
    assert t.tokenize("<|im_end|>", parse_special=False) == _byte_tokens("<|im_end|>")


def test_roundtrip_and_speech_pieces(synth_vocab):
    t = m.Tokenizer(synth_vocab)
    for s in ["hello world", "  two  spaces\n\nnewlines", "日本語のテキスト、です！", "mixed123 ,.;"]:
        assert t.detokenize(t.tokenize(s)) == s
    ids = [m.SYNTH_SPEECH0 + 12, m.SYNTH_SPEECH0 + 7, m.SYNTH_SPEECH0 + 12799]
    text = t.detokenize(ids)
    assert text == "<|s_12|><|s_7|><|s_12799|>"
    assert t.tokenize(text, add_special=False) == ids
    assert m.parse_speech_tokens(text).tolist() == [12, 7, 12799]


def _bpe_vocab(path, pre):
    # GPT-2 byte->unicode stand-ins: printable ASCII maps to itself, space -> 'Ġ' (U+0120)
    byte_tok = []
    n = 0
    for b in range(256):
        keep = 33 <= b <= 126 or 161 <= b <= 172 or 174 <= b <= 255
        byte_tok.append(chr(b) if keep else chr(256 + n))
        if not keep:
            n += 1
    # "o Ġ" (rank 0) and "1 2" only apply if the pre-tokenizer leaves those bytes in one piece
    merges = ["o Ġ", "1 2", "h e", "l l", "he ll", "hell o", "Ġ w", "Ġw o", "o r", "Ġwo r", "Ġwor l", "Ġworl d"]
    toks = byte_tok + ["oĠ", "12", "he", "ll", "hell", "hello", "Ġw", "Ġwo", "or", "Ġwor", "Ġworl", "Ġworld",
                       "<|im_end|>", "<|endoftext|>"]
    types = [1] * (len(toks) - 2) + [3, 3]
    gguf_np.write_kv_gguf(path, {
        "general.architecture": "qwen3",
        "tokenizer.ggml.model": "gpt2",
        "tokenizer.ggml.pre": pre,
        "tokenizer.ggml.tokens": toks,
        "tokenizer.ggml.token_type": types,
        "tokenizer.ggml.merges": merges,
        "tokenizer.ggml.eos_token_id": len(toks) - 1,
        "tokenizer.ggml.bos_token_id": len(toks) - 1,
        "tokenizer.ggml.add_bos_token": False,
    })
    return toks


@pytest.mark.parametrize("pre", ["qwen2", "default"])
def test_bpe_merges_in_rank_order(tmp_path, pre):
    path = str(tmp_path / f"bpe_{pre}.gguf")
    toks = _bpe_vocab(path, pre)
    t = m.Tokenizer(path)
    ids = t.tokenize("hello world<|im_end|>")
    assert [toks[i] for i in ids] == ["hello", "Ġworld", "<|im_end|>"]
    assert t.im_end == len(toks) - 2 and t.eos == len(toks) - 1
    assert t.detokenize(ids) == "hello world<|im_end|>"
    # partial merges: "hellx" -> hell + x
    assert [toks[i] for i in t.tokenize("hellx")] == ["hell", "x"]


@pytest.mark.parametrize("pre", ["qwen2", "default"])
def test_pretokenizer_splits(tmp_path, pre):
    path = str(tmp_path / f"bpe_{pre}.gguf")
    toks = _bpe_vocab(path, pre)
    t = m.Tokenizer(path)
    # the space starts a new piece in both regexes: the rank-0 merge "o Ġ" never fires
    assert [toks[i] for i in t.tokenize("hello world")] == ["hello", "Ġworld"]
    # digits: qwen2 splits them one per piece (\p{N}), gpt2 keeps a run ( ?\p{N}+)
    got = [toks[i] for i in t.tokenize("12")]
    assert got == (["1", "2"] if pre == "qwen2" else ["12"])
    # punctuation + letters is one qwen2 piece ([^\r\n\p{L}\p{N}]?\p{L}+), two gpt2 pieces
    assert t.detokenize(t.tokenize(",hello")) == ",hello"
    # whitespace runs: '\s+(?!\S)' leaves the last space to the following word
    assert [toks[i] for i in t.tokenize("  world")] == ["Ġ", "Ġworld"]


@pytest.mark.parametrize("n,calls,codes", [(700, 18, 7160), (100, 3, 260), (300, 8, 1560), (0, 0, 0), (10, 1, 10)])
def test_streaming_cadence_kat(n, calls, codes):
    """SURVEY 8c KAT 4: the stream commit policy (holdback 32, min step 24, check every 20)."""
    assert m.stream_cadence(n) == (calls, codes)
