"""CPU: the GGUF byte-level BPE tokenizer (csrc/host/tokenizer.cpp) against HuggingFace
`tokenizers` (0.22, installed here) on a trained vocabulary.

llama.cpp's `llama_tokenize` (test-to-speech.cpp:117-125,173-176) is absent (the un-vendored
submodule), so there is no reference output to pin against. `tokenizers` is the
published byte-level BPE that llama.cpp's `llm_tokenizer_bpe` is validated against (its
test-tokenizer-0 vectors come from it), and the GGUF `tokenizer.ggml.pre` types map onto its
pre-tokenizers: "qwen2" / "llama3" (= "llama-bpe", "lfm2") = Split(their regex, isolated) +
ByteLevel(use_regex=False); "gpt2" = ByteLevel(use_regex=True) (the GPT-2 regex); "default" =
llama.cpp's four regexes in sequence as four Splits; "smollm" = Digits(individual) +
ByteLevel(use_regex=True). Each case trains a BPE vocabulary with
`tokenizers` on a seeded corpus, writes it into a GGUF (tokens in id order, merges in rank
order, specials as CONTROL), and requires identical ids on held-out seeded strings: mixed
Japanese / ASCII / other scripts / digits / punctuation / whitespace runs / contractions /
specials. The \\p{L} / \\p{N} classes come from tools/gen_unicode_ranges.py.
"""
import json
import random

import pytest

import miotts_amd as m
from miotts_amd import gguf_np

tokenizers = pytest.importorskip("tokenizers")

QWEN2 = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*"
         r"|\s*[\r\n]+|\s+(?!\S)|\s+")
# llama.cpp LLAMA_VOCAB_PRE_TYPE_LLAMA3 (also "llama-bpe", "lfm2")
LLAMA3 = (r"(?:'[sS]|'[tT]|'[rR][eE]|'[vV][eE]|'[mM]|'[lL][lL]|'[dD])|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}"
          r"| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2 = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"
# llama.cpp's "default" pre-type: four regexes in sequence
DEFAULT = [r"[\p{P}\$\+<=>\^~\|]+", GPT2, r"\p{N}+", r"[0-9][0-9][0-9]"]
SPECIALS = ["<|im_start|>", "<|im_end|>", "<|startoftext|>", "<|endoftext|>"]

# characters drawn from the classes the pre-tokenizers distinguish
_ALPHA = (
    list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ") * 4
    + list("0123456789") * 2
    + list(" ") * 12 + list("\n\t\r")
    + list(".,;:!?-_()[]\"/#$%&*+=<>@^`{|}~'")
    + list("あいうえおかきくけこさしすせそたちつてとなにぬねのはひふへほまみむめもやゆよらりるれろわをんがぎぐげご")
    + list("アイウエオカキクケコサシスセソタチツテトナニヌネノーッャュョ")
    + list("今日天気東京大学生時間語本人") + list("、。！？「」・…")
    # other scripts and classes: Greek, Cyrillic, Hangul, Arabic, Hebrew, Thai (incl. the
    # letters after U+0E30), Devanagari digits, combining marks (M*, neither L nor N), emoji,
    # zero-width space / NBSP / soft hyphen, numbers of class Nl / No, modifier letters (Lm)
    + list("αβγΔΩабвгдЖЯ한국어가나다ابتثعربيאבגกขคงไทยเแโ") + list("́̈​ ­")
    + list("😀🎉٠١१२ⅧⅫ①〇々ｶﾀﾅｰǅʰªº⁰¹")
    + list("０１２３４５ＡＢＣａｂｃ") + list("éüñßçøÅ²½µ") + ["　", " "]
)
_WORDS = ["hello", "world", "The", "it's", "we'LL", "I'm", "you've", "they're", "don't", "12345", "3.14",
          "こんにちは", "今日はいい天気ですね", "ありがとう", "  ", "\n\n", " \n ", "!!", "...", "??\n"]


def _text(rng, n):
    parts = []
    while sum(map(len, parts)) < n:
        r = rng.random()
        if r < 0.35:
            parts.append(rng.choice(_WORDS))
        elif r < 0.4:
            parts.append(rng.choice(SPECIALS))
        else:
            parts.append("".join(rng.choice(_ALPHA) for _ in range(rng.randint(1, 6))))
    return "".join(parts)


def _trained(pre, vocab_size, seed):
    from tokenizers import Regex, Tokenizer, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    split = lambda rx: pre_tokenizers.Split(Regex(rx), behavior="isolated", invert=False)
    bl = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)
    if pre in ("qwen2", "llama3", "llama-bpe", "lfm2"):
        tok.pre_tokenizer = pre_tokenizers.Sequence([split(QWEN2 if pre == "qwen2" else LLAMA3), bl])
    elif pre == "default":
        tok.pre_tokenizer = pre_tokenizers.Sequence([split(rx) for rx in DEFAULT] + [bl])
    elif pre == "smollm":
        tok.pre_tokenizer = pre_tokenizers.Sequence([
            pre_tokenizers.Digits(individual_digits=True),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)])
    else:  # gpt-2 (llama.cpp's converter name) and its aliases
        tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    rng = random.Random(seed)
    corpus = [_text(rng, 200) for _ in range(600)] + _WORDS * 20
    tr = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=SPECIALS, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus, tr)
    return tok


def _to_gguf(tok, path, pre):
    js = json.loads(tok.to_str())
    vocab = tok.get_vocab(with_added_tokens=True)
    toks = [None] * len(vocab)
    for t, i in vocab.items():
        toks[i] = t
    assert all(t is not None for t in toks)
    merges = [" ".join(p) if isinstance(p, list) else p for p in js["model"]["merges"]]
    types = [3 if t in SPECIALS else 1 for t in toks]
    gguf_np.write_kv_gguf(path, {
        "general.architecture": "qwen3",
        "tokenizer.ggml.model": "gpt2",
        "tokenizer.ggml.pre": pre,
        "tokenizer.ggml.tokens": toks,
        "tokenizer.ggml.token_type": types,
        "tokenizer.ggml.merges": merges,
        "tokenizer.ggml.eos_token_id": vocab["<|endoftext|>"],
        "tokenizer.ggml.bos_token_id": vocab["<|endoftext|>"],
        "tokenizer.ggml.add_bos_token": False,
    })
    return len(merges)


@pytest.mark.parametrize("pre,vocab_size,seed", [("qwen2", 1200, 1), ("qwen2", 3000, 2), ("gpt-2", 1200, 3),
                                                  ("default", 1500, 4), ("llama3", 1500, 5), ("lfm2", 3000, 6),
                                                  ("smollm", 1500, 7), ("gpt2", 1200, 8), ("phi-2", 1200, 9)])
def test_tokenize_matches_hf_tokenizers(tmp_path, pre, vocab_size, seed):
    hf = _trained(pre, vocab_size, seed)
    path = str(tmp_path / f"hf_{pre}_{seed}.gguf")
    n_merges = _to_gguf(hf, path, pre)
    assert n_merges > 500
    t = m.Tokenizer(path)
    rng = random.Random(1000 + seed)
    cases = [_text(rng, rng.randint(1, 120)) for _ in range(400)]
    cases += ["", " ", "\n", "  \n  x", "a  b   c", "x\r\ny", "'s's", "ABC'LL", "１２３", "。\n\n", "　あ",
              "1234567", "12345 678901", "a1b22c333d4444", "３．１４１５９", "v1.2.3-rc4", "$100+<=>^~|", "٠١٢٣٤",
              "今日は2024年10月17日です。", "x ,y", "((a))", "¿Qué? ¡Sí!"]
    bad = []
    for s in cases:
        want = hf.encode(s, add_special_tokens=False).ids
        got = t.tokenize(s, add_special=False)
        if got != want:
            bad.append((s, got, want))
        # byte-exact inverse
        assert t.detokenize(got) == s
    assert not bad, f"{len(bad)}/{len(cases)} differ, first: {bad[0]!r}"


def test_unknown_pre_tokenizer_is_refused(tmp_path):
    """A tokenizer.ggml.pre outside the implemented families fails to load with a message
    instead of silently tokenizing with another family's regex."""
    hf = _trained("gpt2", 600, 11)
    path = str(tmp_path / "unknown_pre.gguf")
    _to_gguf(hf, path, "chatglm-bpe")
    with pytest.raises(Exception, match="pre-tokenizer 'chatglm-bpe' is not implemented"):
        m.Tokenizer(path)
