"""CPU: the GGUF WPM tokenizer (tokenizer.ggml.model "bert"; csrc/host/tokenizer.cpp, llama.cpp's
llm_tokenizer_wpm restated) against HuggingFace `tokenizers`' BERT WordPiece on trained
vocabularies.

llama_tokenize (test-to-speech.cpp:117-125,173-176) handles every vocabulary type llama.cpp has;
llama.cpp is absent here (the un-vendored submodule), so the check is against the
published BERT WordPiece algorithm its WPM tokenizer reproduces: a vocabulary trained with
`tokenizers`' WordPieceTrainer under the BERT normalizer (control characters dropped, CJK
ideographs split, accents stripped, lowercase) and pre-tokenizer (whitespace and punctuation
splits) is written into a GGUF the way convert_hf_to_gguf.py writes a BERT vocabulary
(word-initial tokens prefixed with U+2581, "##" continuations without it, the bracketed
specials as CONTROL tokens), and every held-out string must give the same ids. The texts use
precomposed accents and kana with voicing marks, whose first decomposition code point is the
stripped letter in both; llama.cpp's one-code-point NFD differs from the full BERT
normalization on Hangul syllables, stand-alone combining marks and multi-letter lowercase
mappings, which the texts leave out."""
import random

import pytest

import miotts_amd as m
from miotts_amd import gguf_np

tk = pytest.importorskip("tokenizers")

_SPECIALS = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
_ALPHA = (list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ") * 3 + list("0123456789") * 2
          + list(" ") * 16 + list(".,;:!?-()'\"$+<=>^`|~/@#%&*[]{}_\\") + list("\t\n")
          + list("あいうえおかきくけこさしすせそがぎぐげごぱぴアイウエオガギグーッ") + list("今日天気東京大学生時間語本人、。「」")
          + list("éèêëàâäôöùûüçñÉÀÖÜÑßøåÅæ"))
_RARE = list("αβγΔΩабвгдЖЩ😀🎉½™€")
_WORDS = ["hello", "World", "The", "it's", "naïve", "Café", "こんにちは", "今日はいい天気ですね", "ありがとう", "12345",
          "3.14", "don't", "Straße", "ÉCOLE"]


def _text(rng, n, rare=False):
    parts = []
    while sum(map(len, parts)) < n:
        if rng.random() < 0.4:
            parts.append(rng.choice(_WORDS))
        else:
            pool = _ALPHA + (_RARE if rare else [])
            parts.append("".join(rng.choice(pool) for _ in range(rng.randint(1, 7))))
        parts.append(" " if rng.random() < 0.6 else "")
    return "".join(parts)


def _trained(vocab_size, seed):
    rng = random.Random(seed)
    corpus = [_text(rng, 200) for _ in range(600)] + _WORDS * 20
    tok = tk.Tokenizer(tk.models.WordPiece(unk_token="[UNK]", max_input_chars_per_word=1000))
    tok.normalizer = tk.normalizers.BertNormalizer(clean_text=True, handle_chinese_chars=True, strip_accents=True,
                                                   lowercase=True)
    tok.pre_tokenizer = tk.pre_tokenizers.BertPreTokenizer()
    trainer = tk.trainers.WordPieceTrainer(vocab_size=vocab_size, special_tokens=_SPECIALS, show_progress=False)
    tok.train_from_iterator(corpus, trainer)
    return tok


def _to_gguf(tok, path, extra=None):
    """convert_hf_to_gguf.py's BERT vocabulary: "##x" -> "x", a word-initial "x" -> U+2581 "x",
    the specials unchanged (CONTROL; [UNK] UNKNOWN)."""
    vocab = tok.get_vocab()
    toks = [None] * len(vocab)
    for t, i in vocab.items():
        toks[i] = t
    out, types = [], []
    for t in toks:
        if t in _SPECIALS:
            out.append(t)
            types.append(2 if t == "[UNK]" else 3)
        elif t.startswith("##"):
            out.append(t[2:])
            types.append(1)
        else:
            out.append("▁" + t)
            types.append(1)
    kv = {
        "general.architecture": "bert",
        "tokenizer.ggml.model": "bert",
        "tokenizer.ggml.tokens": out,
        "tokenizer.ggml.token_type": types,
        "tokenizer.ggml.bos_token_id": vocab["[CLS]"],
        "tokenizer.ggml.seperator_token_id": vocab["[SEP]"],
        "tokenizer.ggml.unknown_token_id": vocab["[UNK]"],
        "tokenizer.ggml.padding_token_id": vocab["[PAD]"],
    }
    kv.update(extra or {})
    gguf_np.write_kv_gguf(path, kv)
    return vocab


@pytest.mark.parametrize("vocab_size,seed", [(600, 1), (1500, 2), (3000, 3)])
def test_wpm_tokenize_matches_hf_wordpiece(tmp_path, vocab_size, seed):
    tok = _trained(vocab_size, seed)
    path = str(tmp_path / f"wpm_{seed}.gguf")
    _to_gguf(tok, path)
    t = m.Tokenizer(path)
    rng = random.Random(100 + seed)
    cases = [_text(rng, rng.randint(1, 100), rare=(i % 3 == 0)) for i in range(300)]
    cases += ["", " ", "  ", "a", " a", "a  b", "x\ty", "\n", "Hello, World!", "こんにちは 世界", "😀", "ÅÅÅ",
              "3.14159", "abc  ", "東京大学", "naïve café", "A+B=C", "$100", "x^2|y~z", "`code`", "がぎぐ",
              "unknownword😀xyz", "ℵ"]
    bad = []
    for s in cases:
        want = tok.encode(s, add_special_tokens=False).ids
        got = t.tokenize(s, add_special=False)
        if got != want:
            bad.append((s, got, want))
    assert not bad, f"{len(bad)}/{len(cases)} differ, first: {bad[0]!r}"


def test_wpm_cls_sep_and_pieces(tmp_path):
    """[CLS] opens and [SEP] closes the text (llama.cpp's WPM defaults); control tokens in the
    text are matched with parse_special; pieces render U+2581 as a space and the specials as
    their text (llama_token_to_piece, special = true)."""
    tok = _trained(1000, 7)
    path = str(tmp_path / "wpm.gguf")
    vocab = _to_gguf(tok, path)
    t = m.Tokenizer(path)
    cls, sep = vocab["[CLS]"], vocab["[SEP]"]
    ids = tok.encode("Hello world", add_special_tokens=False).ids
    assert t.tokenize("Hello world") == [cls] + ids + [sep]
    assert t.tokenize("", add_special=True) == [cls, sep]
    got = t.tokenize("ab[SEP]cd", add_special=False, parse_special=True)
    assert got == tok.encode("ab", add_special_tokens=False).ids + [sep] + tok.encode("cd", add_special_tokens=False).ids
    assert t.piece(sep) == b"[SEP]" and t.piece(vocab["[UNK]"]) == b"[UNK]"
    # word-initial tokens render with a leading space, continuations without
    text = "".join(t.piece(i).decode() for i in t.tokenize("hello world", add_special=False))
    assert text == " hello world"
    # add_bos_token / add_sep_token switch the wrappers off
    path2 = str(tmp_path / "wpm_nospecial.gguf")
    _to_gguf(tok, path2, {"tokenizer.ggml.add_bos_token": False, "tokenizer.ggml.add_sep_token": False})
    assert m.Tokenizer(path2).tokenize("Hello world") == ids
