"""CPU: the GGUF UGM tokenizer (tokenizer.ggml.model "t5"; csrc/host/tokenizer.cpp, llama.cpp's
llm_tokenizer_ugm restated) against the `sentencepiece` package's Unigram encoder on trained
vocabularies.

llama_tokenize (test-to-speech.cpp:117-125,173-176) handles every vocabulary type llama.cpp has;
llama.cpp is absent here (the un-vendored submodule), so the check is against the
published SentencePiece Unigram algorithm its UGM tokenizer reproduces: Unigram models are
trained with the default nmt_nfkc normalizer (the precompiled character map: NFKC folding of
full-width forms, circled digits, half-width kana, ...) and with the identity normalizer, with
and without whitespace merging, and written into a GGUF as convert_hf_to_gguf.py writes a T5
vocabulary (pieces, scores, token types, the character map as a u8 array, add_space_prefix,
remove_extra_whitespaces); every held-out string must give the same ids. Texts are given to
both as one fragment (parse_special off: llama.cpp normalizes each text fragment between
special tokens on its own). One difference is llama.cpp's and kept: without whitespace merging,
a text of whitespace only gets no prefix space (its normalizer prepends one in front of the first
non-space character), where sentencepiece prepends it anyway ("  " -> two U+2581, not three)."""
import random

import pytest

import miotts_amd as m
from miotts_amd import gguf_np

spm = pytest.importorskip("sentencepiece")
from sentencepiece import sentencepiece_model_pb2 as spm_pb  # noqa: E402

_ALPHA = (list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ") * 3 + list("0123456789") * 2
          + list(" ") * 16 + list(".,;:!?-()'\"") + list("あいうえおかきくけこさしすせそがぎアイウエオーッ")
          + list("今日天気東京大学生時間語本人、。") + list("ＡＢＣａｂｃ１２３①②ｶﾀｶﾅﾞ") + list("éüñÅ"))
_RARE = list("αβγΔΩабвгд한국어😀🎉½™\t")
_WORDS = ["hello", "world", "The", "it's", "こんにちは", "今日はいい天気ですね", "ありがとう", "12345", "  ", "3.14",
          "ＡＢＣ", "ｶﾀｶﾅ", "①②③", "<tag>"]


def _text(rng, n, rare=False):
    parts = []
    while sum(map(len, parts)) < n:
        if rng.random() < 0.4:
            parts.append(rng.choice(_WORDS))
        else:
            pool = _ALPHA + (_RARE if rare else [])
            parts.append("".join(rng.choice(pool) for _ in range(rng.randint(1, 6))))
    return "".join(parts)


def _trained(tmp_path, vocab_size, seed, norm, merge):
    rng = random.Random(seed)
    corpus = tmp_path / f"corpus_{seed}.txt"
    corpus.write_text("\n".join(_text(rng, 200) for _ in range(800)) + "\n" + "\n".join(_WORDS * 20), "utf-8")
    prefix = str(tmp_path / f"ugm_{seed}_{norm}_{int(merge)}")
    spm.SentencePieceTrainer.train(
        input=str(corpus), model_prefix=prefix, model_type="unigram", vocab_size=vocab_size,
        normalization_rule_name=norm, add_dummy_prefix=True, remove_extra_whitespaces=merge,
        character_coverage=0.9995, user_defined_symbols=["<tag>"], minloglevel=2,
        pad_id=0, eos_id=1, unk_id=2, bos_id=-1)
    return prefix + ".model"


def _to_gguf(model_file, path, extra=None):
    mp = spm_pb.ModelProto()
    with open(model_file, "rb") as f:
        mp.ParseFromString(f.read())
    ns = mp.normalizer_spec
    kv = {
        "general.architecture": "t5",
        "tokenizer.ggml.model": "t5",
        "tokenizer.ggml.tokens": [p.piece for p in mp.pieces],
        "tokenizer.ggml.scores": [float(p.score) for p in mp.pieces],
        "tokenizer.ggml.token_type": [int(p.type) for p in mp.pieces],
        "tokenizer.ggml.add_space_prefix": bool(ns.add_dummy_prefix),
        "tokenizer.ggml.remove_extra_whitespaces": bool(ns.remove_extra_whitespaces),
        "tokenizer.ggml.eos_token_id": 1,
        "tokenizer.ggml.unknown_token_id": 2,
        "tokenizer.ggml.padding_token_id": 0,
    }
    if ns.precompiled_charsmap:
        kv["tokenizer.ggml.precompiled_charsmap"] = bytes(ns.precompiled_charsmap)
    kv.update(extra or {})
    gguf_np.write_kv_gguf(path, kv)
    return mp


@pytest.mark.parametrize("vocab_size,seed,norm,merge", [(800, 1, "nmt_nfkc", True), (2000, 2, "nmt_nfkc", False),
                                                         (1500, 3, "identity", True), (2500, 4, "identity", False)])
def test_ugm_tokenize_matches_sentencepiece(tmp_path, vocab_size, seed, norm, merge):
    model = _trained(tmp_path, vocab_size, seed, norm, merge)
    sp = spm.SentencePieceProcessor(model_file=model)
    path = str(tmp_path / f"ugm_{seed}.gguf")
    mp = _to_gguf(model, path)
    assert bool(mp.normalizer_spec.precompiled_charsmap) == (norm == "nmt_nfkc")
    t = m.Tokenizer(path)
    rng = random.Random(100 + seed)
    cases = [_text(rng, rng.randint(1, 100), rare=(i % 3 == 0)) for i in range(300)]
    cases += ["", " ", "  ", "a", " a", "a  b", "a  ", "x\ty", "\n", "こんにちは 世界", "😀", "ÅÅÅ", "3.14159",
              "ＡＢＣ　ａｂｃ", "①②", "ｶﾞｷﾞ", "hello<tag>world", "<tag>", "한국어", "é́", "ﬁle"]
    bad = []
    for s in cases:
        got = t.tokenize(s, add_special=False, parse_special=False)
        if not merge and s and not sp.normalize(s).strip("▁"):  # whitespace only: llama.cpp's form
            want = sp.encode(s)[1:]
        else:
            want = sp.encode(s)
        if got != want:
            bad.append((s, got, want))
    assert not bad, f"{len(bad)}/{len(cases)} differ, first: {bad[0]!r}"


def test_ugm_eos_and_pieces(tmp_path):
    """EOS closes the text (llama.cpp's UGM default), no BOS; pieces render U+2581 as a space,
    UNK and the user-defined token as their text."""
    model = _trained(tmp_path, 1000, 7, "nmt_nfkc", True)
    sp = spm.SentencePieceProcessor(model_file=model)
    path = str(tmp_path / "ugm.gguf")
    _to_gguf(model, path)
    t = m.Tokenizer(path)
    assert t.tokenize("hello world") == sp.encode("hello world") + [1]
    assert t.tokenize("", add_special=True) == [1]
    ids = t.tokenize("hello world", add_special=False)
    assert b"".join(t.piece(i) for i in ids) == b" hello world"
    tag = sp.piece_to_id("<tag>")
    # parse_special: the user-defined token splits the text, each fragment normalized alone
    assert t.tokenize("ab<tag>cd", add_special=False) == sp.encode("ab") + [tag] + sp.encode("cd")
    assert t.piece(tag) == b"<tag>" and t.piece(2) == sp.id_to_piece(2).encode()
    path2 = str(tmp_path / "ugm_noeos.gguf")
    _to_gguf(model, path2, {"tokenizer.ggml.add_eos_token": False})
    assert m.Tokenizer(path2).tokenize("hello world") == sp.encode("hello world")
