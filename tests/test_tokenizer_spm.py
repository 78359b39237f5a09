"""CPU: the GGUF SPM tokenizer (tokenizer.ggml.model "llama"; csrc/host/tokenizer.cpp, llama.cpp's
llm_tokenizer_spm restated) against the `sentencepiece` package's BPE encoder on trained
vocabularies.

llama_tokenize (test-to-speech.cpp:117-125,173-176) handles every vocabulary type llama.cpp has;
llama.cpp is absent here (the un-vendored submodule), so the check is against the
published SentencePiece BPE algorithm its SPM tokenizer reproduces (llama.cpp's own
test-tokenizer-0 vectors for SPM models come from sentencepiece): a BPE model trained with
byte fallback, identity normalization, a dummy prefix and whitespace runs kept (what
llama.cpp's SPM path does: no normalization, " " prefix, ' ' -> U+2581) is written into a GGUF
(pieces, scores, token types in id order) and every held-out string must give the same ids;
pieces must render the text back (byte tokens -> bytes, U+2581 -> ' ')."""
import random

import pytest

import miotts_amd as m
from miotts_amd import gguf_np

spm = pytest.importorskip("sentencepiece")

_ALPHA = (list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ") * 3 + list("0123456789") * 2
          + list(" ") * 14 + list(".,;:!?-()'\"")
          + list("あいうえおかきくけこさしすせそたちつてとなにぬねのはひふへほまみむめもやゆよらりるれろわをん")
          + list("アイウエオカキクケコサシスセソタチツテトナニヌネノーッ") + list("今日天気東京大学生時間語本人、。"))
_RARE = list("αβγΔΩабвгд한국어😀🎉éüñßÅ½\t")
_WORDS = ["hello", "world", "The", "it's", "こんにちは", "今日はいい天気ですね", "ありがとう", "12345", "  ", "3.14"]


def _text(rng, n, rare=False):
    parts = []
    while sum(map(len, parts)) < n:
        r = rng.random()
        if r < 0.4:
            parts.append(rng.choice(_WORDS))
        else:
            pool = _ALPHA + (_RARE if rare else [])
            parts.append("".join(rng.choice(pool) for _ in range(rng.randint(1, 6))))
    return "".join(parts)


def _trained(tmp_path, vocab_size, seed):
    rng = random.Random(seed)
    corpus = tmp_path / f"corpus_{seed}.txt"
    corpus.write_text("\n".join(_text(rng, 200) for _ in range(800)) + "\n" + "\n".join(_WORDS * 20), "utf-8")
    prefix = str(tmp_path / f"spm_{seed}")
    spm.SentencePieceTrainer.train(
        input=str(corpus), model_prefix=prefix, model_type="bpe", vocab_size=vocab_size, byte_fallback=True,
        normalization_rule_name="identity", add_dummy_prefix=True, remove_extra_whitespaces=False,
        character_coverage=1.0, allow_whitespace_only_pieces=True, split_digits=False, minloglevel=2,
        bos_id=1, eos_id=2, unk_id=0, pad_id=-1)
    return spm.SentencePieceProcessor(model_file=prefix + ".model")


def _to_gguf(sp, path, add_bos):
    n = sp.get_piece_size()
    toks = [sp.id_to_piece(i) for i in range(n)]
    scores = [float(sp.get_score(i)) for i in range(n)]
    types = [2 if sp.is_unknown(i) else 3 if sp.is_control(i) else 6 if sp.is_byte(i) else 5 if sp.is_unused(i)
             else 1 for i in range(n)]
    gguf_np.write_kv_gguf(path, {
        "general.architecture": "llama",
        "tokenizer.ggml.model": "llama",
        "tokenizer.ggml.tokens": toks,
        "tokenizer.ggml.scores": scores,
        "tokenizer.ggml.token_type": types,
        "tokenizer.ggml.bos_token_id": sp.bos_id(),
        "tokenizer.ggml.eos_token_id": sp.eos_id(),
        "tokenizer.ggml.unknown_token_id": sp.unk_id(),
        "tokenizer.ggml.add_bos_token": add_bos,
    })
    return types


@pytest.mark.parametrize("vocab_size,seed", [(800, 1), (2000, 2), (4000, 3)])
def test_spm_tokenize_matches_sentencepiece(tmp_path, vocab_size, seed):
    sp = _trained(tmp_path, vocab_size, seed)
    path = str(tmp_path / f"spm_{seed}.gguf")
    types = _to_gguf(sp, path, False)
    assert types.count(6) == 256  # every byte has its <0xXX> token
    t = m.Tokenizer(path)
    rng = random.Random(100 + seed)
    cases = [_text(rng, rng.randint(1, 100), rare=(i % 3 == 0)) for i in range(300)]
    cases += ["", " ", "  ", "a", " a", "a  b", "x\ty", "\n", "こんにちは 世界", "😀", "ÅÅÅ", "3.14159", "abc  ",
              "ℵ", "　あ"]
    bad = []
    for s in cases:
        want = sp.encode(s)
        got = t.tokenize(s, add_special=False)
        if got != want:
            bad.append((s, got, want))
        # pieces render the text back: the dummy-prefix space of a non-empty text dropped
        back = t.detokenize(got)
        assert back == (" " + s if s else ""), (s, back)
    assert not bad, f"{len(bad)}/{len(cases)} differ, first: {bad[0]!r}"


def test_spm_bos_and_special_pieces(tmp_path):
    """add_bos_token puts BOS in front (llama.cpp's SPM default); control tokens in the text are
    matched with parse_special and then open a fragment that takes the space prefix again;
    the BOS / EOS / UNK pieces render as their text (llama_token_to_piece, special = true)."""
    sp = _trained(tmp_path, 1000, 7)
    path = str(tmp_path / "spm_bos.gguf")
    _to_gguf(sp, path, True)
    t = m.Tokenizer(path)
    assert t.tokenize("hello world") == [sp.bos_id()] + sp.encode("hello world")
    assert t.tokenize("", add_special=True) == [sp.bos_id()]
    # "<s>" in the text is the BOS control token; the text after it gets its own space prefix
    got = t.tokenize("ab</s>cd", add_special=False, parse_special=True)
    assert got == sp.encode("ab") + [sp.eos_id()] + sp.encode("cd")
    assert t.piece(sp.eos_id()) == b"</s>" and t.piece(sp.unk_id()) == b"<unk>"
