"""GPU: the reference's own programs (src/main.cpp, examples/stream-benchmark.cpp,
examples/stream-compare.cpp) compiled unchanged against include/ and linked to libmiotts.so
(oracle/_ref/callers/, built by `make -C oracle callers`; see tests/test_reference_callers.py)
run the path end to end on synthetic models, next to the repo's own CLIs with the same
arguments: the WAV files they write are identical byte for byte, and so are the counts
they print (stream_bench.llm_tokens / decode_calls / decoded_codes / emitted_samples,
compare.* sample counts and differences). The reference's sampler seed and options are the
library's defaults on both sides, so the runs are deterministic.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import miotts_amd as m

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "miotts-llama.cpp_amd", "build")
CALLERS = os.path.join(REPO, "oracle", "_ref", "callers")


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    if not os.path.exists(os.path.join(CALLERS, "miotts")):
        pytest.skip("reference callers not built (build() builds them where /root/reference exists)")
    d = tmp_path_factory.mktemp("refcallers_gpu")
    return {"llm": m.synth_llm(str(d / "llm1.gguf"), 1, 1), "codec": m.synth_codec(str(d / "codec.gguf"), 1, 1),
            "voice": m.synth_voice(str(d / "voice.emb.gguf"), 7), "dir": d}


def _run(path, args):
    p = subprocess.run([path] + [str(a) for a in args], capture_output=True, text=True, timeout=300)
    return p.returncode, p.stdout, p.stderr


def _both(name, args_for):
    """Runs the reference's program and the repo's CLI; args_for(tag) builds the arguments
    (output paths differ per side)."""
    ref = _run(os.path.join(CALLERS, name), args_for("ref"))
    ours = _run(os.path.join(BIN, name), args_for("ours"))
    assert ref[0] == ours[0] == 0, f"{name}: rc {ref[0]} / {ours[0]}\n{ref[2][-1500:]}\n{ours[2][-1500:]}"
    return ref, ours


def _kv(out):
    return dict(re.findall(r"^([\w.]+)=([^\s]+)", out, re.M))


def test_reference_main_synthesizes_same_wav(files):
    d = files["dir"]
    args = lambda t: ["-m", files["llm"], "-c", files["codec"], "-v", files["voice"], "-p", "テストです。",
                      "-o", d / f"main_{t}.wav", "--max-tokens", 64]
    _both("miotts", args)
    a, b = (d / "main_ref.wav").read_bytes(), (d / "main_ours.wav").read_bytes()
    assert len(a) > 44 and a == b


def test_reference_main_skip_llm_same_wav(files):
    d = files["dir"]
    codes = np.random.default_rng(3).integers(0, 12800, 90)
    text = "".join(f"<|s_{c}|>" for c in codes)
    args = lambda t: ["-c", files["codec"], "-v", files["voice"], "-p", text, "--skip-llm", "-o", d / f"skip_{t}.wav"]
    _both("miotts", args)
    a, b = (d / "skip_ref.wav").read_bytes(), (d / "skip_ours.wav").read_bytes()
    assert len(a) == 44 + 2 * 90 * 1764 and a == b


def test_reference_stream_benchmark_same_counts(files):
    args = lambda t: ["-m", files["llm"], "-c", files["codec"], "-v", files["voice"], "-p", "こんにちは。",
                      "--max-tokens", 120]
    (_, out_ref, _), (_, out_ours, _) = _both("miotts-stream-benchmark", args)
    r, o = _kv(out_ref), _kv(out_ours)
    for k in ["llm_tokens", "decode_calls", "decoded_codes", "emitted_samples", "audio_sec"]:
        assert r[f"stream_bench.{k}"] == o[f"stream_bench.{k}"], k
    assert int(r["stream_bench.emitted_samples"]) > 0


def test_reference_stream_compare_same_files(files):
    d = files["dir"]
    codes = np.random.default_rng(4).integers(0, 12800, 200)
    text = "".join(f"<|s_{c}|>" for c in codes)
    args = lambda t: ["-c", files["codec"], "-v", files["voice"], "-p", text, "--skip-llm",
                      "--out-offline", d / f"off_{t}.wav", "--out-stream", d / f"str_{t}.wav"]
    (_, out_ref, _), (_, out_ours, _) = _both("miotts-stream-compare", args)
    r, o = _kv(out_ref), _kv(out_ours)
    assert r and {k: v for k, v in r.items() if "sec" not in k} == {k: v for k, v in o.items() if "sec" not in k}
    for n in ("off", "str"):
        assert (d / f"{n}_ref.wav").read_bytes() == (d / f"{n}_ours.wav").read_bytes()
