"""The drop-in boundary as a tested fact: the reference's OWN command-line programs
(/root/reference/src/main.cpp, examples/stream-benchmark.cpp, examples/stream-compare.cpp),
compiled unchanged against this repo's include/ and linked to libmiotts.so in place of
llama.cpp/ggml + src/*.cpp (`make -C oracle callers`, output only
in oracle/_ref/callers/, git-ignored). examples/stream-to-device.cpp needs miniaudio, which
the snapshot lacks, so it is not built.

CPU part (this file): the three programs build and link; every option the reference's usage
text lists is accepted by the repo's own CLIs (csrc/tools/*) under the same name; usage
errors and --help give the same exit codes and the same first error line; without a GPU
both fail the same way (exit 1, the same messages: there is no CPU fallback). The GPU part,
tests/test_reference_callers_gpu.py, runs the reference's programs on synthetic models and
compares their output files byte for byte with the repo's CLIs.
"""
import os
import re
import subprocess

import pytest

import miotts_amd as m

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "miotts-llama.cpp_amd", "build")
CALLERS = os.path.join(REPO, "oracle", "_ref", "callers")
PAIRS = [("miotts", "main.cpp"), ("miotts-stream-benchmark", "stream-benchmark.cpp"),
         ("miotts-stream-compare", "stream-compare.cpp")]


@pytest.fixture(scope="module")
def callers():
    if os.path.isdir("/root/reference/src"):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "callers"])
    if not all(os.path.exists(os.path.join(CALLERS, n)) for n, _ in PAIRS):
        pytest.skip("reference callers not built (no /root/reference here)")
    return CALLERS


def _run(path, args):
    p = subprocess.run([path] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout, p.stderr


def _flags(usage):
    """Option names of a usage text: '-m, --model PATH  ...' -> {'-m', '--model'}."""
    out = set()
    for line in usage.splitlines():
        mm = re.match(r"\s+(-[\w-]+)(?:,\s*(--[\w-]+))?", line)
        if mm:
            out.update(x for x in mm.groups() if x)
    return out


@pytest.mark.parametrize("name,src", PAIRS)
def test_reference_cli_options_are_accepted(callers, name, src):
    rc_ref, out_ref, err_ref = _run(os.path.join(callers, name), ["--help"])
    rc_ours, out_ours, err_ours = _run(os.path.join(BIN, name), ["--help"])
    assert rc_ref == rc_ours == 0
    ref_flags = _flags(out_ref + err_ref)
    assert {"-m", "--model", "-c", "--codec", "-v", "--voice", "-p", "--prompt", "-h", "--help"} <= ref_flags
    missing = ref_flags - _flags(out_ours + err_ours)
    assert not missing, f"{src} options the repo's {name} does not list: {sorted(missing)}"


@pytest.mark.parametrize("name,src", PAIRS)
@pytest.mark.parametrize("args", [[], ["--bogus"], ["-c", "x.gguf"], ["-p", "hi"], ["--max-tokens"]])
def test_reference_cli_usage_errors_match(callers, name, src, args):
    rc_ref, out_ref, err_ref = _run(os.path.join(callers, name), args)
    rc_ours, out_ours, err_ours = _run(os.path.join(BIN, name), args)
    assert rc_ref == rc_ours != 0, (rc_ref, rc_ours)
    assert out_ref == out_ours
    first = lambda e: e.strip().splitlines()[0] if e.strip() else ""
    if not first(err_ref).startswith("Usage:"):
        assert first(err_ref) == first(err_ours)


@pytest.fixture(scope="module")
def models(tmp_path_factory):
    d = tmp_path_factory.mktemp("refcallers")
    return {"llm": m.synth_llm(str(d / "llm.gguf"), 0, 1), "codec": m.synth_codec(str(d / "codec.gguf"), 1, 1),
            "voice": m.synth_voice(str(d / "voice.emb.gguf"), 7), "dir": d}


def _no_gpu():
    try:
        return m.device_count() == 0
    except Exception:
        return True


@pytest.mark.skipif(not _no_gpu(), reason="checks the no-GPU failure path")
@pytest.mark.parametrize("name,extra", [("miotts", ["-o", "x.wav"]), ("miotts-stream-benchmark", []),
                                        ("miotts-stream-compare", [])])
def test_reference_cli_without_gpu_fails_loudly(callers, models, name, extra):
    args = ["-m", models["llm"], "-c", models["codec"], "-v", models["voice"], "-p", "hello",
            "--max-tokens", 8] + extra
    rc_ref, out_ref, err_ref = _run(os.path.join(callers, name), args)
    rc_ours, out_ours, err_ours = _run(os.path.join(BIN, name), args)
    assert rc_ref == rc_ours == 1
    assert out_ref == out_ours and err_ref == err_ours
    assert "no HIP device" in err_ref


def test_miotts_batch_flags(tmp_path):
    """The batch extension of `miotts` (--batch FILE, --gpus N): listed in
    --help, --gpus without --batch and an unreadable or empty --batch file are usage errors
    (exit 1 with a message) before any device is touched."""
    exe = os.path.join(BIN, "miotts")
    rc, out, err = _run(exe, ["--help"])
    assert rc == 0 and "--batch" in out + err and "--gpus" in out + err
    common = ["-c", "c.gguf", "-v", "v.gguf", "-m", "m.gguf"]
    rc, _, err = _run(exe, common + ["-p", "x", "--gpus", "2"])
    assert rc == 1 and "--gpus needs --batch" in err
    rc, _, err = _run(exe, common + ["--batch", str(tmp_path / "missing.txt")])
    assert rc == 1 and "cannot read --batch file" in err
    (tmp_path / "empty.txt").write_text("\n\n")
    rc, _, err = _run(exe, common + ["--batch", str(tmp_path / "empty.txt")])
    assert rc == 1 and "has no prompts" in err
