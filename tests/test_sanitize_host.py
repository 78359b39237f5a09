"""Host parsers under AddressSanitizer + UndefinedBehaviorSanitizer (CPU; SURVEY §5 "Race
detection / sanitizers"). tests/sanitize/host_fuzz.cpp builds the product's own GGUF reader
(gguf.cpp), tokenizer (tokenizer.cpp: BPE, and WPM / UGM vocabularies written here),
quant re-layout (quant.cpp), text / WAV helpers
(text.cpp) and the synthetic-GGUF writers host-only with -fsanitize=address,undefined
-fno-sanitize-recover=all, and drives them over valid files, every truncation of the headers,
seeded random corruptions and extreme values in every header field (counts, string lengths,
shapes, offsets, general.alignment): every malformed file must be refused with a message, every
accepted one must keep all tensors inside the mapping, and no sanitizer may report. The
reference loader these replace reads by offset the same way (miocodec.cpp:92-135, 426-504).

Quick mode here (one LLM, fewer mutations, ~80 s); `host_fuzz DIR full` is the long run
(3 LLM GGUFs, 12k files opened / 36k refused, clean)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = os.path.join(REPO, "miotts-llama.cpp_amd", "csrc")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"  # g++ 11 has no _Float16 in C++ (quant.cpp)
SRCS = [os.path.join(REPO, "tests", "sanitize", "host_fuzz.cpp")] + [
    os.path.join(H, "host", f) for f in ("gguf.cpp", "tokenizer.cpp", "text.cpp", "quant.cpp")] + [
    os.path.join(H, "testlib", f) for f in ("synth.cpp", "synth_llm.cpp")]


def build(out):
    cmd = [CLANG, "-std=c++20", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-I" + os.path.join(REPO, "include"), "-I" + H, "-I" + os.path.join(H, "host"),
           "-I" + os.path.join(H, "testlib")] + SRCS + ["-o", out]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=600)


def _tokenizer_ggufs(d):
    """Tokenizer-only GGUFs of the WPM and UGM vocabulary types (trained as in their tests; the
    UGM one carries sentencepiece's nmt_nfkc character map), fuzzed beside the LLM GGUF."""
    import pathlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    out = []
    try:
        import test_tokenizer_wpm as w
        p = os.path.join(d, "wpm.gguf")
        w._to_gguf(w._trained(600, 1), p)
        out.append(p)
    except ImportError:
        pass
    try:
        import test_tokenizer_ugm as u
        p = os.path.join(d, "ugm.gguf")
        u._to_gguf(u._trained(pathlib.Path(d), 800, 1, "nmt_nfkc", True), p)
        out.append(p)
    except ImportError:
        pass
    return out


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang++ (host build with sanitizers) absent")
def test_host_parsers_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_fuzz")
    build(exe)
    work = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
    d = os.path.join(work, f"mio_fuzz_{os.getpid()}")
    os.makedirs(d, exist_ok=True)
    try:
        # a small quarantine: the tokenizer reloads its 13k-token vocabulary for every file that opens
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:quarantine_size_mb=4:malloc_context_size=2",
                   OMP_NUM_THREADS="1")
        extra = _tokenizer_ggufs(d)
        p = subprocess.run([exe, d, "quick"] + extra, capture_output=True, text=True, timeout=900, env=env)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-6000:]
    assert "host_fuzz: clean" in p.stdout
    print(p.stdout.strip().splitlines()[-1])
