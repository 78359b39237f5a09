"""Diagnostic: the bench's HIP-event launch timing of the decode step's kernels
(mio_hip_llm_time_kernel) repeated, at decode position ~400 of the bench model; run it under
rocprofv3 --kernel-trace to compare each launch's own duration with the event figure.
usage: python tools/time_kernel_probe.py [preset] [which ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

preset = int(sys.argv[1]) if len(sys.argv) > 1 else 3
which = [int(w) for w in sys.argv[2:]] or [11, 12, 6]
wd = os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench")
os.makedirs(wd, exist_ok=True)
path = os.path.join(wd, f"llm_preset{preset}.gguf")
if not os.path.exists(path):
    m.synth_llm(path + ".tmp", preset, 1)
    os.replace(path + ".tmp", path)
dev = m.Device(0)
llm = m.Llm(dev, path, 2048)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
prompt = [256, 257] + list(b"user\nhello") + [258, 257]
for _ in range(int(os.environ.get("PROBE_HEAVY", 0))):  # the bench's timed region before
    llm.generate(prompt, 700, 0.8, 42, allow=allow)
llm.generate(prompt, 400, 0.8, 42, allow=allow)
if os.environ.get("PROBE_TL") == "1":  # bench.roofline takes the step timeline first
    llm.timeline()
for w in which:
    for r in range(int(os.environ.get("PROBE_REPS", 4))):
        ms, by = llm.time_kernel(w, 40)
        print(f"which {w} rep {r}: {ms * 1e3:.3f} us per launch, {by} B", flush=True)
