"""Diagnostic: per-checkpoint timing inside the decode-step kernels (1.7B preset), from the
s_memtime tracing of mio_hip_llm_trace_kernel. Run on the GPU box:
    python tools/trace_kernels.py [--preset 3] [--pos 700]
Prints, per kernel, the delta (us) from kernel entry to each reached checkpoint."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import numpy as np  # noqa: E402
import miotts_amd as m  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--preset", type=int, default=3)
p.add_argument("--pos", type=int, default=700)
a = p.parse_args()
path = f"/tmp/trace_llm{a.preset}.gguf"
if not os.path.exists(path):
    m.synth_llm(path, a.preset, 1)
dev = m.Device(0)
llm = m.Llm(dev, path, 2048)
prompt = [256, 257, 65, 258, 257]
llm.generate(prompt, a.pos, 0.8, 1, allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800), check_interval=50)
names = {0: "attn_in", 1: "attention", 2: "attn_out", 3: "ffn_in", 4: "ffn_down", 6: "lm_head", 7: "sample"}
for which, name in names.items():
    best = None
    for rep in range(5):
        t = llm.trace_kernel(which).astype(np.int64)
        if t[0] == 0:
            break
        if best is None or t[15] - t[0] < best[15] - best[0]:
            best = t
    if best is None:
        print(f"{name:10s} (no checkpoints)")
        continue
    t = best
    real_us = (int(t[31]) - int(t[16])) * 0.01
    cyc = int(t[15]) - int(t[0])
    ghz = cyc / (real_us * 1e3) if real_us > 0 else 0.0
    parts = []
    for k in range(1, 16):
        if t[k]:
            parts.append(f"c{k}={(int(t[k]) - int(t[0])) / max(ghz, 1e-9) / 1e3:.2f}")
    print(f"{name:10s} total {real_us:6.2f} us ({ghz:.2f} GHz)  " + " ".join(parts))
    if which != 7:
        llm.time_kernel(which, 3)
