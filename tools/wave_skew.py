"""Diagnostic (-DMIO_TL_DIAG -DMIO_TL_WAVES builds, MIO_BUILD_DIR): per RMSNorm matvec launch,
each wave's activation-arrival time relative to wave 0's, median over workgroups (us).
    MIO_BUILD_DIR=.../build_waves python tools/wave_skew.py [--pos 400]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import numpy as np  # noqa: E402
import miotts_amd as m  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--preset", type=int, default=3)
p.add_argument("--pos", type=int, default=400)
a = p.parse_args()
path = f"/tmp/trace_llm{a.preset}.gguf"
if not os.path.exists(path):
    m.synth_llm(path, a.preset, 1)
dev = m.Device(0)
llm = m.Llm(dev, path, 2048)
llm.generate([256, 257, 65, 258, 257], a.pos, 0.8, 1, allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800),
             check_interval=50)
t = llm.timeline()
nl = t.shape[0]
names = ["attn_in", "attention", "attn_out", "ffn_in", "ffn_down"] * ((nl - 1) // 5) + ["lm_head"]
for k in ["attn_in", "ffn_in", "lm_head"]:
    idx = [i for i, n in enumerate(names) if n == k]
    rel = t[idx][:, :, 1:8] - t[idx][:, :, 0:1]
    med = np.nanmedian(rel.reshape(-1, 7), axis=0)
    p90 = np.nanpercentile(rel.reshape(-1, 7), 90, axis=0)
    print(f"{k:8s} median " + " ".join(f"w{w + 1}={med[w]:5.2f}" for w in range(7)))
    print(f"{'':8s} p90    " + " ".join(f"w{w + 1}={p90[w]:5.2f}" for w in range(7)))
