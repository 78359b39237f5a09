"""Diagnostic: phase timeline of one persistent decode step (1.7B preset by default), per
phase type the median over workgroups of each segment: body start -> prologue done ->
body done -> arrived (stores drained) -> poll done -> inputs staged, the prefetch issue
time of the row waves, and the phase span (start to the next phase's start, max over
workgroups). Run on the GPU box:  python tools/persist_timeline.py [--preset 3] [--pos 400]"""
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
             check_interval=a.pos)
for rep in range(3):
    t = llm.persist_timeline()
n = t.shape[0]
names = ["attn_in", "attention", "attn_out", "ffn_in", "ffn_down"] * ((n - 2) // 5) + ["lm_head", "sample"]
start = np.nanmax(t[:, :, 0], axis=1)
span = np.r_[start[1:] - start[:-1], np.nan]
print(f"step: {np.nanmax(t[:, :, 3]) - np.nanmin(t[:, :, 0]):.1f} us over {n} phases (first start -> last arrive)")
seg = {
    "start->prologue": (0, 1), "prologue->body": (1, 2), "body->arrived": (2, 3),
    "arrived->polled": (3, 4), "polled->staged": (4, 5), "arrived->prefetched": (3, 6),
}
print(f"{'phase':10s} {'span':>7s} " + " ".join(f"{k:>18s}" for k in seg))
for nm in dict.fromkeys(names):
    idx = [i for i, x in enumerate(names) if x == nm]
    row = [np.nanmean(span[idx])]
    for k, (i0, i1) in seg.items():
        row.append(np.nanmean([np.nanmedian(t[i, :, i1] - t[i, :, i0]) for i in idx]))
    print(f"{nm:10s} " + " ".join(f"{v:7.2f}" if j == 0 else f"{v:18.2f}" for j, v in enumerate(row)))
# arrival skew: last arriving workgroup vs median, per phase type
print("arrival skew (max - median of 'arrived'):")
for nm in dict.fromkeys(names):
    idx = [i for i, x in enumerate(names) if x == nm]
    sk = [np.nanmax(t[i, :, 3]) - np.nanmedian(t[i, :, 3]) for i in idx]
    print(f"  {nm:10s} {np.nanmean(sk):6.2f}")
