"""Diagnostic: batched vs single-stream decode vs the oracle on a preset (default the 1.7B).
usage: python tools/batch_diag.py [preset] [n_ctx]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import miotts_amd as m  # noqa: E402
import pyoracle  # noqa: E402

preset = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n_ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 512
path = f"/tmp/diag_llm{preset}.gguf"
if not os.path.exists(path):
    m.synth_llm(path, preset, 1)
dev = m.Device(0)
g = m.Llm(dev, path, n_ctx)
o = pyoracle.Llm(path, n_ctx)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
rng = np.random.default_rng(17)
for plen, temp in ((10, 0.8), (10, 0.0), (1, 0.8), (40, 0.8)):
    p = list(rng.integers(0, 256, plen))
    b1 = g.generate_batch([p], 12, temp, [42], allow=allow)[0]
    s1 = g.generate(p, 12, temp, 42, allow=allow)
    b2 = g.generate_batch([p, p], 12, temp, [42, 42], allow=allow)
    to = o.generate(p, 12, temp, 42, allow=allow)
    print(f"plen {plen} temp {temp}", flush=True)
    print("  batch1 ", b1.tolist())
    print("  batch2a", b2[0].tolist())
    print("  batch2b", b2[1].tolist())
    print("  single ", s1.tolist())
    print("  oracle ", to.tolist(), flush=True)
# teacher-forced: prefill logits (batched prefill + decode step) vs token-by-token eval
toks = list(rng.integers(0, 256, 20))
lp = g.prefill(toks)
for pos, t in enumerate(toks):
    le = g.eval(int(t), pos)
print("prefill vs eval max|diff|", float(np.abs(lp - le).max()), flush=True)
