"""Diagnostic: the ragged 4-stream batch of tests/test_llm_batch_gpu.py::test_batch_1p7b_q4km."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import numpy as np  # noqa: E402

import miotts_amd as m  # noqa: E402

preset = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n_ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 512
path = f"/tmp/diag_llm{preset}.gguf"
if not os.path.exists(path):
    m.synth_llm(path, preset, 1)
dev = m.Device(0)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
rng = np.random.default_rng(17)
lens = [1 if b == 1 else int(rng.integers(3, 40)) for b in range(4)]
prompts = [list(rng.integers(0, 256, n)) for n in lens]
print("lens", lens, flush=True)
g = m.Llm(dev, path, n_ctx)
single = [g.generate(prompts[b], 16, 0.8, 42 + b, allow=allow) for b in range(4)]
g2 = m.Llm(dev, path, n_ctx)
got = g2.generate_batch(prompts, 16, 0.8, [42, 43, 44, 45], allow=allow)
for b in range(4):
    print(b, "eq" if np.array_equal(got[b], single[b]) else "DIFF", got[b].tolist(), single[b].tolist(), flush=True)
for b in range(4):
    one = g2.generate_batch([prompts[b]], 16, 0.8, [42 + b], allow=allow)[0]
    print("alone", b, "eq" if np.array_equal(one, single[b]) else "DIFF", flush=True)
for sub in ([0, 2], [0, 1], [2, 3], [0, 3]):
    r = g2.generate_batch([prompts[b] for b in sub], 16, 0.8, [42 + b for b in sub], allow=allow)
    print("pair", sub, ["eq" if np.array_equal(r[i], single[b]) else "DIFF" for i, b in enumerate(sub)], flush=True)
