"""Diagnostic: wall time of batched prefill (llm_prefill.hip) on the bench model vs the
token count, to price the one-weight-pass-per-chunk engine against the single-token step.
usage: python tools/prefill_time.py [preset]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import numpy as np  # noqa: E402

import miotts_amd as m  # noqa: E402

preset = int(sys.argv[1]) if len(sys.argv) > 1 else 3
wd = os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench")
os.makedirs(wd, exist_ok=True)
path = os.path.join(wd, f"llm_preset{preset}.gguf")
if not os.path.exists(path):
    m.synth_llm(path + ".tmp", preset, 1)
    os.replace(path + ".tmp", path)
dev = m.Device(0)
llm = m.Llm(dev, path, 2048)
rng = np.random.default_rng(0)
base = None
for n in (1, 2, 9, 17, 33, 65, 68, 129, 257):
    toks = rng.integers(0, 256, n).astype(np.int32)
    llm.prefill(toks)
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        llm.prefill(toks)
        best = min(best, time.perf_counter() - t0)
    if base is None:
        base = best
    extra = (best - base) * 1e3
    chunks = (n - 1 + 15) // 16
    print(f"n={n:4d} prefill+eval {best * 1e3:8.3f} ms  prefill part {extra:8.3f} ms "
          f"({extra / max(chunks, 1):.3f} ms per 16-token chunk, {extra / max(n - 1, 1):.4f} ms/token)", flush=True)
