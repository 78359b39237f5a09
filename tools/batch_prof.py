"""Workload for rocprofv3 of the batched decode path (MIO_NO_GRAPH=1 for eager launches):
B streams x N steps on the bench model. usage: python tools/batch_prof.py [B] [N] [preset]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
preset = int(sys.argv[3]) if len(sys.argv) > 3 else 3
wd = os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench")
os.makedirs(wd, exist_ok=True)
path = os.path.join(wd, f"llm_preset{preset}.gguf")
if not os.path.exists(path):
    m.synth_llm(path + ".tmp", preset, 1)
    os.replace(path + ".tmp", path)
dev = m.Device(0)
llm = m.Llm(dev, path, int(os.environ.get("AB_NCTX", 2048)))
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
prompt = [256, 257] + list(b"user\nhello") + [258, 257]
llm.generate_batch([prompt] * B, 8, 0.8, list(range(B)), allow=allow)
t0 = time.perf_counter()
out = llm.generate_batch([prompt] * B, N, 0.8, list(range(B)), allow=allow)
dt = time.perf_counter() - t0
print(f"B={B} N={N}: {dt * 1e3:.1f} ms, {dt * 1e3 / N:.3f} ms/step", flush=True)
