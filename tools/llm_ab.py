"""LLM-only timing of one build (MIO_BUILD_DIR selects it): 1 warm + K timed 700-token
generations of the bench workload; prints one JSON line. Used for same-box A/B runs:
  for b in build_a build; do MIO_BUILD_DIR=miotts-llama.cpp_amd/$b python tools/llm_ab.py; done"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import bench  # noqa: E402
import miotts_amd as m  # noqa: E402

preset = int(os.environ.get("AB_PRESET", 3))
K = int(os.environ.get("AB_K", 3))
wd = os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench")
llm_path, _, _ = bench.ensure_files(wd, preset, 0, lambda: None)
dev = m.Device(0)
llm = m.Llm(dev, llm_path, int(os.environ.get("AB_NCTX", 2048)))
prompt = bench.prompt_tokens(bench.PROMPT)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
CI = int(os.environ.get("AB_CI", 20))
llm.generate(prompt, 700, 0.8, 1, allow=allow, check_interval=CI)
ts = []
for k in range(K):
    t0 = time.perf_counter()
    llm.generate(prompt, 700, 0.8, 2 + k, allow=allow, check_interval=CI)
    ts.append(time.perf_counter() - t0)
ev = {}
for which, nm in ((0, "attn_in"), (1, "attention"), (2, "attn_out"), (3, "ffn_in"), (4, "ffn_down"), (6, "lm_head")):
    ev[nm] = round(llm.time_kernel(which, 100)[0] * 1e3, 3)
print(json.dumps({"build": os.environ.get("MIO_BUILD_DIR", "build"), "ms": [round(t * 1e3, 2) for t in ts],
                  "ms_per_token": round(min(ts) * 1e3 / 700, 4), "event_us_at_end": ev}), flush=True)
