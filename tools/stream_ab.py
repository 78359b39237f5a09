"""C5 streaming benchmark (BASELINE configs[4]: miotts-stream-benchmark, 1.7B Q4_K_M, 700
speech tokens) of one build (AB_BIN_DIR selects its binaries), K runs; one JSON line with the
stream_bench.* keys of the fastest run."""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import bench  # noqa: E402

build = os.environ.get("AB_BIN_DIR", os.path.join(REPO, "miotts-llama.cpp_amd", "build"))
llm, codec, voice = bench.ensure_files(os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"), 3, 0, lambda: None)
runs = []
for _ in range(int(os.environ.get("AB_K", 3))):
    p = subprocess.run([os.path.join(REPO, build, "miotts-stream-benchmark") if not os.path.isabs(build)
                        else os.path.join(build, "miotts-stream-benchmark"), "-m", llm, "-c", codec, "-v", voice,
                        "-p", bench.PROMPT, "--max-tokens", "700", "--speech-only", "--ignore-eos"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    runs.append({k: float(v) for k, v in re.findall(r"^stream_bench\.([\w.]+)=([-\d.eE+]+)", p.stdout, re.M)})
best = min(runs, key=lambda r: r["total_sec"])
print(json.dumps({"build": build, "x_realtime": [round(r["x_realtime"], 3) for r in runs], "best": best}), flush=True)
