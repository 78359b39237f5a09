"""LLM load wall time of one build (MIO_BUILD_DIR selects it): 1.7B Q4_K_M GGUF (page-cache
warm after the first load) -> HBM arena, 3 loads; one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import bench  # noqa: E402
import miotts_amd as m  # noqa: E402

llm_path, codec_path, _ = bench.ensure_files(os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"), 3, 0,
                                             lambda: None)
dev = m.Device(0)
walls = []
for _ in range(3):
    t0 = time.perf_counter()
    llm = m.Llm(dev, llm_path, 2048)
    walls.append(round((time.perf_counter() - t0) * 1e3, 1))
    del llm
t0 = time.perf_counter()
codec = m.Codec(dev, codec_path)
print(json.dumps({"build": os.environ.get("MIO_BUILD_DIR", "build"), "llm_load_wall_ms": walls,
                  "codec_load_wall_ms": round((time.perf_counter() - t0) * 1e3, 1)}), flush=True)
