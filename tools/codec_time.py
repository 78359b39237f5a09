"""Codec decode time at T = 700 (the bench's codec shape): 2 warm decodes, then 8 timed,
HIP-event codec / iSTFT ms (mio_hip_codec_last_timings): min and median. A/B helper, e.g.
MIO_CODEC_GEMM=f32 python tools/codec_time.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import miotts_amd as m  # noqa: E402

_, cp, vp = bench.ensure_files(os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"), 3, 0, lambda: None)
dev = m.Device(0)
c = m.Codec(dev, cp)
emb = m.read_voice(vp)
codes = (np.arange(700) * 7919) % 12800
for _ in range(2):
    c.decode_pcm(codes, emb)
ms = []
for _ in range(8):
    c.decode_pcm(codes, emb)
    ms.append(c.last_timings())
cm = sorted(x[0] for x in ms)
print(f"codec ms min {cm[0]:.3f} median {cm[len(cm) // 2]:.3f}; flops {c.last_flops():.4g} -> "
      f"{c.last_flops() / (cm[len(cm) // 2] * 1e-3) / 1e12:.1f} TF/s", flush=True)
