"""MioCodec decode (T = 700, preset 0 shapes) twice, for a rocprofv3 kernel trace of the
second run: rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/codec_trace.py
then: python3 tools/codec_trace.py --report OUT/.../run_kernel_trace.csv"""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))

if len(sys.argv) > 2 and sys.argv[1] == "--report":
    rows = []
    with open(sys.argv[2]) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(rows) // 2
    tot = 0
    for r in rows[n:]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        g = f'{r.get("Grid_Size_X", r.get("Grid_Size", "?"))}x{r.get("Grid_Size_Y", "")}'
        nm = r["Kernel_Name"][:70]
        print(f"{d:9.1f} us  grid {g:>14}  wg {r.get('Workgroup_Size_X', r.get('Workgroup_Size', '?'))}  {nm}")
    print(f"total {tot / 1e3:.3f} ms over {len(rows) - n} kernels")
    sys.exit(0)

import numpy as np  # noqa: E402
import miotts_amd as m  # noqa: E402

wd = "/tmp/miotts_bench"
os.makedirs(wd, exist_ok=True)
cp = os.path.join(wd, "miocodec_synth.gguf")
vp = os.path.join(wd, "voice_synth.emb.gguf")
if not os.path.exists(cp):
    m.synth_codec(cp, 0, 1)
if not os.path.exists(vp):
    m.synth_voice(vp, 7)
dev = m.Device(0)
c = m.Codec(dev, cp)
emb = m.read_voice(vp)
codes = (np.arange(700) * 7919) % 12800
for _ in range(2):
    c.decode_pcm(codes, emb)
print("codec ms", c.last_timings())
