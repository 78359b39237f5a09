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
    # wall (first start -> last end of the second decode), gaps between kernels, totals per kind
    # the second decode: everything after the last host copy (the codes upload)
    last_copy = max(i for i, r in enumerate(rows) if "copyBuffer" in r["Kernel_Name"])
    sec = [r for r in rows[last_copy + 1:]]
    wall = (int(sec[-1]["End_Timestamp"]) - int(sec[0]["Start_Timestamp"])) / 1e3
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(sec, sec[1:])]
    print(f"wall {wall / 1e3:.3f} ms, gaps {sum(gaps) / 1e3:.3f} ms (median {sorted(gaps)[len(gaps) // 2]:.2f} us)")
    kinds = {}
    for r in sec:
        nm = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        k = nm.split("(")[0].split("<")[0].split("::")[-1]
        if nm.startswith("_ZN"):
            k = nm[nm.index("N_1") + 4:][:24]
        if "gemm_f32_kernel" in nm:
            k = "gemm_f32_kernel" + nm[nm.index("<"):nm.index(">") + 1]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c = kinds.setdefault(k, [0, 0.0])
        c[0] += 1
        c[1] += d
    for k, (cnt, d) in sorted(kinds.items(), key=lambda x: -x[1][1]):
        print(f"  {k:40s} {cnt:4d} x  {d:8.1f} us")
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
codes = (np.arange(int(os.environ.get("CODEC_T", 700))) * 7919) % 12800
for _ in range(2):
    c.decode_pcm(codes, emb)
print("codec ms", c.last_timings())
