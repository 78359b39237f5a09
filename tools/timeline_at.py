"""Per-kernel in-graph time per token (step timeline) at several decode positions, for the
build MIO_BUILD_DIR selects: generate up to position p, then one timeline replay."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import bench  # noqa: E402
import miotts_amd as m  # noqa: E402

preset = int(os.environ.get("AB_PRESET", 3))
llm_path, _, _ = bench.ensure_files(os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"), preset, 0, lambda: None)
dev = m.Device(0)
llm = m.Llm(dev, llm_path, 2048)
prompt = bench.prompt_tokens(bench.PROMPT)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
names = ["attn_in", "attention", "attn_out", "ffn_in", "ffn_down"]
res = {}
for n_new in [int(x) for x in os.environ.get('TL_NEW', '30,330,630').split(',')]:
    llm.generate(prompt, n_new, 0.8, 1, allow=allow, check_interval=20)
    tl = llm.timeline()
    nl = tl.shape[0]
    dur = np.nanmax(tl[:, :, 7], axis=1) - np.nanmin(tl[:, :, 0], axis=1)
    per = {nm: round(float(dur[i:nl - 1:5].sum()), 1) for i, nm in enumerate(names)}
    per["lm_head"] = round(float(dur[nl - 1]), 1)
    per["wall"] = round(float(np.nanmax(tl[-1, :, 7]) - np.nanmin(tl[0, :, 0])), 1)
    # attention phases (mean over the layers' launches): first WG start -> mean mark 1 / 2 /
    # end, and the gap from the previous launch's last end to this launch's first start
    att = tl[1:nl - 1:5]
    t0 = np.nanmin(att[:, :, 0], axis=1)
    per["att_m1"] = round(float(np.nanmean(np.nanmean(att[:, :, 1], axis=1) - t0)), 2)
    for k in (2, 3, 4, 5, 6):
        per[f"att_m{k}"] = round(float(np.nanmean(np.nanmean(att[:, :, k], axis=1) - t0)), 2)
    ao = tl[2:nl - 1:5]  # attn_out: mark 1 = first weights issued, 2 = merge + quant done
    a0 = np.nanmin(ao[:, :, 0], axis=1)
    for k in (1, 2):
        per[f"ao_m{k}"] = round(float(np.nanmean(np.nanmean(ao[:, :, k], axis=1) - a0)), 2)
    for i, nm in enumerate(names):  # every kernel: mean mark 2 (prologue done) after its first start
        kk = tl[i:nl - 1:5]
        k0 = np.nanmin(kk[:, :, 0], axis=1)
        per[f"{nm}_m2"] = round(float(np.nanmean(np.nanmean(kk[:, :, 2], axis=1) - k0)), 2)
        per[f"{nm}_end"] = round(float(np.nanmean(np.nanmean(kk[:, :, 7], axis=1) - k0)), 2)
    per["ao_end_mean"] = round(float(np.nanmean(np.nanmean(ao[:, :, 7], axis=1) - a0)), 2)
    per["ao_end_max"] = round(float(np.nanmean(np.nanmax(ao[:, :, 7], axis=1) - a0)), 2)
    per["att_end_mean"] = round(float(np.nanmean(np.nanmean(att[:, :, 7], axis=1) - t0)), 2)
    per["att_end_max"] = round(float(np.nanmean(np.nanmax(att[:, :, 7], axis=1) - t0)), 2)
    per["att_wgs"] = int(np.sum(~np.isnan(att[0, :, 0])))
    prev_end = np.nanmax(tl[0:nl - 1:5][:, :, 7], axis=1)
    per["gap_before_att"] = round(float(np.nanmean(t0 - prev_end)), 2)
    nxt = tl[2:nl - 1:5]
    per["gap_after_att"] = round(float(np.nanmean(np.nanmin(nxt[:, :, 0], axis=1) - np.nanmax(att[:, :, 7], axis=1))), 2)
    res[len(prompt) + n_new] = per
print(json.dumps({"build": os.environ.get("MIO_BUILD_DIR", "build"), "per_pos": res}), flush=True)
