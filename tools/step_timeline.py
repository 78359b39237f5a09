"""Diagnostic: timeline of one graph-replayed decode step (1.7B preset by default): per
kernel the duration (first workgroup start -> last workgroup end), the spread of workgroup
start and end times, and the gaps between consecutive launches. Run on the GPU box:
    python tools/step_timeline.py [--preset 3] [--pos 700]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import numpy as np  # noqa: E402
import miotts_amd as m  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--preset", type=int, default=3)
p.add_argument("--pos", type=int, default=700)
a = p.parse_args()
path = f"/tmp/trace_llm{a.preset}.gguf"
if not os.path.exists(path):
    m.synth_llm(path, a.preset, 1)
dev = m.Device(0)
llm = m.Llm(dev, path, 2048)
llm.generate([256, 257, 65, 258, 257], a.pos, 0.8, 1, allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800),
             check_interval=50)
t = llm.timeline()
nl = t.shape[0]
KN = {0: "attn_in", 1: "attention", 2: "attn_out", 3: "ffn_in", 4: "ffn_down", 6: "lm_head", 8: "conv_in",
      9: "conv_out", 10: "att_o", 11: "layer_att", 12: "ffn", 13: "layer"}
names = [KN[k] for k in llm.step_kinds()]
s0 = np.nanmin(t[:, :, 0], axis=1)
s1 = np.nanmax(t[:, :, 0], axis=1)
e0 = np.nanmin(t[:, :, 7], axis=1)
e1 = np.nanmax(t[:, :, 7], axis=1)
wd = np.nanmedian(t[:, :, 7] - t[:, :, 0], axis=1)
# per-workgroup phases (median over workgroups): start -> mark 1 -> mark 2 -> end
ph1 = np.nanmedian(t[:, :, 1] - t[:, :, 0], axis=1)
ph2 = np.nanmedian(t[:, :, 2] - t[:, :, 1], axis=1)
ph3 = np.nanmedian(t[:, :, 7] - t[:, :, 2], axis=1)
m2 = np.nanmax(t[:, :, 2], axis=1) - s0
dur = e1 - s0
gap = np.r_[0.0, s0[1:] - e1[:-1]]
print(f"step wall {e1[-1] - s0[0]:.1f} us over {nl} launches; kernel time {dur.sum():.1f} us, "
      f"gaps {gap[1:].sum():.1f} us (mean {gap[1:].mean():.2f}, min {gap[1:].min():.2f}, max {gap[1:].max():.2f})")
print("  kernel      dur    gap-before  start-spread  end-spread  median-wg   wg:->m1  m1->m2  m2->end  last-m2")
for k in ["attn_in", "attention", "attn_out", "layer_att", "ffn_in", "ffn_down", "ffn", "layer", "lm_head"]:
    idx = [i for i, n in enumerate(names) if n == k]
    print(f"  {k:10s} {dur[idx].mean():6.2f} {gap[idx].mean():8.2f} {(s1 - s0)[idx].mean():12.2f} "
          f"{(e1 - e0)[idx].mean():11.2f} {wd[idx].mean():10.2f} {np.nanmean(ph1[idx]):9.2f} "
          f"{np.nanmean(ph2[idx]):7.2f} {np.nanmean(ph3[idx]):8.2f} {np.nanmean(m2[idx]):8.2f}")
# every recorded mark (1-6) and the end, as median offsets from the workgroup's own start
print("  kernel      " + " ".join(f"{'m' + str(k):>6s}" for k in range(1, 7)) + "    end   (us after workgroup start)")
for k in ["attn_in", "attention", "attn_out", "layer_att", "ffn_in", "ffn_down", "ffn", "layer", "lm_head"]:
    idx = [i for i, n in enumerate(names) if n == k]
    cols = []
    for j in list(range(1, 7)) + [7]:
        v = t[idx, :, j] - t[idx, :, 0]
        cols.append(f"{np.nanmedian(v):6.2f}" if np.isfinite(v).any() else "     -")
    print(f"  {k:10s}  " + " ".join(cols))
# the fused attention + O launch: attention workgroups end without mark 3, O workgroups mark 3
# when their wait is over
ia = [i for i, n in enumerate(names) if n == "att_o"]
if ia:
    T = t[ia]
    base = s0[ia][:, None]
    isO = np.isfinite(T[:, :, 3])
    isA = np.isfinite(T[:, :, 7]) & ~isO

    def med(x, msk):
        return float(np.nanmedian(np.where(msk, x, np.nan)))

    def lastv(x, msk):
        return float(np.nanmedian(np.nanmax(np.where(msk, x, np.nan), axis=1)))
    print(f"  att_o: {int(isA[0].sum())} attention workgroups: start {med(T[:, :, 0] - base, isA):.2f} end "
          f"{med(T[:, :, 7] - base, isA):.2f} (last {lastv(T[:, :, 7] - base, isA):.2f}); {int(isO[0].sum())} O "
          f"workgroups: start {med(T[:, :, 0] - base, isO):.2f} (last {lastv(T[:, :, 0] - base, isO):.2f}) wait done "
          f"{med(T[:, :, 3] - base, isO):.2f} (first {-lastv(-(T[:, :, 3] - base), isO):.2f}) x in "
          f"{med(T[:, :, 1] - base, isO):.2f} end {med(T[:, :, 7] - base, isO):.2f} "
          f"(last {lastv(T[:, :, 7] - base, isO):.2f}) us after the launch's first start")
# the whole attention block in one launch: producers (no mark 3), attention (mark 4 = K/V
# staged, mark 3 = q|k|v ready), O workgroups (mark 3, no mark 4)
il = [i for i, n in enumerate(names) if n == "layer_att"]
if il:
    T = t[il]
    base = s0[il][:, None]
    m3, m4 = np.isfinite(T[:, :, 3]), np.isfinite(T[:, :, 4])
    isA, isO = m3 & m4, m3 & ~m4
    isP = np.isfinite(T[:, :, 2]) & ~m3

    def med(x, msk):
        return float(np.nanmedian(np.where(msk, x, np.nan)))

    def lastv(x, msk):
        return float(np.nanmedian(np.nanmax(np.where(msk, x, np.nan), axis=1)))
    print(f"  layer_att: {int(isP[0].sum())} producers end {med(T[:, :, 7] - base, isP):.2f} (last "
          f"{lastv(T[:, :, 7] - base, isP):.2f}); {int(isA[0].sum())} attention: K/V staged "
          f"{med(T[:, :, 4] - base, isA):.2f}, q|k|v ready {med(T[:, :, 3] - base, isA):.2f}, end "
          f"{med(T[:, :, 7] - base, isA):.2f} (last {lastv(T[:, :, 7] - base, isA):.2f}); {int(isO[0].sum())} O: "
          f"wait done {med(T[:, :, 3] - base, isO):.2f}, end {med(T[:, :, 7] - base, isO):.2f} (last "
          f"{lastv(T[:, :, 7] - base, isO):.2f}) us after the launch's first start")
    mg = np.isfinite(T[:, :, 5])
    print(f"  layer_att mergers ({int(mg[0].sum())}): ticket {med(T[:, :, 5] - base, mg):.2f}, outputs written "
          f"{med(T[:, :, 6] - base, mg):.2f}, end {med(T[:, :, 7] - base, mg):.2f}; chunk compute done (m2->end "
          f"of non-mergers) {med(T[:, :, 7] - base, isA & ~mg):.2f} (last {lastv(T[:, :, 7] - base, isA & ~mg):.2f})")
# the FFN pair in one launch: gate|up producers (no mark 3), down workgroups (mark 3 = their
# wait for h is over, mark 1 = h loaded, mark 2 = h quantized)
jf = [i for i, n in enumerate(names) if n == "ffn"]
if jf:
    T = t[jf]
    base = s0[jf][:, None]
    isD = np.isfinite(T[:, :, 3])
    isP = np.isfinite(T[:, :, 7]) & ~isD

    def med(x, msk):
        return float(np.nanmedian(np.where(msk, x, np.nan)))

    def lastv(x, msk):
        return float(np.nanmedian(np.nanmax(np.where(msk, x, np.nan), axis=1)))

    def firstv(x, msk):
        return -lastv(-x, msk)
    print(f"  ffn: {int(isP[0].sum())} gate|up producers: start {med(T[:, :, 0] - base, isP):.2f} (last "
          f"{lastv(T[:, :, 0] - base, isP):.2f}), quantized {med(T[:, :, 2] - base, isP):.2f}, end "
          f"{med(T[:, :, 7] - base, isP):.2f} (last {lastv(T[:, :, 7] - base, isP):.2f}); {int(isD[0].sum())} down: "
          f"start {med(T[:, :, 0] - base, isD):.2f} (last {lastv(T[:, :, 0] - base, isD):.2f}), wait done "
          f"{med(T[:, :, 3] - base, isD):.2f} (first {firstv(T[:, :, 3] - base, isD):.2f}), h in "
          f"{med(T[:, :, 1] - base, isD):.2f}, quantized {med(T[:, :, 2] - base, isD):.2f}, end "
          f"{med(T[:, :, 7] - base, isD):.2f} (last {lastv(T[:, :, 7] - base, isD):.2f}) us after the launch's first start")
# the whole layer in one launch (k_layer): roles by workgroup slot (1.7B: GW = no = GI = GD = 256
# workgroups; the attention chunks are the slots with mark 4 = K/V staged)
jl = [i for i, n in enumerate(names) if n == "layer"]
if jl:
    T = t[jl]
    base = s0[jl][:, None]
    n_act = int(np.isfinite(T[0, :, 4]).sum())
    GW = NO = GI = GD = int(os.environ.get("TL_ROLE_WG", 256))
    j = np.arange(T.shape[1])[None, :].repeat(T.shape[0], 0)
    isP = j < GW
    isA = (j >= GW) & (j < GW + n_act)
    isO = (j >= GW + n_act) & (j < GW + n_act + NO)
    isF = (j >= GW + n_act + NO) & (j < GW + n_act + NO + GI)
    isD = (j >= GW + n_act + NO + GI) & (j < GW + n_act + NO + GI + GD)

    def med(x, msk):
        return float(np.nanmedian(np.where(msk, x, np.nan)))

    def lastv(x, msk):
        return float(np.nanmedian(np.nanmax(np.where(msk, x, np.nan), axis=1)))

    def firstv(x, msk):
        return -lastv(-x, msk)
    R = T - base[:, :, None]
    mg = isA & np.isfinite(T[:, :, 5])
    print(f"  layer: producers end {med(R[:, :, 7], isP):.2f} (last {lastv(R[:, :, 7], isP):.2f}); {n_act} attention: "
          f"q|k|v ready {med(R[:, :, 3], isA):.2f}, end {med(R[:, :, 7], isA):.2f}; mergers ticket "
          f"{med(R[:, :, 5], mg):.2f}, outputs written {med(R[:, :, 6], mg):.2f}")
    print(f"  layer: O start {med(R[:, :, 0], isO):.2f} (last {lastv(R[:, :, 0], isO):.2f}), wait done "
          f"{med(R[:, :, 3], isO):.2f}, x written {med(R[:, :, 6], isO):.2f} (last {lastv(R[:, :, 6], isO):.2f}), end "
          f"{med(R[:, :, 7], isO):.2f}")
    print(f"  layer: gate|up start {med(R[:, :, 0], isF):.2f} (last {lastv(R[:, :, 0], isF):.2f}), x wait done "
          f"{med(R[:, :, 3], isF):.2f} (first {firstv(R[:, :, 3], isF):.2f}), x in {med(R[:, :, 1], isF):.2f}, "
          f"quantized {med(R[:, :, 2], isF):.2f}, end {med(R[:, :, 7], isF):.2f} (last {lastv(R[:, :, 7], isF):.2f})")
    print(f"  layer: down start {med(R[:, :, 0], isD):.2f} (last {lastv(R[:, :, 0], isD):.2f}), h wait done "
          f"{med(R[:, :, 3], isD):.2f} (first {firstv(R[:, :, 3], isD):.2f}), h in {med(R[:, :, 1], isD):.2f}, "
          f"quantized {med(R[:, :, 2], isD):.2f}, end {med(R[:, :, 7], isD):.2f} (last {lastv(R[:, :, 7], isD):.2f}) "
          f"us after the launch's first start")
