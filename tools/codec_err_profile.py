"""Diagnostic: per-stage GPU-vs-oracle error profile of the codec (prints a table)."""
import os, sys, tempfile
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "miotts-llama.cpp_amd", "python"), os.path.join(REPO, "oracle")]
import miotts_amd as m, pyoracle

def rel(g, o):
    d = g.astype(np.float64) - o.astype(np.float64)
    return (np.sqrt(np.mean(d * d)) / (np.sqrt(np.mean(o.astype(np.float64) ** 2)) + 1e-30),
            np.abs(d).max() / (np.abs(o).max() + 1e-30), np.sqrt(np.mean(o.astype(np.float64)**2)))

td = tempfile.mkdtemp()
dev = m.Device(0)
voice = m.read_voice(m.synth_voice(os.path.join(td, "v.gguf"), 7))
for preset, T in [(1, 2), (1, 33), (0, 20), (0, 200)]:
    path = m.synth_codec(os.path.join(td, f"c{preset}.gguf"), preset, 1)
    gc, oc = m.Codec(dev, path), pyoracle.Codec(path)
    codes = (np.arange(T) * 7919 + 13) % 12800
    cap = 18 * T * 512 + 4096
    for st in range(oc.n_stages):
        r = rel(gc.decode_stage(codes, voice, st, cap), oc.decode_stage(codes, voice, st, cap))
        print(f"preset={preset} T={T} stage={st:2d} rel_rms={r[0]:.3e} rel_max={r[1]:.3e} ref_rms={r[2]:.3g}")
    pg = gc.decode_pcm(codes, voice); po = oc.decode_pcm(codes, voice)
    d = pg.astype(np.float64) - po
    print(f"preset={preset} T={T} PCM rms_diff={np.sqrt(np.mean(d*d)):.3e} ref_rms={np.sqrt(np.mean(po.astype(np.float64)**2)):.3g} max={np.abs(d).max():.3e}")
    sys.stdout.flush()
