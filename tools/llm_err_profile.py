"""Diagnostic: GPU-vs-oracle teacher-forced logits and sampled-token agreement."""
import os, sys, tempfile, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "miotts-llama.cpp_amd", "python"), os.path.join(REPO, "oracle")]
import miotts_amd as m, pyoracle

td = tempfile.mkdtemp()
dev = m.Device(0)
presets = [int(a) for a in sys.argv[1:]] or [0, 1]
for preset in presets:
    path = m.synth_llm(os.path.join(td, f"llm{preset}.gguf"), preset, 1)
    t = time.time(); g = m.Llm(dev, path, 512); print(f"preset {preset} load {time.time()-t:.2f}s vocab {g.n_vocab} layers {g.n_layer} wbytes {g.weight_bytes()/1e6:.1f}MB", flush=True)
    o = pyoracle.Llm(path, 512)
    rng = np.random.default_rng(preset)
    npos = 80 if preset < 2 else 6
    toks = rng.integers(0, g.n_vocab, npos)
    worst = 0; amax_ok = 0
    for pos, tk in enumerate(toks):
        lg = g.eval(int(tk), pos); lo = o.eval(int(tk), pos)
        d = np.abs(lg.astype(np.float64) - lo)
        rel = d.max() / (np.abs(lo).max() + 1e-30)
        worst = max(worst, rel); amax_ok += int(lg.argmax() == lo.argmax())
        if pos in (0, 1, 63, 64, 65, npos - 1):
            print(f"  pos {pos:3d} maxabs {d.max():.3e} rel {rel:.3e} rms {np.sqrt(np.mean(d*d)):.3e} |lo|max {np.abs(lo).max():.3g} argmax_eq {lg.argmax()==lo.argmax()}", flush=True)
    print(f"  worst rel {worst:.3e} argmax agree {amax_ok}/{npos}", flush=True)
    prompt = [256, 257] + list(rng.integers(0, 256, 10)) + [258, 257]
    ng = 40 if preset < 2 else 8
    allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
    t = time.time(); tg = g.generate(prompt, ng, 0.8, 42, allow=allow); tgt = time.time() - t
    tor = o.generate(prompt, ng, 0.8, 42, allow=allow)
    print(f"  generate {len(tg)} toks gpu {tgt:.3f}s; agree {int((tg[:len(tor)]==tor[:len(tg)]).sum())}/{len(tor)}; first {tg[:6]} vs {tor[:6]}", flush=True)
