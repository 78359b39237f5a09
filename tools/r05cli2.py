"""Diagnose test_miotts_batch_equals_single_runs: determinism of the single and batch CLI runs,
and which engine switch makes the batch WAV of the third prompt equal the single run's."""
import hashlib
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

d = "/tmp/r05cli2"
os.makedirs(d, exist_ok=True)
llm = m.synth_llm(d + "/llm1.gguf", 1, 1)
codec = m.synth_codec(d + "/codec.gguf", 0, 1)
voice = m.synth_voice(d + "/voice.emb.gguf", 7)
prompts = ["テストです。", "こんにちは。", "今日はいい天気ですね。"]
open(d + "/batch.txt", "w", encoding="utf-8").write("\n".join(prompts) + "\n")
BIN = os.path.join(REPO, "miotts-llama.cpp_amd", "build", "miotts")
common = ["-m", llm, "-c", codec, "-v", voice, "--max-tokens", "40", "--speech-only", "--ignore-eos"]


def h(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()[:12]


def run(args, env=None):
    p = subprocess.run([BIN] + common + args, capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, **(env or {})))
    if p.returncode != 0 or "unavailable" in p.stderr:
        print("  rc", p.returncode, p.stderr[-400:].replace("\n", " | "), flush=True)


for i in range(3):
    for r in range(2):
        run(["-p", prompts[i], "-o", f"{d}/s{i}_{r}.wav"])
    print("single", i, h(f"{d}/s{i}_0.wav"), h(f"{d}/s{i}_1.wav"), flush=True)
for name, env in (("def_a", {}), ("def_b", {}), ("lm_dot4", {"MIO_BT_LM_MMQ": "0"}), ("no_early", {"MIO_KQ_EARLY": "0"}),
                  ("no_qf", {"MIO_BT_QF": "0"}), ("no_kqloop", {"MIO_MMQ_LOOP_KQ": "0"}), ("gn1", {"MIO_GN": "1"}),
                  ("nograph", {"MIO_NO_GRAPH": "1"})):
    run(["--batch", d + "/batch.txt", "-o", f"{d}/b_{name}.wav", "--gpus", "1"], env)
    print(name, [h(f"{d}/b_{name}_{i:03d}.wav") for i in range(3)], flush=True)
