"""Diagnose test_miotts_batch_equals_single_runs: determinism of the single and batch CLI runs,
and which engine switch makes the batch WAV of the third prompt equal the single run's."""
import hashlib
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

d = "/tmp/batch_cli_repro"
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
    run(["-p", prompts[i], "-o", f"{d}/s{i}_0.wav"])
print("single", [h(f"{d}/s{i}_0.wav") for i in range(3)], flush=True)
runs = [("def", {})] * 3 + [("no_qf", {"MIO_BT_QF": "0"})] * 3 + [("nograph", {"MIO_NO_GRAPH": "1"})] * 2 + \
       [("no_attq", {"MIO_ATT_Q": "0"})] * 2 + [("no_btatt", {"MIO_BT_ATT": "0"})] * 2
for k, (name, env) in enumerate(runs):
    run(["--batch", d + "/batch.txt", "-o", f"{d}/b{k}.wav", "--gpus", "1"], env)
    print(name, [h(f"{d}/b{k}_{i:03d}.wav") for i in range(3)], flush=True)
