"""Diagnose: `miotts --batch` on the tiny Q4_K_M preset (test_miotts_batch_equals_single_runs),
timed, stderr kept, under a few engine switches."""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

d = "/tmp/r05cli"
os.makedirs(d, exist_ok=True)
llm = m.synth_llm(d + "/llm1.gguf", 1, 1)
codec = m.synth_codec(d + "/codec.gguf", 0, 1)
voice = m.synth_voice(d + "/voice.emb.gguf", 7)
open(d + "/batch.txt", "w", encoding="utf-8").write("テストです。\nこんにちは。\n今日はいい天気ですね。\n")
BIN = os.path.join(REPO, "miotts-llama.cpp_amd", "build", "miotts")
common = ["-m", llm, "-c", codec, "-v", voice, "--max-tokens", "40", "--speech-only", "--ignore-eos"]
for name, env in (("default", {}), ("lm_dot4", {"MIO_BT_LM_MMQ": "0"}), ("no_dq", {"MIO_BT_DQ": "0"}),
                  ("no_q6loop", {"MIO_MMQ_LOOP_Q6": "0"}), ("no_qf", {"MIO_BT_QF": "0"})):
    t0 = time.time()
    p = subprocess.run([BIN] + common + ["--batch", d + "/batch.txt", "-o", d + f"/b_{name}.wav", "--gpus", "1"],
                       capture_output=True, text=True, timeout=100, env=dict(os.environ, **env))
    print(name, "rc", p.returncode, "s %.1f" % (time.time() - t0), p.stderr[-600:].replace("\n", " | "), flush=True)
