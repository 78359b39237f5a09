"""The CPU baseline run in full (no extrapolation): one whole bench utterance through the C
oracle on the host's cores — the chat-template prompt prefilled token by token, 700 sampled
speech tokens (temperature 0.8, the bench's allow range), MioCodec + iSTFT of the 700 codes —
timed end to end. bench.py's cpu_baseline samples the same work and extrapolates, so that the
default bench stays within minutes; this run checks that extrapolation.
usage: python tools/cpu_full.py [threads] [preset] [tokens]  ->  one JSON line"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import miotts_amd as m  # noqa: E402
import pyoracle  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
preset = int(sys.argv[2]) if len(sys.argv) > 2 else 3
tokens = int(sys.argv[3]) if len(sys.argv) > 3 else 700
sys.path.insert(0, REPO)
import bench  # noqa: E402  (the bench's prompt and synthetic files)

llm_path, codec_path, voice_path = bench.ensure_files(os.environ.get("MIOTTS_BENCH_DIR", "/tmp/miotts_bench"),
                                                      preset, 0, lambda: None)
prompt = bench.prompt_tokens(bench.PROMPT)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
pyoracle.set_threads(threads)
o = pyoracle.Llm(llm_path, len(prompt) + tokens + 8)
c = pyoracle.Codec(codec_path)
emb = m.read_voice(voice_path)
o.eval(prompt[0], 0)  # page the weights in (not timed)
o.reset()
t0 = time.perf_counter()
ids = o.generate(prompt, tokens, 0.8, 42, allow=allow)
t1 = time.perf_counter()
codes = np.asarray(ids, np.int64) - m.SYNTH_SPEECH0
pcm = c.decode_pcm(codes, emb)
t2 = time.perf_counter()
audio = pcm.size / 44100.0
print(json.dumps({"metric": "CPU oracle, one whole utterance", "value": round(audio / (t2 - t0), 4),
                  "unit": "x realtime (audio s / wall s)", "cores": threads, "kind": "port",
                  "preset": preset, "prompt_tokens": len(prompt), "tokens": len(ids),
                  "llm_s": round(t1 - t0, 3), "llm_ms_per_token": round((t1 - t0) * 1e3 / (len(prompt) + len(ids)), 2),
                  "codec_istft_s": round(t2 - t1, 3), "audio_s": round(audio, 3), "wall_s": round(t2 - t0, 3)}),
      flush=True)
