"""Workload for the rocprofv3 PMC passes (tools/pmc_traffic.py): a few eager decode steps
of the 1.7B preset at positions ~400 (mid-utterance; PMC collection serializes every
dispatch, so the bench's ~100k dispatches are far too many). Run with MIO_NO_GRAPH=1 under
rocprofv3 --pmc ... --kernel-trace -- python3 tools/pmc_run.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

path = "/tmp/miotts_bench/llm_preset3.gguf"
os.makedirs(os.path.dirname(path), exist_ok=True)
if not os.path.exists(path):
    m.synth_llm(path + ".tmp", 3, 1)
    os.replace(path + ".tmp", path)
dev = m.Device(0)
llm = m.Llm(dev, path, 2048)
# a 400-token prompt goes through the batched prefill (k_pf_* kernels, not counted below),
# then PMC_TOKENS decode steps run at positions 399.. (mid-utterance attention traffic)
prompt = [256, 257] + [65 + (i * 7) % 26 for i in range(396)] + [258, 257]
toks = llm.generate(prompt, int(os.environ.get("PMC_TOKENS", "8")), 0.8, 1,
                    allow=(m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800), check_interval=1000)
print("ok", len(toks), "decode positions", len(prompt) - 1, "..", len(prompt) - 2 + len(toks))
