"""Graph-mode decode under rocprofv3: a short generate on the tiny model
with the step graphs replayed (no MIO_NO_GRAPH). Run as
  rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/rocprof_graph_repro.py [preset] [tokens] [maps_out]"""
import faulthandler
import os
import sys
import tempfile

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

preset = int(sys.argv[1]) if len(sys.argv) > 1 else 0
n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
d = tempfile.mkdtemp()
dev = m.Device(0)
g = m.Llm(dev, m.synth_llm(os.path.join(d, "l.gguf"), preset, 1), 512)
allow = (m.SYNTH_SPEECH0, m.SYNTH_SPEECH0 + 12800)
if len(sys.argv) > 3:  # address map of this process (symbolizing a native crash offline)
    with open("/proc/self/maps") as f, open(sys.argv[3], "w") as o:
        o.write(f.read())
for rep in range(2):
    t = g.generate([256, 257, 65, 66, 258, 257], n, 0.8, 42 + rep, allow=allow, check_interval=20)
    print("rep", rep, "tokens", len(t), flush=True)
g.close()
dev.close()
print("done", flush=True)
