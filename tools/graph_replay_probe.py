"""the profiler's graph-replay fault with nothing of the decode step in the
process — a graph of one empty kernel (mio_hip_debug_graph_replay) replayed 30,000 times.
Run under `rocprofv3 --kernel-trace`; prints the per-replay wall time as it goes.
usage: python3 tools/graph_replay_probe.py [replays] [nodes]"""
import faulthandler
import os
import sys

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "miotts-llama.cpp_amd", "python"))
import miotts_amd as m  # noqa: E402

replays = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = m.Device(0)
done = 0
while done < replays:
    n = min(5000, replays - done)
    ms = dev.graph_replay(n, nodes)
    done += n
    print(f"{done} replays of a {nodes}-node graph: {ms * 1e3 / n:.2f} us per replay", flush=True)
dev.close()
print("done", flush=True)
