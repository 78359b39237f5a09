"""HBM traffic per launch of the decode-step kernels from rocprofv3 PMC runs.

Two counter passes (gfx950 cannot fit FETCH_SIZE and WRITE_SIZE in one), each on a short
eager run of bench.py (MIO_NO_GRAPH=1: rocprofv3 tracing of graph replays is unreliable on
ROCm 7.2 here), e.g. on the GPU box:
    MIO_NO_GRAPH=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc \\
        -o fetch -- python3 bench.py --steps 1 --warmup 0 --tokens 64 --no-cpu-baseline
    ... the same with --pmc WRITE_SIZE -o write
then here:  python tools/pmc_traffic.py gpurun_out/pmc/fetch_counter_collection.csv \\
                gpurun_out/pmc/write_counter_collection.csv > profiles/pmc_traffic.json
Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) counts exactly half the
bytes of wide coalesced streaming reads on gfx950 -> x2; WRITE_SIZE (KB) is exact for
16-B-per-lane stores. Infinity-Cache hits are counted, not excluded.
"""
import csv
import json
import re
import sys
from collections import defaultdict

KERNELS = ["k_attn_in", "k_attention", "k_attn_out", "k_att_o", "k_layer_att", "k_ffn", "k_ffn_in", "k_ffn_down", "k_lm_head", "k_sample"]


def base(name):
    # demangled ("mio::(anonymous namespace)::k_ffn_in<1, 12>(...)") or mangled
    # ("_ZN3mio12_GLOBAL__N_18k_ffn_inILi1ELi12EEEv...") kernel names
    for k in KERNELS:
        if re.search(r"(?<![A-Za-z_])" + k + r"(?![a-z_])", name) or re.search(r"\d" + k + r"I", name):
            return k
    return None


def load(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            k = base(r.get("Kernel_Name", ""))
            if k:
                acc[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    fetch, nf = load(sys.argv[1], "FETCH_SIZE")
    write, _ = load(sys.argv[2], "WRITE_SIZE") if len(sys.argv) > 2 else ({}, {})
    per_launch = {}
    for k in fetch:
        per_launch[k] = int(round(fetch[k] * 1024 * 2 + write.get(k, 0.0) * 1024))
    out = {
        "preset": int(sys.argv[3]) if len(sys.argv) > 3 else 3,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace only), eager "
                  "launches; bytes = 2 * FETCH_SIZE[KB] * 1024 (gfx950 streaming-read correction) + "
                  "WRITE_SIZE[KB] * 1024; mean per dispatch",
        "dispatches": nf,
        "fetch_kb_mean": {k: round(v, 1) for k, v in fetch.items()},
        "write_kb_mean": {k: round(v, 1) for k, v in write.items()},
        "per_launch_bytes": per_launch,
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
