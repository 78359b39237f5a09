"""MFMA-busy share of the codec kernels from one rocprofv3 PMC pass.

On the GPU box (kernel trace only beside the counters; tools/codec_trace.py decodes T = 700
twice, the second decode is used):
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \\
        -d gpurun_out/pmcc -o codec -- python3 tools/codec_trace.py
then:  python tools/pmc_codec.py gpurun_out/pmcc/.../codec_counter_collection.csv > profiles/pmc_codec_mfma.json

SQ_VALU_MFMA_BUSY_CYCLES counts the cycles the matrix pipes are busy, summed over the SIMDs
(MI355X_MICROARCH.md: 32 per 32x32x16 bf16 MFMA; a 32x32x2 f32 MFMA = 4,096 FLOP at 64
FLOP/clk/SIMD = 64 cycles). GRBM_GUI_ACTIVE counts GPU-busy cycles summed over the 8 XCDs.
mfma_busy_frac = sum(MFMA busy) / (sum(GRBM_GUI_ACTIVE) / 8 x 1024 SIMDs) over the codec's
dispatches: the share of the chip's matrix-pipe cycles the codec kept busy while it ran,
i.e. the achieved fraction of the f32 MFMA peak at the clock the chip held.
"""
import csv
import json
import sys
from collections import defaultdict

N_SIMD = 256 * 4
CODEC = ("gemm_f32", "gemm_x3", "conv_f16", "band_attention", "rownorm", "gn_partial", "gn_final", "gn_apply", "gn_fused", "cond_gemv",
         "embed_kernel", "istft_fused")


def kind(name):
    for k in CODEC:
        if k in name:
            return k
    return None


def main(path):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    ds = sorted(d for d in per if kind(names[d]))
    ds = ds[len(ds) // 2:]  # the second of the two decodes
    by = defaultdict(lambda: [0.0, 0.0, 0])
    for d in ds:
        k = kind(names[d])
        by[k][0] += per[d]["SQ_VALU_MFMA_BUSY_CYCLES"]
        by[k][1] += per[d]["GRBM_GUI_ACTIVE"]
        by[k][2] += 1
    codec = [k for k in by if k != "istft_fused"]
    busy = sum(by[k][0] for k in codec)
    active = sum(by[k][1] for k in codec)
    out = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, tools/codec_trace.py (T=700)",
           "mfma_busy_frac": round(busy / (active / 8 * N_SIMD), 4) if active else None,
           "by_kernel": {k: {"dispatches": v[2], "mfma_busy_frac": round(v[0] / (v[1] / 8 * N_SIMD), 4) if v[1] else None}
                         for k, v in sorted(by.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
