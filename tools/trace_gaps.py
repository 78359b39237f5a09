"""Summarize a rocprofv3 kernel trace (CSV): per kernel family, launches, mean duration and
mean gap from the previous kernel's end (same queue), over the last `span` kernels of the
run. usage: python tools/trace_gaps.py TRACE.csv [n_last]"""
import csv
import json
import re
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
rows = rows[-n_last:]


def fam(name):
    m = re.search(r"(k_[a-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
prev_end = None
for s, e, n in rows:
    k = fam(n)
    dur[k] += e - s
    cnt[k] += 1
    if prev_end is not None:
        gap[k] += s - prev_end
    prev_end = e
span = rows[-1][1] - rows[0][0]
out = {"kernels": len(rows), "span_ms": round(span / 1e6, 3),
       "per_family": {k: {"n": cnt[k], "dur_us": round(dur[k] / cnt[k] / 1e3, 3),
                          "gap_before_us": round(gap[k] / cnt[k] / 1e3, 3)} for k in sorted(cnt)}}
print(json.dumps(out))
