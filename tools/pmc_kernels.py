"""Per-kernel sums of one rocprofv3 PMC pass (counter_collection.csv), grouped by kernel name
(template arguments kept): dispatches, and each counter summed and per dispatch.
usage: python tools/pmc_kernels.py COUNTERS.csv [name-substring ...]"""
import csv
import sys
from collections import defaultdict


def main(path, keys):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for d, cs in per.items():
        n = names[d]
        if keys and not any(k in n for k in keys):
            continue
        cnt[n] += 1
        for c, v in cs.items():
            agg[n][c] += v
    for n in sorted(agg, key=lambda n: -sum(agg[n].values())):
        print(f"{n[:70]}  x{cnt[n]}")
        for c, v in sorted(agg[n].items()):
            print(f"    {c:28s} {v:16.0f}  {v / cnt[n]:14.1f} /dispatch")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
