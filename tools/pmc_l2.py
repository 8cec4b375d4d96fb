"""Per-kernel L2 hit rate from a rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum counter CSV."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "TCC_HIT_sum" not in v:
        continue
    h = sum(v["TCC_HIT_sum"]) / len(v["TCC_HIT_sum"])
    m = sum(v["TCC_MISS_sum"]) / len(v["TCC_MISS_sum"])
    if h + m > 5e7:
        print(f"{k:70s} n={len(v['TCC_HIT_sum'])} hit {h:.3e} miss {m:.3e} rate {h / (h + m):.3f}")
