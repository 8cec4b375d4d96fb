"""Average every PMC counter per dispatch of the kernels whose name contains a substring,
over one or more rocprofv3 counter_collection.csv files (one per --pmc pass); or, with
--l2, each busy kernel's L2 hit rate from a TCC_HIT_sum / TCC_MISS_sum pass. Not part of
the product.   python tools/pmc_table.py <substring> <csv> [<csv> ...]
               python tools/pmc_table.py --l2 <csv>"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(paths, match):
    """{kernel: {counter: {dispatch: value}}} for the kernels match() accepts"""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for p in paths:
        for r in csv.DictReader(open(p)):
            if match(r["Kernel_Name"]):
                per[r["Kernel_Name"][:70]][r["Counter_Name"]][int(r["Dispatch_Id"])] += \
                    float(r["Counter_Value"])
    return per


mean = lambda d: sum(d.values()) / len(d)  # noqa: E731


def main():
    if sys.argv[1] == "--l2":
        for k, v in per_dispatch(sys.argv[2:], lambda n: True).items():
            if "TCC_HIT_sum" not in v:
                continue
            h, m = mean(v["TCC_HIT_sum"]), mean(v["TCC_MISS_sum"])
            if h + m > 5e7:
                print(f"{k:70s} n={len(v['TCC_HIT_sum'])} hit {h:.3e} miss {m:.3e} rate {h / (h + m):.3f}")
        return
    sub, out = sys.argv[1], {}
    for p in sys.argv[2:]:   # one file at a time: a counter's dispatches are that pass's
        for v in per_dispatch([p], lambda n: sub in n).values():
            for name, d in v.items():
                out[name] = mean(d)
                out.setdefault("_dispatches", len(d))
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
