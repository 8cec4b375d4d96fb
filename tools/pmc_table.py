"""Average every PMC counter per dispatch of the kernels whose name contains a substring,
over one or more rocprofv3 counter_collection.csv files (one per --pmc pass). Not part of
the product.   python tools/pmc_table.py <substring> <csv> [<csv> ...]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    sub, paths = sys.argv[1], sys.argv[2:]
    out = {}
    for p in paths:
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(p)):
            if sub in r["Kernel_Name"]:
                per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for name, d in per.items():
            out[name] = sum(d.values()) / len(d)
            out.setdefault("_dispatches", len(d))
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
