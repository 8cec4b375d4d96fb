"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel time over the last 1/`parts` of the
dispatches (one step of a run of `parts` equal steps), and the span it covers.
usage: python tools/trace_tail.py <kernel_trace.csv> [parts]"""
import collections
import csv
import sys

rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
               for r in csv.DictReader(open(sys.argv[1]))), key=lambda t: t[1])
parts = int(sys.argv[2]) if len(sys.argv) > 2 else 1
last = rows[-(len(rows) // parts):]
tot, cnt = collections.defaultdict(float), collections.Counter()
for name, s, e in last:
    tot[name[:90]] += (e - s) / 1e6
    cnt[name[:90]] += 1
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:40]:
    print(f"{v:9.3f} ms {cnt[k]:5d}  {k}")
print(f"busy {sum(tot.values()):.3f} ms, span {(last[-1][2] - last[0][1]) / 1e6:.3f} ms, "
      f"{len(last)} dispatches")
