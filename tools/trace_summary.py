"""Summarise a rocprofv3 kernel_trace.csv: per dispatch (name, start, end) relative to the
first, and for consecutive dispatches whether they overlapped. Not part of the product."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keep = [r for r in rows if any(k in r["Kernel_Name"] for k in sys.argv[2].split(","))]
t0 = int(keep[0]["Start_Timestamp"])
for r in keep[-int(sys.argv[3]) if len(sys.argv) > 3 else 0:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'][:40]:40s} q={r.get('Queue_Id', '?'):>3} start={s / 1e3:10.1f}us "
          f"end={e / 1e3:10.1f}us dur={(e - s) / 1e3:7.1f}us")
