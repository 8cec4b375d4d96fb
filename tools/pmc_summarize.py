"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into the per-launch HBM
traffic figure bench.py reports as roofline.traffic.

    python tools/pmc_summarize.py <fetch_csv> <write_csv> <out_json> [kernel_substring]
                                  [bench_json_of_the_pmc_run]

The bench JSON line of the profiled run carries roofline.kernel_key (SHA-256 of the hop
kernel's sources and plan parameters); it is stored in the summary, and bench.py reports the
summary's traffic only while its own kernel_key matches.

Counters are collected in two separate passes (MI355X_MICROARCH.md § rocprofv3 PMC slots:
FETCH_SIZE and WRITE_SIZE do not fit one TCC pass). Both are in KiB. gfx950 correction
(MI355X_MICROARCH.md § HBM): FETCH_SIZE reports exactly half of the bytes of wide streaming
reads (128-B requests tallied as 64 B), so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is
exact (calibrated here: the first hop writes y + acc = 2 * 512 MB and reads 1,000,000 KiB).
Both count L2 -> fabric requests, i.e. they include Infinity Cache hits.
"""
import csv
import json
import sys
from statistics import mean


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and kernel in row["Kernel_Name"]:
                vals[int(row["Dispatch_Id"])] = vals.get(int(row["Dispatch_Id"]), 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "spmm_vec_kernel"
    key = None
    if len(sys.argv) > 5:
        for line in open(sys.argv[5]):
            if line.startswith("{"):
                key = json.loads(line)["roofline"].get("kernel_key")
    fetch = per_dispatch(fetch_csv, "FETCH_SIZE", kernel)
    write = per_dispatch(write_csv, "WRITE_SIZE", kernel)
    rd = [2.0 * v * 1024 for v in fetch]
    wr = [v * 1024 for v in write]
    res = {
        "kernel": kernel,
        "kernel_key": key,
        "launches": len(fetch),
        "fetch_size_kib_per_launch": fetch,
        "write_size_kib_per_launch": write,
        "read_bytes_per_launch_corrected": mean(rd),
        "write_bytes_per_launch": mean(wr),
        "hbm_bytes_per_launch": mean(rd) + mean(wr),
        "correction": "read = 2 * FETCH_SIZE KiB (gfx950 half-count of 128-B requests); "
                      "write = WRITE_SIZE KiB; both include Infinity Cache hits",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if "per_launch" in k and not isinstance(v, list)}))


if __name__ == "__main__":
    main()
