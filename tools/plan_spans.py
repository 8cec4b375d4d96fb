"""Column spans of the G100M column-ordered plan's chunks (host planner, CPU only): can a slot
word drop to 3 bytes with a per-chunk (or per-stream) column base?

    python tools/plan_spans.py > profiles/r05/plan_spans_g100m.json
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402

g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, bench.host_threads())
plan = g.tiled_plan(rows_per_block=1117, planner="host")
R = plan["rows_per_block"]
slot = plan["slot"].numpy().view(np.uint32).reshape(-1, 64)   # chunk-major: lane = 8 stream + step
row, col = slot & 2047, (slot >> 11).astype(np.int64)
real = row < R
BIG = np.iinfo(np.int64).max


def spans(c, r, axis):
    lo = np.where(r, c, BIG).min(axis)
    hi = np.where(r, c, -1).max(axis)
    return (hi - lo)[hi >= 0]


chunk = spans(col, real, 1)
stream = spans(col.reshape(-1, 8, 8), real.reshape(-1, 8, 8), 2)
print(json.dumps({
    "plan": {"chunks": int(slot.shape[0]), "rows_per_block": R, "panel": plan["panel"],
             "sub_panel": plan["sub_panel"], "row_bits": 11},
    "chunk_span_below": {b: float((chunk < b).mean()) for b in (4096, 8192, 16384, 32768)},
    "stream_span_below": {b: float((stream < b).mean()) for b in (1024, 2048, 4096, 8192)},
}))
