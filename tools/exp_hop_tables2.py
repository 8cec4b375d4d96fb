"""d = 64 hop-table start offset A/B on the bench path (as tools/exp_hop_tables.py): 512-B
rows starting at byte 0 of a 1-KB window (lines at 0, 128, 512, 640) vs at byte 128 (lines
at 128, 256, 640, 768). The per-offset map (profiles/r04/exp_hop_line_offset.jsonl) has
offsets 0 and 128 a few % slower than 256 / 640 / 768. Median ms per K = 3 step over 10."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402
from src.ops.distributed import lightgcn_propagate_dist  # noqa: E402

dev = torch.device("cuda", 0)
full = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
x0 = torch.randn(full.shape[0], 64, generator=torch.Generator().manual_seed(0)) * 0.1
for start in (0, 128, 0, 128):
    F.HOP_TABLE_LAYOUT = {**F.HOP_TABLE_LAYOUT, 64: (128, start)}
    lay = bench.Layout(full, 0, 1, dev, 64, 1, "p2p").prepare(x0, dev)
    for _ in range(2):
        out = lightgcn_propagate_dist(lay.dg, lay.x0_pad, 3, work=lay.work)
    ev = []
    for _ in range(10):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = lightgcn_propagate_dist(lay.dg, lay.x0_pad, 3, work=lay.work)
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    ms = [s.elapsed_time(e) for s, e in ev]
    print(json.dumps({"d": 64, "start_byte": start, "x0_addr_mod_1k": lay.x0_pad.data_ptr() % 1024,
                      "ms_per_step_median": float(np.median(ms)), "ms": [round(v, 3) for v in ms],
                      "out_sha256": hashlib.sha256(out.contiguous().cpu().numpy().tobytes())
                      .hexdigest()[:16]}), flush=True)
    lay.release()
    del lay, out
    torch.cuda.empty_cache()
