"""Rows per block on the bench path with placed tables (as tools/exp_hop_tables.py): G100M
LightGCN K = 3 d = 64 with the column-ordered plan capped at 1279 rows (the default: 1117
rows, 7 passes per slice) vs 977 rows (8 passes), alternating, median ms per step of 10."""
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
default = F.TILED_MAX_ROWS
for cap in (default, 977, default, 977, default, 977):
    F.TILED_MAX_ROWS = cap
    lay = bench.Layout(full, 0, 1, dev, 64, 1, "p2p").prepare(x0, dev)
    R = F._tiled_rows_per_block(lay.dg.shard.n_rows, dev)
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
    print(json.dumps({"cap": cap, "rows_per_block": R, "ms_per_step_median": float(np.median(ms)),
                      "ms": [round(v, 3) for v in ms],
                      "out_sha256": hashlib.sha256(out.contiguous().cpu().numpy().tobytes())
                      .hexdigest()[:16]}), flush=True)
    lay.release()
    del lay, out
    torch.cuda.empty_cache()
