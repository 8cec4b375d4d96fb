"""A/B of the hop-table layout (functional.HOP_TABLE_LAYOUT) on the bench's own path: G100M
LightGCN K = 3 through bench.Layout + lightgcn_propagate_dist on one GPU (x0, y1, y2 tables
compact vs placed), d = 32 / 64 / 128 (d = 128 placed: 1-KB rows starting at byte 512).
Per case: median ms per K = 3 step over 10 (HIP events) and a SHA-256 of the output bits."""
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
x0_all = torch.randn(full.shape[0], 128, generator=torch.Generator().manual_seed(0)) * 0.1
default = dict(F.HOP_TABLE_LAYOUT)
for d in (64, 32, 128):
    for policy in ("compact", "placed", "compact"):
        F.HOP_TABLE_LAYOUT = {} if policy == "compact" else {**default, 128: (256, 512)}
        lay = bench.Layout(full, 0, 1, dev, d, 1, "p2p").prepare(x0_all[:, :d].contiguous(), dev)

        def step():
            return lightgcn_propagate_dist(lay.dg, lay.x0_pad, 3, work=lay.work)

        for _ in range(2):
            out = step()
        ev = []
        for _ in range(10):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = step()
            e.record()
            ev.append((s, e))
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e in ev]
        print(json.dumps({"d": d, "policy": policy, "x0_ld": lay.x0_pad.stride(0),
                          "ms_per_step_median": float(np.median(ms)),
                          "ms": [round(v, 3) for v in ms],
                          "out_sha256": hashlib.sha256(out.contiguous().cpu().numpy().tobytes())
                          .hexdigest()[:16]}), flush=True)
        lay.release()
        del lay, out
        torch.cuda.empty_cache()
F.HOP_TABLE_LAYOUT = default
