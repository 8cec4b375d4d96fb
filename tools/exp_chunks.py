"""Row-parallel CSR hop vs column-ordered tiled hop on row slices of G100M (d=64, the full
source table): where does the tiled kernel stop paying? Row slices stand for the overlap
chunks of the sharded hop (src/ops/distributed.py). One JSON line per slice size. Not part
of the product.

    python tools/exp_chunks.py [rows ...]
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402


def timed(fn, reps=10):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
x = torch.randn(g.shape[0], 64, device=dev, generator=torch.Generator(dev).manual_seed(0)) * 0.1
sizes = [int(v) for v in sys.argv[1:]] or [15625, 31250, 62500, 125000, 250000, 500000]
for n in sizes:
    s = g.row_slice(0, n)
    y1 = torch.empty((n, 64), device=dev)
    y2 = torch.empty((n, 64), device=dev)
    F.TILED_HOP = False
    t_csr = timed(lambda: F.spmm_into(s, x, y1))
    R = F._tiled_rows_per_block(n, dev)
    plan = s.tiled_plan(rows_per_block=R)
    t_tiled = timed(lambda: F.spmm_tiled_into(s, x, y2, plan))
    t_tiled0 = timed(lambda: F.spmm_tiled_into(s, x, y2, plan, meet_us=0))
    print(json.dumps({"rows": n, "nnz": s.nnz, "R": R, "csr_ms": t_csr, "tiled_ms": t_tiled,
                      "tiled_no_meet_ms": t_tiled0,
                      "bit_exact": bool(torch.equal(y1, y2))}), flush=True)
    F.TILED_HOP = True
    s._plans.clear()
