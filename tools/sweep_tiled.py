"""Sweep the column-ordered hop's plan shape on G100M d=64 (rows per block, panel, sub-panel):
per shape, build the plan, time one hop with HIP events (median of N), and check its bits
against the row-parallel CSR kernel. One JSON line per shape (not part of the product).

    python tools/sweep_tiled.py R:PANEL:SUB [R:PANEL:SUB ...]
"""
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
x = torch.randn(g.shape[0], 64, device=dev, generator=torch.Generator(dev).manual_seed(0)) * 0.1
ref = torch.empty_like(x)
F.TILED_HOP = False
F.spmm_into(g, x, ref)
torch.cuda.synchronize()
y = torch.empty_like(x)
for spec in sys.argv[1:]:
    R, panel, sub = (int(v) for v in spec.split(":"))
    t0 = time.time()
    plan = g.tiled_plan(64, rows_per_block=R, panel=panel, sub_panel=sub)
    t_plan = time.time() - t0
    times = []
    for _ in range(12):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        F.spmm_tiled_into(g, x, y, plan)
        b.record()
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b))
    exact = bool(torch.equal(y.view(torch.int32), ref.view(torch.int32)))
    times.sort()
    print(json.dumps({"R": R, "panel": panel, "sub_panel": sub, "n_blocks": plan["n_blocks"],
                      "pad": plan["n_slots"] / g.nnz - 1, "ms_median": times[len(times) // 2],
                      "ms_min": times[0], "bit_exact": exact, "plan_s": round(t_plan, 1)}),
          flush=True)
    g._plans.pop(("tiled", 64, R, panel, sub), None)
    del plan
