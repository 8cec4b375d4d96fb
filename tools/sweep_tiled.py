"""Sweep the column-ordered hop's plan shape on G100M d=64 (rows per block, panel, sub-panel):
per shape, build the plan, time one hop with HIP events (median of N), and check its bits
against the row-parallel CSR kernel. One JSON line per shape (not part of the product).

    python tools/sweep_tiled.py [--d 64] R:PANEL:SUB[:MEET_US] [...]
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
from src.ops import graph as G  # noqa: E402

if __import__("os").environ.get("TILED_FACTOR") == "0":   # explicit-value plans (A/B)
    G.TILED_FACTOR = False

args = sys.argv[1:]
D, LDX, FOLD = 64, None, 0
while args and args[0] in ("--d", "--ldx", "--fold"):
    if args[0] == "--d":
        D = int(args[1])
    elif args[0] == "--ldx":
        LDX = int(args[1])
    else:   # timing floor: every gather folded into the first FOLD bytes of x (L2-resident)
        FOLD = int(args[1])
    args = args[2:]
LDX = LDX or D
dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
x = (torch.randn(g.shape[0], LDX, device=dev, generator=torch.Generator(dev).manual_seed(0))
     * 0.1)[:, :D]
ref = torch.empty(x.shape, device=dev)
F.TILED_HOP = False
F.spmm_into(g, x, ref)
torch.cuda.synchronize()
y = torch.empty(x.shape, device=dev)
for spec in args:
    R, panel, sub, *rest = (int(v) for v in spec.split(":"))
    meet = rest[0] if rest else F.TILED_MEET_US
    t0 = time.time()
    plan = g.tiled_plan(rows_per_block=R, panel=panel, sub_panel=sub)
    t_plan = time.time() - t0
    if FOLD:
        plan = dict(plan)
        rows = FOLD // (4 * LDX)     # slot words re-pointed into the first FOLD bytes
        w = plan["slot"].long() & 0xFFFFFFFF
        plan["slot"] = ((torch.remainder(w >> 11, rows) << 11) | (w & 2047)).int()
        hdr = plan["hdr"].clone().view(-1, 4)
        hdr[:, 3] = 0                                   # panel base
        plan["hdr"] = hdr.view(-1)
    times = []
    for _ in range(12):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        F.spmm_tiled_into(g, x, y, plan, meet_us=meet)
        b.record()
        torch.cuda.synchronize()
        times.append(a.elapsed_time(b))
    exact = bool(torch.equal(y.view(torch.int32), ref.view(torch.int32)))
    times.sort()
    print(json.dumps({"d": D, "ldx": LDX, "fold": FOLD, "R": R, "panel": panel, "sub_panel": sub, "meet_us": meet,
                      "n_blocks": plan["n_blocks"], "factored": "cls" in plan,
                      "pad": plan["n_slots"] / g.nnz - 1, "ms_median": times[len(times) // 2],
                      "ms_min": times[0], "bit_exact": exact, "plan_s": round(t_plan, 1)}),
          flush=True)
    g._plans.pop(("tiled", R, panel, sub), None)
    del plan
