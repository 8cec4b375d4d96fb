"""Row stride vs the slow gather line (tools/exp_hop_offset2.py: a 128-B line at byte 384 of a
1-KB window): the G100M d = 64 hop (HIP events, median of 10) on column block 0 of [N, ld]
tables, ld = 64 / 128 / 256 floats, and ld = 128 with a 256-B base shift (half the rows'
second line at the slow offset). ld = 64 runs first and last (drift check)."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
n = g.shape[0]
gen = torch.Generator(dev).manual_seed(0)


def hop_ms(x, reps=12):
    work = torch.empty(n, x.shape[1], device=dev)
    plan = F.tiled_plan_for(g, x)
    assert plan is not None
    ev = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        F.spmm_tiled_into(g, x, work, plan)
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    return float(np.median([s.elapsed_time(e) for s, e in ev[2:]]))


def table(ld, shift_floats):
    buf = torch.randn(n * ld + shift_floats, device=dev, generator=gen) * 0.1
    return buf[shift_floats:].view(n, ld)


for ld, shift in ((64, 0), (128, 0), (256, 0), (128, 64), (64, 0)):
    T = table(ld, shift)
    x = T[:, :64]
    print(json.dumps({"ld": ld, "shift_B": 4 * shift, "d": 64,
                      "addr_mod_1k": x.data_ptr() % 1024, "ms": hop_ms(x)}), flush=True)
    del T, x
