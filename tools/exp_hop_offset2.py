"""Map of the column-block effect found by tools/exp_hop_offset.py (the G100M hop gathering
the 64-column block at byte offset 256 of 1-KB rows runs ~4.0 ms, the others ~3.33 ms):
hop time (HIP events, median of 10) for
  A  d = 32 slices at every 128-B line offset of a [N, 256] table;
  B  d = 64 blocks of a [N, 256] table whose base is shifted by 512 B (a contiguous tensor
     with a storage offset);
  C  the same with a 128-B shift;
  D  d = 64 blocks of a [N, 264] table (1056-B rows)."""
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


T = table(256, 0)
for c in range(0, 256, 32):
    print(json.dumps({"case": "A", "ld": 256, "shift_B": 0, "d": 32, "col": c,
                      "addr_mod_1k": (T[:, c:].data_ptr()) % 1024,
                      "ms": hop_ms(T[:, c:c + 32])}), flush=True)
del T
for case, ld, shift in (("B", 256, 128), ("C", 256, 32), ("D", 264, 0)):
    T = table(ld, shift)
    for k in range(4):
        x = T[:, 64 * k:64 * k + 64]
        print(json.dumps({"case": case, "ld": ld, "shift_B": 4 * shift, "d": 64, "col": 64 * k,
                          "addr_mod_1k": x.data_ptr() % 1024, "ms": hop_ms(x)}), flush=True)
    del T
