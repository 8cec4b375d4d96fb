"""Inside the heavy-row kernel on config 2's operand: per-wave timestamps (wall clock, 10 ns)
(and core cycles) of the first 8 heavy workgroups — the longest row's feature slices — at entry, after the
loaders' prologue, after each round's work and after each round's barrier, and at the
consumer's store. Needs a trace build:

    bash tools/build_variant.sh tools/ab/htrace.so spmm.hip -DGNNREC_HEAVY_TRACE=1
    GNNREC_LIB=tools/ab/htrace.so python tools/exp_heavy_trace.py
"""
import ctypes as C
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.ops import CsrGraph  # noqa: E402
from src.ops import _lib  # noqa: E402
from src.ops import functional as F  # noqa: E402

BLOCKS, WAVES, EVENTS = 8, 8, 64
dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
deg = g.row_ptr[1:] - g.row_ptr[:-1]
L = _lib.lib()
L.gnnrec_debug_heavy_trace.argtypes = [C.c_void_p]
buf = torch.zeros(2 * BLOCKS * WAVES * EVENTS, dtype=torch.int64, device=dev)
assert L.gnnrec_debug_heavy_trace(C.c_void_p(buf.data_ptr())) == 0


def sub_of(keep):
    rows = torch.nonzero(keep).flatten()
    cnt = deg[rows]
    rp = torch.zeros(rows.numel() + 1, dtype=torch.int64, device=dev)
    rp[1:] = torch.cumsum(cnt, 0)
    off = torch.repeat_interleave(g.row_ptr[rows] - rp[:-1], cnt)
    idx = torch.arange(int(rp[-1]), device=dev, dtype=torch.int64) + off
    return CsrGraph(rp, g.col[idx].contiguous(), g.val[idx].contiguous(), (rows.numel(), g.shape[1]))


x = torch.randn(g.shape[1], 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
bands = {"top1": deg == deg.max(), "heavy_gt128": deg > 128, "all": deg >= 0}
for name, keep in bands.items():
    sg = g if name == "all" else sub_of(keep)
    y = torch.empty(sg.n_rows, 64, device=dev)
    for _ in range(2000):   # ~0.1 s of back-to-back hops first (clocks up)
        F.spmm_into(sg, x, y)
    buf.zero_()
    F.spmm_into(sg, x, y)
    torch.cuda.synchronize()
    t, cy = buf.view(2, BLOCKS, WAVES, EVENTS).cpu()
    t0 = int(t[t > 0].min()) if bool((t > 0).any()) else 0
    for b in range(BLOCKS):
        for w in (0, 1, 7):
            ev, cv = t[b, w], cy[b, w]
            cv = cv[ev > 0]
            ev = ev[ev > 0]
            if ev.numel() == 0:
                continue
            print(json.dumps({"band": name, "block": b, "wave": w,
                              "us": [round((int(v) - t0) / 100.0, 2) for v in ev],
                              "kcycles": [round((int(v) - int(cv[0])) / 1000.0, 1) for v in cv]}),
                  flush=True)
