"""Does the slow gather line (functional.SLOW_GATHER_LINE) cost the GAT aggregation too? Config
5's 2M x 2M power-law slice (GAT d = 64, 4 heads, K = 3) through gat_forward_dist on one GPU,
with the tables its kernels gather from compact (the projection [N, 72], the layer outputs
[N, 64]) vs placed (512-B rows, 1-KB aligned: no gathered line at byte 384). Median ms per
forward over 10 (HIP events) and a SHA-256 of the output bits per case."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
import bench_configs as bc  # noqa: E402
from src import ops  # noqa: E402
from src.models.baselines.gat import GATLayer  # noqa: E402
from src.ops import functional as F  # noqa: E402
from src.ops.distributed import DistributedGraph, gat_forward_dist  # noqa: E402

dev = torch.device("cuda", 0)
shape = (2_000_000, 2_000_000, 50_000_000)
g = bc.powerlaw_graph(*shape, 0.9, 0, 16)
m = bc.config5_model(shape, dev)
dg = DistributedGraph(g, 0, 1, dev)
x0p = dg.pad_table(m._initial_table())
orig_project = GATLayer._project
orig_agg = ops.gat_aggregate


def placed_project(x, w):
    p = w.shape[0]
    if x.is_cuda and F.rows_gemm_supported(x.shape[1], p) and p <= 128:
        out = F.hop_table(x.shape[0], p, device=x.device, layout=(128, 0))
        return F.rows_gemm(x if F._rows_view_ok(x) else x.contiguous(), w.t(), out=out)
    return orig_project(x, w)


def placed_agg(adj, h, s_self, s_neigh, heads, o_dim, *a, **kw):
    width = o_dim if kw.get("mean_heads") else heads * o_dim
    if kw.get("out") is None and not (kw.get("epi", 0) & F.EPI_NO_Y) and width == 64:
        kw["out"] = F.hop_table(adj.n_rows, 64, device=h.device, layout=(128, 0))
    return orig_agg(adj, h, s_self, s_neigh, heads, o_dim, *a, **kw)


with torch.no_grad():
    for policy in ("compact", "placed", "compact", "placed"):
        GATLayer._project = staticmethod(placed_project if policy == "placed" else orig_project)
        ops.gat_aggregate = placed_agg if policy == "placed" else orig_agg
        for _ in range(2):
            out = gat_forward_dist(dg, m, x0p)
        ev = []
        for _ in range(10):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = gat_forward_dist(dg, m, x0p)
            e.record()
            ev.append((s, e))
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e in ev]
        print(json.dumps({"policy": policy, "ms_median": float(np.median(ms)),
                          "ms": [round(v, 3) for v in ms],
                          "out_sha256": hashlib.sha256(out.contiguous().cpu().numpy().tobytes())
                          .hexdigest()[:16]}), flush=True)
