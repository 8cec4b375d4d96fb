"""GAT training step on a power-law operand (the native training kernels walk each
row, and in the backward's column pass each column, serially in one lane group — what does
that cost on config 5's degree distribution?). One forward + backward of the config-5 model
(d = 64, 4 heads, K = 3, attention dropout) with loss = sum(out * R), on the 2M x 2M Zipf-0.9
graph (93M nnz, max degree ~4e5) and on a capped-degree graph of the same size for contrast.
Median ms of --reps steps; run under rocprofv3 --kernel-trace to split the kernels.

    python tools/exp_gat_train.py [--shape 2000000 2000000 50000000] [--reps 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
from bench_configs import powerlaw_graph  # noqa: E402
from src.models import GAT  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", type=int, nargs=3, default=[2_000_000, 2_000_000, 50_000_000])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--dropout", type=float, default=0.1)
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = powerlaw_graph(*a.shape, 0.9, 0, 16, device=dev)
deg = g.row_ptr[1:] - g.row_ptr[:-1]
torch.manual_seed(0)
m = GAT(a.shape[0], a.shape[1], 64, 3, 4, a.dropout, 0.2, 0.1).to(dev).train()
assert all(layer.train_ok(g) for layer in m.layers)
R = torch.randn(g.shape[0], 64, device=dev, generator=torch.Generator(device=dev).manual_seed(1))


def step():
    m.zero_grad(set_to_none=True)
    u, i = m(g)
    loss = (torch.cat([u, i]) * R).sum()
    loss.backward()
    return loss


step()
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    loss = step()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
ts.sort()
print(json.dumps({"case": "gat_train_step", "shape": a.shape, "nnz": g.nnz,
                  "max_degree": int(deg.max()), "dropout": a.dropout,
                  "ms_median": ts[len(ts) // 2], "ms_samples": ts,
                  "loss_finite": bool(torch.isfinite(loss).item())}), flush=True)
