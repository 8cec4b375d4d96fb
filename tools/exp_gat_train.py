"""GAT training step on a power-law operand (the native training kernels walk each
row, and in the backward's column pass each column, serially in one lane group — what does
that cost on config 5's degree distribution?). One forward + backward of the config-5 model
(d = 64, 4 heads, K = 3, attention dropout) with loss = sum(out * R), on the 2M x 2M Zipf-0.9
graph (93M nnz, max degree ~4e5) and on a capped-degree graph of the same size for contrast.
Median ms of --reps steps; run under rocprofv3 --kernel-trace to split the kernels.

    python tools/exp_gat_train.py [--shape 2000000 2000000 50000000] [--reps 5]
    python tools/exp_gat_train.py --ml1m --train-knobs 2048:1024 64:32   # ML-1M shape, split knobs
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
ap.add_argument("--ml1m", action="store_true", help="config 2's ML-1M-shaped operand instead")
ap.add_argument("--split-k-ab", action="store_true",
                help="also time the steps with the library weight-gradient GEMM (no row chunks)")
ap.add_argument("--train-knobs", nargs="*", default=[],
                help="GAT_TRAIN_HEAVY_THRESHOLD:GAT_TRAIN_SEGMENT settings to time in turn")
a = ap.parse_args()
dev = torch.device("cuda", 0)
if a.ml1m:
    from src.data.dataset import RecommendationDataset
    ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
    g = ds.get_graph(dev)
    a.shape = [ds.n_users, ds.n_items, 1_000_209]
else:
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


from src.ops import functional as F  # noqa: E402

runs = [(k, None) for k in (a.train_knobs or [None])]
if a.split_k_ab:
    runs = [(k, mn) for k in (a.train_knobs or [None]) for mn in (10 ** 12, None)]
split_default = F.LINEAR_SPLIT_K_MIN_ROWS
for knob, split_min in runs:
    F.LINEAR_SPLIT_K_MIN_ROWS = split_min if split_min is not None else split_default
    if knob is not None:
        F.GAT_TRAIN_HEAVY_THRESHOLD, F.GAT_TRAIN_SEGMENT = (int(v) for v in knob.split(":"))
    torch.manual_seed(5)
    step()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        torch.manual_seed(5)
        t0 = time.perf_counter()
        loss = step()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    grads = torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])
    ts.sort()
    print(json.dumps({"case": "gat_train_step", "shape": a.shape, "nnz": g.nnz,
                      "max_degree": int(deg.max()), "dropout": a.dropout,
                      "train_knobs": list(F.gat_train_knobs(g.n_rows)),
                      "weight_grad": "library" if split_min else "row_chunks",
                      "ms_median": ts[len(ts) // 2], "ms_samples": ts, "loss": float(loss.detach()),
                      "grad_abs_sum": float(grads.abs().sum()),
                      "loss_finite": bool(torch.isfinite(loss).item())}), flush=True)
