"""Every model's eval forward on the ML-1M-shaped operand (config 2's graph: 9 746 rows, 1.0M
nnz, rows up to 5 857 neighbours) — the size of the reference's own dataset configs — with a
kernel trace under rocprofv3 if wanted: which kernels a forward launches and how long each
model takes.

    python tools/exp_ml1m_models.py
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.models import GAT, LightGCN, NGCF, NGCFGroupShuffle, OrthogonalBundleGNN  # noqa: E402

dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
nu, ni = ds.n_users, ds.n_items


def ms_of(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(5):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) / reps)
    return sorted(best)[2]


models = {
    "lightgcn": lambda: LightGCN(nu, ni, 64, 3, 0.1),
    "ngcf": lambda: NGCF(nu, ni, 64, [64, 64, 64]),
    "ngcf_gas": lambda: NGCFGroupShuffle(nu, ni, 64, [64, 64, 64]),
    "orthogonal_bundle": lambda: OrthogonalBundleGNN(nu, ni, 64, 3),
    "gat": lambda: GAT(nu, ni, 64, 3, 4),
}
for name, make in models.items():
    torch.manual_seed(0)
    m = make().to(dev).eval()
    with torch.no_grad():
        t = ms_of(lambda: m(g))
    print(json.dumps({"model": name, "ms_forward": t}), flush=True)
