"""Per-dispatch view of config 2's hops (run under rocprofv3 --kernel-trace): a few forwards
of LightGCN K=3 d=64 on the ML-1M-shaped graph with the default heavy-row settings."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
x = torch.randn(g.shape[0], 64, device=dev) * 0.1
for split in (0, 2048):
    F.SPMM_HEAVY_SPLIT = split
    for _ in range(5):
        F.lightgcn_forward(g, x, 3)
    torch.cuda.synchronize()
