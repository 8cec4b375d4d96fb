"""Config 5 slice (power-law 2M x 2M GAT d=64, 4 heads, K=3) forward, for rocprofv3."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
from bench_configs import powerlaw_graph  # noqa: E402
from src.models import GAT  # noqa: E402

dev = torch.device("cuda", 0)
g = powerlaw_graph(2_000_000, 2_000_000, 50_000_000, 0.9, 0).to(dev)
torch.manual_seed(0)
m = GAT(2_000_000, 2_000_000, 64, 3, 4, 0.1, 0.2, 0.1).to(dev).eval()
with torch.no_grad():
    for _ in range(6):
        m(g)
torch.cuda.synchronize()
