"""Config 6 (G100M LightGCN BPR train step) for rocprofv3: 5 steps after 2 warm-up steps."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.models import LightGCN  # noqa: E402
from src.training import BPRLoss, DeviceSampler, make_adam, train_step  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
rp = g.row_ptr.numpy()
users = np.repeat(np.arange(1_000_000), np.diff(rp[:1_000_001]))
items = g.col.numpy()[:rp[1_000_000]] - 1_000_000
g1 = g.to(dev)
torch.manual_seed(0)
m = LightGCN(1_000_000, 1_000_000, 64, 3, 0.1).to(dev).train()
samp = DeviceSampler(users, items, 1_000_000, 2048, 1, dev, seed=0)
opt = make_adam(m.parameters(), 1e-3, 1e-4, dev)
for _ in range(7):
    train_step(m, g1, *samp(), opt, BPRLoss(), 1.0)
torch.cuda.synchronize()
