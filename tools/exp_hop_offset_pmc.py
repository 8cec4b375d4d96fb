"""Counters for the slow gather line: the G100M d = 32 hop gathering the 32-column slice at
byte 256 (fast) and at byte 384 (slow) of 1-KB rows, 3 launches each, in that order, for a
per-launch / per-L2-channel PMC pass (rocprofv3 --pmc TCC_HIT TCC_MISS)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
n = g.shape[0]
T = torch.randn(n, 256, device=dev, generator=torch.Generator(dev).manual_seed(0)) * 0.1
work = torch.empty(n, 32, device=dev)
for col in (64, 96):
    x = T[:, col:col + 32]
    plan = F.tiled_plan_for(g, x)
    for _ in range(3):
        F.spmm_tiled_into(g, x, work, plan)
    torch.cuda.synchronize()
    print(f"col {col} done", flush=True)
