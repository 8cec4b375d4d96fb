"""Run the product column-ordered hop (gnnrec_spmm_tiled_f32) on G100M d=64 a few times, for
rocprofv3 kernel-trace / PMC passes (not part of the product)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
x = torch.randn(g.shape[0], 64, device=dev) * 0.1
y = torch.empty_like(x)
plan = F.tiled_plan_for(g, x)
assert plan is not None
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    F.spmm_into(g, x, y)
torch.cuda.synchronize()
