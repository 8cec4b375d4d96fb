"""hipGraph capture of the fused LightGCN propagation (config 2 shape): eager vs replay."""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.ops import functional as F  # noqa: E402


def t_ms(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
x = torch.randn(g.shape[0], 64, device=dev) * 0.1
eager = t_ms(lambda: F.lightgcn_forward(g, x, 3))
ref, _ = F.lightgcn_forward(g, x, 3)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        F.lightgcn_forward(g, x, 3)
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out, _ = F.lightgcn_forward(g, x, 3)
graph.replay()
torch.cuda.synchronize()
same = torch.equal(out, ref)
replay = t_ms(graph.replay)
print(json.dumps({"eager_ms": eager, "graph_replay_ms": replay, "bit_identical": same}))
