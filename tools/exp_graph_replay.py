"""Config 2's propagation launched eagerly vs replayed from a captured HIP graph (the six
kernel launches of a K = 3 forward as one graph launch). Same bits either way.

    python tools/exp_graph_replay.py
"""
import hashlib
import json
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
x0 = torch.randn(g.n_rows, 64, device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 0.1


def ms_of(fn, reps=200):
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


def sha(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]


with torch.no_grad():
    out_eager, _ = F.lightgcn_forward(g, x0, 3)
    t_eager = ms_of(lambda: F.lightgcn_forward(g, x0, 3))
    # capture on a side stream (torch's graph capture rule), then replay
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            F.lightgcn_forward(g, x0, 3)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out_g, _ = F.lightgcn_forward(g, x0, 3)
    graph.replay()
    torch.cuda.synchronize()
    t_graph = ms_of(graph.replay)
    print(json.dumps({"case": "config2_propagate", "eager_ms": t_eager, "graph_replay_ms": t_graph,
                      "same_bits": sha(out_eager) == sha(out_g)}), flush=True)
