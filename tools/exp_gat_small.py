"""GAT forward (eval, 4 heads, K = 3, d = 64) on the ML-1M-shaped operand over the heavy-row
split knobs (functional.GAT_HEAVY_THRESHOLD / GAT_SEGMENT): on a graph this small the
per-row chains, not the line requests, set the time. Each setting's output against the
unsplit (threshold 0) output: max |diff| (tolerance-level: the segments reassociate the
softmax sums).

    python tools/exp_gat_small.py [threshold:segment ...]
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.models import GAT  # noqa: E402
from src.ops import functional as F  # noqa: E402

dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
torch.manual_seed(0)
m = GAT(ds.n_users, ds.n_items, 64, 3, 4).to(dev).eval()


def ms_of(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(5):
        s.record()
        for _ in range(reps):
            out = fn()
        e.record()
        e.synchronize()
        best.append(s.elapsed_time(e) / reps)
    return sorted(best)[2], out


with torch.no_grad():
    F.GAT_HEAVY_THRESHOLD = 0
    t0, (u0, i0) = ms_of(lambda: m(g))
    ref = torch.cat([u0, i0])
    print(json.dumps({"threshold": 0, "segment": None, "ms": t0}), flush=True)
    knobs = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [
        (2048, 1024), (1024, 512), (512, 256), (256, 256), (256, 128), (128, 128), (128, 64),
        (64, 64), (64, 32)]
    for thr, seg in knobs:
        F.GAT_HEAVY_THRESHOLD, F.GAT_SEGMENT = thr, seg
        t, (u, i) = ms_of(lambda: m(g))
        d = (torch.cat([u, i]) - ref).abs().max().item()
        print(json.dumps({"threshold": thr, "segment": seg, "ms": t, "max_abs_diff_vs_unsplit": d,
                          "max_abs": ref.abs().max().item()}), flush=True)
