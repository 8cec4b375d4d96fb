"""Heavy-row bucket sweep (not part of the product): LightGCN K=3 d=64 forward on the
ML-1M-shaped graph (BASELINE config 2) per (heavy_threshold, split_above), with the heavy
launch concurrent with the row-parallel kernel. One JSON line per setting."""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT), str(ROOT / "tools")]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.ops import functional as F  # noqa: E402


def t_ms(fn, reps=100):
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
deg = (g.row_ptr[1:] - g.row_ptr[:-1])
x = torch.randn(g.shape[0], 64, device=dev) * 0.1
ref, _ = F.lightgcn_forward(g, x, 3, heavy_threshold=0)
for thr in (128, 256, 512):
    for split in (0, 1024, 2048, 4096):
        F.SPMM_HEAVY_SPLIT = split
        out, _ = F.lightgcn_forward(g, x, 3, heavy_threshold=thr)
        ms = t_ms(lambda: F.lightgcn_forward(g, x, 3, heavy_threshold=thr))
        print(json.dumps({"graph": "ml1m", "heavy_threshold": thr, "split_above": split,
                          "rows_heavy": int((deg > thr).sum()),
                          "rows_split": int((deg > split).sum()) if split else 0,
                          "ms_forward": ms, "bit_exact": bool(torch.equal(out, ref))}),
              flush=True)
