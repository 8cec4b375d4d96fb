"""A BPR training step (batch 2048, trainer.py:248-279 semantics: propagation, loss, backward,
clip, Adam) at the ML-1M shape for LightGCN and NGCF, with the row-subset forward forced on,
off, and as train_step picks it (default). Median ms per step; run under rocprofv3
--kernel-trace to split it.

    python tools/exp_train_ml1m.py
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.models import LightGCN, NGCF  # noqa: E402
from src.training import BPRLoss, DeviceSampler, make_adam, train_step  # noqa: E402

from src.training import trainer  # noqa: E402
from src.training.trainer import _row_subset_pays as _pays  # noqa: E402

dev = torch.device("cuda", 0)
ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
g = ds.get_graph(dev)
nu, ni = ds.n_users, ds.n_items
rp = g.row_ptr.cpu().numpy()
users = np.repeat(np.arange(nu), np.diff(rp[:nu + 1]))
items = g.col.cpu().numpy()[:rp[nu]] - nu

for name, make in (("lightgcn", lambda: LightGCN(nu, ni, 64, 3, 0.1)),
                   ("ngcf", lambda: NGCF(nu, ni, 64, [64, 64, 64]))):
    # each form twice, alternating (the first timed configuration of a process runs slow)
    for form in ("full", "subset", "full", "subset", "default"):
        subset = form != "full"
        trainer._row_subset_pays = (lambda adj: True) if form == "subset" else _pays
        torch.manual_seed(0)
        m = make().to(dev).train()
        samp = DeviceSampler(users, items, ni, 2048, 1, dev, seed=0)
        opt = make_adam(m.parameters(), 1e-3, 1e-4, dev)
        loss_fn = BPRLoss()
        for _ in range(5):
            train_step(m, g, *samp(), opt, loss_fn, 1.0, row_subset=subset)
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            loss = train_step(m, g, *samp(), opt, loss_fn, 1.0, row_subset=subset)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        print(json.dumps({"model": name, "form": form, "ms_median": ts[len(ts) // 2],
                          "ms_min": ts[0], "loss": float(loss)}), flush=True)
