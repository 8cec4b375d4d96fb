"""NGCF (K = 3, d = 64) BPR training step on G100M (batch 2048), the six W1 / W2 weight
gradients as one library GEMM each against the row-chunked form (functional.linear_rows),
alternating, same process. Median ms per step and the loss after the timed steps of each mode
(both modes start from the same weights and batches).

    python tools/exp_ngcf_train.py
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gnn-recommendations_amd"), str(ROOT)]
import bench  # noqa: E402
from src.models import NGCF  # noqa: E402
from src.ops import functional as F  # noqa: E402
from src.training import BPRLoss, DeviceSampler, make_adam, train_step  # noqa: E402

dev = torch.device("cuda", 0)
g100 = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
g = g100.to(dev)
rp = g100.row_ptr.numpy()
users = np.repeat(np.arange(1_000_000), np.diff(rp[:1_000_001]))
items = g100.col.numpy()[:rp[1_000_000]] - 1_000_000
default = F.LINEAR_SPLIT_K_MIN_ROWS
for mode in ("library", "row_chunks", "library", "row_chunks"):
    F.LINEAR_SPLIT_K_MIN_ROWS = 10 ** 12 if mode == "library" else default
    torch.manual_seed(0)
    m = NGCF(1_000_000, 1_000_000, 64, [64, 64, 64]).to(dev).train()
    samp = DeviceSampler(users, items, 1_000_000, 2048, 1, dev, seed=0)
    opt = make_adam(m.parameters(), 1e-3, 1e-4, dev)
    loss_fn = BPRLoss()
    for _ in range(2):
        train_step(m, g, *samp(), opt, loss_fn, 1.0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        loss = train_step(m, g, *samp(), opt, loss_fn, 1.0)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    print(json.dumps({"mode": mode, "ms_median": ts[len(ts) // 2], "ms_samples": ts,
                      "loss": float(loss)}), flush=True)
    del m, opt
    torch.cuda.empty_cache()
