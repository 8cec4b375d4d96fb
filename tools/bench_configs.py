"""Secondary benchmarks: the BASELINE.json configs other than the headline (1 GPU).

    python tools/bench_configs.py [--configs 2 3 4 5] [--steps 10]

  2  ML-1M-shaped LightGCN K=3 d=64 (synthetic 6040 x 3706, 1M ratings -> reference
     preprocessing), model-class forward
  3  G100M NGCF K=3 d=64 + GAS after every layer (NGCFGroupShuffle, one fused MFMA kernel
     per layer), eval forward
  4  G100M LightGCN K=3 d=128 (the 8-GPU config run on one GPU; the sharded run is bench.py)
  5  power-law bipartite graph, GAT d=64 4 heads K=3 (a 1-GPU slice of the G1B config:
     Zipf-popularity users/items, every node degree >= 1)

Each config prints one JSON line: ms per forward, edges/s (= layers * nnz / t), and the
per-kernel times from HIP events where the kernels are called directly.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gnn-recommendations_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from src.data.dataset import RecommendationDataset  # noqa: E402
from src.models import GAT, LightGCN, NGCFGroupShuffle  # noqa: E402
from src.ops import CsrGraph  # noqa: E402


def time_fn(fn, steps, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / steps


def powerlaw_graph(n_users, n_items, n_pairs, a, seed):
    rng = np.random.default_rng(seed)
    pu = 1.0 / np.arange(1, n_users + 1) ** a
    pi = 1.0 / np.arange(1, n_items + 1) ** a
    u = rng.choice(n_users, n_pairs, p=pu / pu.sum())
    i = rng.choice(n_items, n_pairs, p=pi / pi.sum())
    # min degree >= 1 (the reference's dense GAT turns an isolated node into all-NaN)
    u = np.concatenate([u, np.arange(n_users), rng.integers(0, n_users, n_items)])
    i = np.concatenate([i, rng.integers(0, n_items, n_users), np.arange(n_items)])
    return CsrGraph.from_interactions(u, i, n_users, n_items, binary=True, n_threads=16)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", type=int, default=[2, 3, 4, 5])
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    out = []
    g100 = None
    if 3 in a.configs or 4 in a.configs:
        g100 = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16).to(dev)
    with torch.no_grad():
        if 2 in a.configs:
            ds = RecommendationDataset.synthetic_movielens(6040, 3706, 1_000_209, seed=1, name="ml-1m")
            g = ds.get_graph(dev)
            torch.manual_seed(0)
            m = LightGCN(ds.n_users, ds.n_items, 64, 3, 0.1).to(dev).eval()
            t = time_fn(lambda: m(g), a.steps * 10)
            out.append({"config": 2, "workload": "ML-1M-shaped LightGCN K=3 d=64 forward",
                        "nnz": g.nnz, "n_nodes": g.shape[0], "ms": t,
                        "edges_per_s": 3 * g.nnz / (t * 1e-3)})
        if 3 in a.configs:
            torch.manual_seed(0)
            m = NGCFGroupShuffle(1_000_000, 1_000_000, 64, [64, 64, 64], 0.1, 0.01, 8, 0.3).to(dev).eval()
            t = time_fn(lambda: m(g100), a.steps)
            for L in m.layers:
                L.single_kernel = True
            t1 = time_fn(lambda: m(g100), a.steps)
            out.append({"config": 3, "workload": "G100M NGCF K=3 d=64 + GAS (hop + streaming "
                        "MFMA transform per layer)", "nnz": g100.nnz, "ms": t,
                        "edges_per_s": 3 * g100.nnz / (t * 1e-3),
                        "ms_single_kernel_form": t1,
                        "mfma_flops_per_s": 3 * 2 * 2_000_000 * 128 * 64 / (t * 1e-3)})
            del m
        if 4 in a.configs:
            torch.manual_seed(0)
            m = LightGCN(1_000_000, 1_000_000, 128, 3, 0.1).to(dev).eval()
            t = time_fn(lambda: m(g100), a.steps)
            out.append({"config": 4, "workload": "G100M LightGCN K=3 d=128 on ONE GPU",
                        "nnz": g100.nnz, "ms": t, "edges_per_s": 3 * g100.nnz / (t * 1e-3)})
            del m
        del g100
        torch.cuda.empty_cache()
        if 5 in a.configs:
            t0 = time.time()
            g = powerlaw_graph(2_000_000, 2_000_000, 50_000_000, 0.9, 0).to(dev)
            deg = torch.diff(g.row_ptr).cpu().numpy()
            torch.manual_seed(0)
            m = GAT(2_000_000, 2_000_000, 64, 3, 4, 0.1, 0.2, 0.1).to(dev).eval()
            t = time_fn(lambda: m(g), a.steps)
            out.append({"config": 5, "workload": "power-law 2Mx2M (50M pairs, Zipf 0.9) GAT d=64 "
                        "4 heads K=3 forward (1-GPU slice of the G1B config)",
                        "nnz": g.nnz, "max_degree": int(deg.max()), "median_degree": float(np.median(deg)),
                        "ms": t, "edges_per_s": 3 * g.nnz / (t * 1e-3),
                        "graph_build_s": time.time() - t0})
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
