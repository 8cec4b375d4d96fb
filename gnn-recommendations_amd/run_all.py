"""Experiment entry point (reference: run_all.py + scripts/run_multiple_seeds.py +
scripts/run_all_experiments.py), kept to the plumbing the propagation path needs.

    python run_all.py [--quick] [--skip-check] [--models lightgcn ...] [--datasets ml-100k]
                      [--seeds 42 43] [--n_layers K] [--embedding_dim d] [--epochs E]
                      [--device cpu|cuda]

For every dataset x model x seed: load the dataset (data/processed/<name> if present, else
data/raw/<name>/u.data or ratings.dat through the reference's preprocessing, else an
ML-100K-shaped synthetic stand-in — there is no network), build the model from
config/models/<name>.yaml (kwargs filtered by the constructor signature, as
run_all_experiments.py:99-126) with the CLI overrides, train with BPR for `epochs`
(full-graph propagation per batch, as trainer.py:239-279), evaluate recall/ndcg@{10,20} and
write results/run_all.json. On a ROCm device every propagation goes through libgnnrec.
"""
from __future__ import annotations

import argparse
import inspect
import json
import sys
import time
from pathlib import Path

import numpy as np
import pandas as pd
import torch
import yaml

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from src.data import RecommendationDataset  # noqa: E402
from src.evaluation import Evaluator  # noqa: E402
from src.models import GAT, NGCF, LightGCN, NGCFGroupShuffle, OrthogonalBundleGNN  # noqa: E402
from src.training import Trainer  # noqa: E402

MODEL_REGISTRY = {"lightgcn": LightGCN, "ngcf": NGCF, "ngcf_gs": NGCFGroupShuffle, "gat": GAT,
                  "orthogonal_bundle": OrthogonalBundleGNN}


def create_model(name: str, n_users: int, n_items: int, overrides: dict) -> torch.nn.Module:
    cls = MODEL_REGISTRY.get(name)
    if cls is None:
        raise ValueError(f"unknown model: {name}")
    cfg = ROOT / "config" / "models" / f"{name}.yaml"
    params = {"embedding_dim": 64}
    if cfg.exists():
        params.update(yaml.safe_load(cfg.read_text()).get("model", {}))
    params.update({k: v for k, v in overrides.items() if v is not None})
    if "n_layers" in overrides and overrides["n_layers"] is not None and "layer_sizes" in params:
        params["layer_sizes"] = [params["embedding_dim"]] * int(overrides["n_layers"])
    valid = set(inspect.signature(cls.__init__).parameters) - {"self"}
    return cls(n_users=n_users, n_items=n_items, **{k: v for k, v in params.items() if k in valid})


def load_dataset(name: str, seed: int) -> RecommendationDataset:
    ds = RecommendationDataset(name, ROOT)
    try:
        return ds.load_processed_data()
    except FileNotFoundError:
        pass
    raw = ROOT / "data" / "raw" / name
    if (raw / "u.data").exists():
        r = pd.read_csv(raw / "u.data", sep="\t", names=["userId", "itemId", "rating", "timestamp"])
        return RecommendationDataset.from_ratings(r, name)
    if (raw / "ratings.dat").exists():
        r = pd.read_csv(raw / "ratings.dat", sep="::", engine="python",
                        names=["userId", "itemId", "rating", "timestamp"])
        return RecommendationDataset.from_ratings(r, name, min_user=10, min_item=10)
    print(f"[run_all] {name}: no local data, using the ML-100K-shaped synthetic stand-in")
    return RecommendationDataset.synthetic_movielens(seed=seed, name=f"{name}-synthetic")


def train_bpr(model, dataset, adj, cfg: dict, epochs: int, device, seed: int) -> float:
    """BPR training (src/training/trainer.py: the reference's per-batch full-graph propagation,
    [B, 1] negatives, clipping, Adam) for `epochs` epochs; returns the wall time."""
    if epochs <= 0:
        return 0.0
    t = Trainer(model, dataset, dict(cfg, epochs=epochs), device=device, seed=seed)
    t0 = time.time()
    for _ in range(epochs):
        t.train_epoch()
    if device.type == "cuda":
        torch.cuda.synchronize()
    return time.time() - t0


def check_device(device) -> dict:
    info = {"device": str(device), "torch": torch.__version__}
    if device.type == "cuda":
        from src.ops import _lib
        info.update(gpu=torch.cuda.get_device_name(device), libgnnrec=_lib.version())
    print("[run_all] " + json.dumps(info))
    return info


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--quick", action="store_true", help="1 seed, 1 epoch, LightGCN only")
    ap.add_argument("--skip-check", action="store_true")
    ap.add_argument("--models", nargs="+", default=["lightgcn", "orthogonal_bundle"])
    ap.add_argument("--datasets", nargs="+", default=["ml-100k"])
    ap.add_argument("--seeds", nargs="+", type=int, default=[42, 43])
    ap.add_argument("--n_layers", type=int, default=None)
    ap.add_argument("--embedding_dim", type=int, default=None)
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--output", default=str(ROOT / "results" / "run_all.json"))
    a = ap.parse_args(argv)
    if a.quick:
        a.seeds = a.seeds[:1]
    device = torch.device(a.device)
    if not a.skip_check:
        check_device(device)
    cfg = yaml.safe_load((ROOT / "config" / "training.yaml").read_text())
    epochs = a.epochs if a.epochs is not None else (1 if a.quick else int(cfg.get("epochs", 10)))
    results = []
    for ds_name in a.datasets:
        for model_name in a.models:
            for seed in a.seeds:
                rec = {"model": model_name, "dataset": ds_name, "seed": seed, "status": "failed"}
                try:
                    torch.manual_seed(seed)
                    ds = load_dataset(ds_name, seed)
                    model = create_model(model_name, ds.n_users, ds.n_items,
                                         {"n_layers": a.n_layers,
                                          "embedding_dim": a.embedding_dim}).to(device)
                    adj = ds.get_graph(device) if device.type == "cuda" else ds.get_torch_adjacency()
                    rec["training_time"] = train_bpr(model, ds, adj, cfg, epochs, device, seed)
                    t0 = time.time()
                    rec["test_metrics"] = Evaluator(device=device).evaluate(model, ds, adj_matrix=adj)
                    rec["eval_time"] = time.time() - t0
                    rec.update(status="success", n_users=ds.n_users, n_items=ds.n_items,
                               n_train=len(ds.train_data), epochs=epochs)
                except Exception as e:  # recorded like run_all_experiments.py:218-221
                    rec["error"] = f"{type(e).__name__}: {e}"
                print(f"[run_all] {json.dumps(rec)}", flush=True)
                results.append(rec)
    out = Path(a.output)
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(results, indent=1))
    return 0 if all(r["status"] == "success" for r in results) else 1


if __name__ == "__main__":
    sys.exit(main())
