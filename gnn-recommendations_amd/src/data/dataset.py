"""Minimal dataset holder around the operand (reference: src/data/dataset.py).

The reference's raw-data ETL (loaders, binarisation, k-core, id remap) is out of scope
(SURVEY §2 rows 13-15); what the hot path needs is kept: train/valid/test interaction
tables with the reference's column names, `build_graph`, `get_torch_adjacency` (same
semantics, dataset.py:472-491) and `get_graph(device)` — the operand built ONCE and kept
resident instead of being re-wrapped and copied to the device every epoch
(trainer.py:233-234). `from_ratings` reproduces the reference's preprocessing for a ratings
table (rating >= threshold, iterative k-core, id remap, per-user temporal split
dataset.py:281-364); `synthetic_movielens` makes an ML-100K-shaped stand-in offline.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, Optional, Tuple

import numpy as np
import pandas as pd
import torch

from ..ops.graph import CsrGraph
from .graph_builder import build_bipartite_graph, convert_to_torch_sparse, normalize_adjacency_matrix


class RecommendationDataset:
    def __init__(self, name: str = "custom", root_dir: Optional[str] = None,
                 train_data: Optional[pd.DataFrame] = None,
                 valid_data: Optional[pd.DataFrame] = None,
                 test_data: Optional[pd.DataFrame] = None,
                 n_users: Optional[int] = None, n_items: Optional[int] = None):
        self.name = name
        self.root_dir = Path(root_dir) if root_dir else Path.cwd()
        self.train_data, self.valid_data, self.test_data = train_data, valid_data, test_data
        self.n_users, self.n_items = n_users, n_items
        self.adj_matrix = None
        self.norm_adj_matrix = None
        self._graphs: Dict[Tuple[str, bool], CsrGraph] = {}

    # ---- construction ---------------------------------------------------------------------
    @classmethod
    def from_ratings(cls, ratings: pd.DataFrame, name: str = "ratings",
                     rating_threshold: float = 3.0, min_user: int = 5, min_item: int = 5):
        df = ratings[ratings["rating"] >= rating_threshold][["userId", "itemId", "timestamp"]]
        df = df.drop_duplicates(["userId", "itemId"])
        while True:  # iterative k-core (preprocessing.py:16-77)
            uc = df["userId"].map(df["userId"].value_counts())
            ic = df["itemId"].map(df["itemId"].value_counts())
            keep = (uc >= min_user) & (ic >= min_item)
            if keep.all():
                break
            df = df[keep]
        umap = {u: k for k, u in enumerate(sorted(df["userId"].unique()))}
        imap = {i: k for k, i in enumerate(sorted(df["itemId"].unique()))}
        df = df.assign(userId=df["userId"].map(umap), itemId=df["itemId"].map(imap))
        df = df.sort_values(["userId", "timestamp"], kind="stable")
        pos = df.groupby("userId").cumcount(ascending=False)   # 0 = last interaction
        n = df["userId"].map(df["userId"].value_counts())
        test = df[(pos == 0) & (n >= 2)]
        valid = df[(pos == 1) & (n >= 3)]
        train = df[~(((pos == 0) & (n >= 2)) | ((pos == 1) & (n >= 3)))]
        cols = ["userId", "itemId"]
        return cls(name, None, train[cols].reset_index(drop=True), valid[cols].reset_index(drop=True),
                   test[cols].reset_index(drop=True), len(umap), len(imap))

    @classmethod
    def synthetic_movielens(cls, n_users: int = 943, n_items: int = 1682, n_ratings: int = 100_000,
                            seed: int = 42, name: str = "ml-100k-synthetic"):
        """ML-100K-shaped stand-in (943 x 1682, 100k ratings, Zipf item popularity)."""
        rng = np.random.default_rng(seed)
        pop = 1.0 / np.arange(1, n_items + 1) ** 0.8
        pop /= pop.sum()
        u = rng.integers(0, n_users, n_ratings)
        i = rng.choice(n_items, n_ratings, p=pop)
        r = rng.integers(1, 6, n_ratings).astype(np.float32)
        t = rng.integers(8.7e8, 8.9e8, n_ratings)
        return cls.from_ratings(pd.DataFrame({"userId": u, "itemId": i, "rating": r,
                                              "timestamp": t}), name)

    def load_processed_data(self):
        """Reads data/processed/<name>/{train,valid,test}.txt + stats.json (dataset.py:493-524)."""
        base = self.root_dir / "data" / "processed" / self.name
        files = [base / f for f in ("train.txt", "valid.txt", "test.txt", "stats.json")]
        if not all(f.exists() for f in files):
            raise FileNotFoundError(f"processed data not found under {base}")
        rd = lambda f: pd.read_csv(f, sep="\t", header=None, names=["userId", "itemId"])  # noqa: E731
        self.train_data, self.valid_data, self.test_data = (rd(f) for f in files[:3])
        stats = json.loads(files[3].read_text())
        self.n_users, self.n_items = stats["n_users"], stats["n_items"]
        return self

    # ---- operand ------------------------------------------------------------------------
    def build_graph(self, normalize: bool = True, self_loop: bool = False,
                    normalization_type: str = "symmetric"):
        self.adj_matrix = build_bipartite_graph(self.train_data, self.n_users, self.n_items,
                                                self_loop=self_loop)
        self.norm_adj_matrix = (normalize_adjacency_matrix(self.adj_matrix, normalization_type)
                                if normalize else self.adj_matrix)
        return self.adj_matrix, self.norm_adj_matrix

    def get_torch_adjacency(self, normalized: bool = True) -> torch.Tensor:
        if self.norm_adj_matrix is None:
            self.build_graph()
        return convert_to_torch_sparse(self.norm_adj_matrix if normalized else self.adj_matrix)

    def get_graph(self, device="cuda", normalized: bool = True) -> CsrGraph:
        key = (str(device), normalized)
        g = self._graphs.get(key)
        if g is None:
            args = (self.train_data["userId"].to_numpy(), self.train_data["itemId"].to_numpy(),
                    self.n_users, self.n_items)
            norm = "symmetric" if normalized else "none"
            if torch.device(device).type == "cuda":   # built in HBM (§8f3)
                g = CsrGraph.from_interactions_device(*args, normalization=norm, device=device)
            else:
                g = CsrGraph.from_interactions(*args, normalization=norm)
            self._graphs[key] = g
        return g

    def seen_items(self, include_valid: bool = True) -> Tuple[np.ndarray, np.ndarray]:
        """Per-user sorted train(+valid) items as CSR (seen_ptr int64, seen_col int32)."""
        parts = [self.train_data] + ([self.valid_data] if include_valid and self.valid_data is not None else [])
        df = pd.concat(parts).drop_duplicates().sort_values(["userId", "itemId"])
        cnt = np.bincount(df["userId"].to_numpy(), minlength=self.n_users)
        ptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        return ptr, df["itemId"].to_numpy().astype(np.int32)
