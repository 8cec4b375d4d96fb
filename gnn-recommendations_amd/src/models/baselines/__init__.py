"""Baseline graph recommenders (reference: src/models/baselines/__init__.py)."""
from .lightgcn import LightGCN
from .ngcf import NGCF, NGCFGroupShuffle
from .gat import GAT

__all__ = ["LightGCN", "NGCF", "NGCFGroupShuffle", "GAT"]
