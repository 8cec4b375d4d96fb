"""Recommender models over the MI355X propagation kernels (import surface of the
reference's src/models/__init__.py for the propagation models)."""
from .base import BaseRecommender
from .orthogonal_bundle import OrthogonalBundleGNN, GroupShuffleLayer
from .baselines import LightGCN, NGCF, NGCFGroupShuffle, GAT

__all__ = ["BaseRecommender", "OrthogonalBundleGNN", "GroupShuffleLayer", "LightGCN", "NGCF",
           "NGCFGroupShuffle", "GAT"]
