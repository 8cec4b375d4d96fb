"""Orthogonal Bundle GNN (reference: src/models/orthogonal_bundle/__init__.py)."""
from .model import OrthogonalBundleGNN
from .group_shuffle_layer import GroupShuffleLayer
from .bundle_layer import BundleConnectionLayer, EdgeSpecificBundleConnection
from .parallel_transport import ParallelTransportLayer, parallel_transport_along_edges

__all__ = ["OrthogonalBundleGNN", "GroupShuffleLayer", "BundleConnectionLayer",
           "EdgeSpecificBundleConnection", "ParallelTransportLayer",
           "parallel_transport_along_edges"]
