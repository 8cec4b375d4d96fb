"""Operand construction (reference: src/data/graph_builder.py) and a minimal dataset holder."""
from .graph_builder import (build_bipartite_graph, build_csr_graph, convert_to_torch_sparse,
                            load_adjacency_matrix, normalize_adjacency_matrix,
                            save_adjacency_matrix)
from .dataset import RecommendationDataset

__all__ = ["build_bipartite_graph", "normalize_adjacency_matrix", "convert_to_torch_sparse",
           "save_adjacency_matrix", "load_adjacency_matrix", "build_csr_graph",
           "RecommendationDataset"]
