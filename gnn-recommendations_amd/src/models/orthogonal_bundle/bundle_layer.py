"""Bundle connection matrices (reference: orthogonal_bundle/bundle_layer.py:9-149).

W_conn = blockdiag(expm(P_b - P_b^T))[:, shuffle_perm] — note the reference permutes the
COLUMNS OF W here, not of the product (contrast GroupShuffleLayer). Same parameter names and
creation order as the reference.
"""
from typing import Tuple

import torch
import torch.nn as nn


class BundleConnectionLayer(nn.Module):
    def __init__(self, embedding_dim, block_size, n_blocks=None):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.block_size = block_size
        self.n_blocks = n_blocks or (embedding_dim // block_size)
        self.skew_params = nn.ParameterList(
            nn.Parameter(torch.randn(block_size, block_size) * 0.01)
            for _ in range(self.n_blocks))
        self.register_buffer("shuffle_perm", self._create_shuffle_permutation())

    def _create_shuffle_permutation(self):
        return torch.randperm(self.embedding_dim)

    def forward(self, edge_index=None) -> torch.Tensor:
        blocks = [torch.matrix_exp(p - p.transpose(-2, -1)) for p in self.skew_params]
        return torch.block_diag(*blocks)[:, self.shuffle_perm]

    def get_connection_matrix_for_edge(self, src_node, dst_node):
        return self.forward()

    def get_orthogonality_metrics(self) -> Tuple[torch.Tensor, torch.Tensor]:
        W = self.forward()
        diff = W.T @ W - torch.eye(self.embedding_dim, device=W.device, dtype=W.dtype)
        return torch.norm(diff, p="fro"), diff.abs().max()


class EdgeSpecificBundleConnection(nn.Module):
    """One connection matrix per edge type (bundle_layer.py:106-149)."""

    def __init__(self, embedding_dim, block_size, n_edge_types=2):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.connection_layers = nn.ModuleList(
            BundleConnectionLayer(embedding_dim, block_size) for _ in range(n_edge_types))

    def forward(self, edge_index, edge_type):
        n_edges = edge_index.size(1)
        W = torch.zeros(n_edges, self.embedding_dim, self.embedding_dim, device=edge_index.device)
        for t, layer in enumerate(self.connection_layers):
            W[edge_type == t] = layer().unsqueeze(0)
        return W

    def type_matrices(self) -> torch.Tensor:
        """[n_edge_types, d, d]: the per-type connection matrices forward() broadcasts."""
        return torch.stack([layer() for layer in self.connection_layers])

    def transport(self, x, edge_index, edge_type):
        """parallel_transport_along_edges(x, edge_index, self(edge_index, edge_type)) without
        the [E, d, d] tensor (parallel_transport_typed: one native launch per edge type)."""
        from .parallel_transport import parallel_transport_typed
        return parallel_transport_typed(x, edge_index, edge_type, self.type_matrices())
