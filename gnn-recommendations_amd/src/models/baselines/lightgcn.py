"""LightGCN (He et al. 2020) over the MI355X propagation kernels.

Reference: src/models/baselines/lightgcn.py. Semantics kept: x0 = cat(U, I); K hops
x_k = A x_{k-1}; output = mean(x0..xK) split into (users, items). On a ROCm operand the K
hops and the layer mean run as one native call (`gnnrec_lightgcn_f32`: K SpMM launches with
the mean fused into their epilogues, bit-exact with the reference CPU path); on a CPU
torch-sparse operand the reference's own torch.sparse.mm path runs.
"""
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from ..base import BaseRecommender
from ... import ops
from ...ops.graph import CsrGraph


class LightGCN(BaseRecommender):
    def __init__(self, n_users: int, n_items: int, embedding_dim: int = 64, n_layers: int = 3,
                 init_scale: float = 0.01):
        super().__init__(n_users, n_items, embedding_dim)
        self.n_layers = n_layers
        self.init_scale = init_scale
        self.user_embedding = nn.Embedding(n_users, embedding_dim)
        self.item_embedding = nn.Embedding(n_items, embedding_dim)
        self.reset_parameters()

    def reset_parameters(self):
        # lightgcn.py:57-60
        nn.init.normal_(self.user_embedding.weight, mean=0.0, std=self.init_scale)
        nn.init.normal_(self.item_embedding.weight, mean=0.0, std=self.init_scale)

    def _propagate(self, adj_matrix) -> torch.Tensor:
        x0 = self._initial_table()
        a = ops.as_operand(adj_matrix)
        if isinstance(a, CsrGraph):
            return ops.lightgcn_propagate(a, x0, self.n_layers)
        layers = [x0]
        x = x0
        for _ in range(self.n_layers):  # reference CPU path (lightgcn.py:86-95)
            x = ops.sparse_mm(a, x)
            layers.append(x)
        return torch.stack(layers, dim=0).mean(dim=0)

    def forward(self, adj_matrix) -> Tuple[torch.Tensor, torch.Tensor]:
        out = self._propagate(adj_matrix)
        user_emb, item_emb = torch.split(out, [self.n_users, self.n_items], dim=0)
        return user_emb, item_emb

    def forward_rows(self, adj_matrix, need: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """forward() where only the output rows marked in `need` (uint8 [n_users + n_items])
        are defined — what a training batch reads (ops.lightgcn_forward_rows: the last hops
        compute only those rows and their neighbourhoods; same bits at the marked rows). On
        a CPU operand it is forward()."""
        a = ops.as_operand(adj_matrix)
        if not isinstance(a, CsrGraph):
            return self.forward(adj_matrix)
        out = ops.lightgcn_propagate(a, self._initial_table(), self.n_layers, need=need)
        user_emb, item_emb = torch.split(out, [self.n_users, self.n_items], dim=0)
        return user_emb, item_emb

    def predict(self, users: torch.Tensor, items: torch.Tensor,
                adj_matrix: Optional[torch.Tensor] = None) -> torch.Tensor:
        if adj_matrix is None:
            raise ValueError("adj_matrix must be given for LightGCN")
        user_emb, item_emb = self._serving_embeddings(adj_matrix)
        return self._score_pairs(user_emb, item_emb, users, items)

    def get_all_embeddings(self, adj_matrix=None) -> Tuple[torch.Tensor, torch.Tensor]:
        if adj_matrix is None:
            raise ValueError("adj_matrix must be given for LightGCN")
        return self.forward(adj_matrix)

    def get_layer_embeddings(self, adj_matrix) -> List[torch.Tensor]:
        """[x0, x1, ..., xK] (lightgcn.py:153-183)."""
        x0 = self._initial_table()
        a = ops.as_operand(adj_matrix)
        if isinstance(a, CsrGraph) and not (torch.is_grad_enabled() and x0.requires_grad):
            _, layers = ops.functional.lightgcn_forward(a, x0.detach(), self.n_layers,
                                                        return_layers=True)
            return [x0.detach().clone()] + list(layers.unbind(0))
        out = [x0.clone()]
        x = x0
        for _ in range(self.n_layers):
            x = ops.sparse_mm(a, x)
            out.append(x.clone())
        return out
