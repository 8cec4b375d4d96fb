"""NGCF as implemented by the reference (src/models/baselines/ngcf.py), MI355X kernels.

Per layer (ngcf.py:52-86, the code's form, not the paper's):
    n = A x;   out = Dropout(LeakyReLU_0.2(W1 n + b1 + W2 (x * n) + b2))
and the model output is cat(x0, x1, ..., xK) along features (ngcf.py:186).

On a ROCm operand in inference (no autograd, dropout inactive) each layer is ONE kernel:
SpMM + both Linear layers on MFMA + bias + LeakyReLU (gnnrec_spmm_ngcf_f32). With autograd
on, the SpMM stays native (differentiable) and the two 64x64 Linear layers run through torch.
"""
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from ..base import BaseRecommender
from ... import ops
from ...ops.graph import CsrGraph


class NGCFLayer(nn.Module):
    """One NGCF propagation layer (ngcf.py:19-86)."""

    def __init__(self, in_dim: int, out_dim: int, dropout: float = 0.0):
        super().__init__()
        self.W1 = nn.Linear(in_dim, out_dim, bias=True)
        self.W2 = nn.Linear(in_dim, out_dim, bias=True)
        self.dropout = nn.Dropout(dropout)
        self.activation = nn.LeakyReLU(negative_slope=0.2)
        self.single_kernel = False  # True: gather + MFMA in one launch (see ops.ngcf_layer)

    def _fused_ok(self, x: torch.Tensor, a) -> bool:
        return (isinstance(a, CsrGraph) and not (torch.is_grad_enabled() and (
            x.requires_grad or self.W1.weight.requires_grad))
            and (not self.training or self.dropout.p == 0.0)
            and self.W1.in_features == self.W1.out_features
            and self.W1.in_features in (32, 64, 128))

    def forward(self, x: torch.Tensor, adj_matrix, gas: Optional[nn.Module] = None) -> torch.Tensor:
        a = ops.as_operand(adj_matrix)
        if self._fused_ok(x, a) and (gas is None or gas.fusable()):
            blocks, perm = (gas.blocks(), gas.perm) if gas is not None else (None, None)
            return ops.ngcf_layer(a, x, self.W1.weight, self.W1.bias, self.W2.weight,
                                  self.W2.bias, self.activation.negative_slope,
                                  gas_blocks=blocks, gas_perm=perm, fused=self.single_kernel)
        n = ops.sparse_mm(a, x)
        if isinstance(a, CsrGraph):   # device path: row-chunked weight gradients (training)
            lin = ops.functional.linear_rows
            out = lin(n, self.W1) + lin(x * n, self.W2)
        else:
            out = self.W1(n) + self.W2(x * n)
        out = self.dropout(self.activation(out))
        return gas(out) if gas is not None else out


class NGCF(BaseRecommender):
    def __init__(self, n_users: int, n_items: int, embedding_dim: int = 64,
                 layer_sizes: Optional[List[int]] = None, dropout: float = 0.1,
                 init_scale: float = 0.01):
        super().__init__(n_users, n_items, embedding_dim)
        layer_sizes = [64, 64, 64] if layer_sizes is None else list(layer_sizes)
        self.layer_sizes = layer_sizes
        self.n_layers = len(layer_sizes)
        self.dropout = dropout
        self.init_scale = init_scale
        self.user_embedding = nn.Embedding(n_users, embedding_dim)
        self.item_embedding = nn.Embedding(n_items, embedding_dim)
        dims = [embedding_dim] + layer_sizes
        self.layers = nn.ModuleList(NGCFLayer(dims[k], dims[k + 1], dropout)
                                    for k in range(self.n_layers))
        self.reset_parameters()

    def reset_parameters(self):
        # ngcf.py:143-155
        nn.init.normal_(self.user_embedding.weight, mean=0.0, std=self.init_scale)
        nn.init.normal_(self.item_embedding.weight, mean=0.0, std=self.init_scale)
        for layer in self.layers:
            for lin in (layer.W1, layer.W2):
                nn.init.xavier_uniform_(lin.weight)
                nn.init.zeros_(lin.bias)

    def forward(self, adj_matrix) -> Tuple[torch.Tensor, torch.Tensor]:
        x_final = self._native_concat_forward(adj_matrix, [None] * self.n_layers)
        if x_final is None:
            x = self._initial_table()
            outs = [x]
            for layer in self.layers:
                x = layer(x, adj_matrix)
                outs.append(x)
            x_final = torch.cat(outs, dim=1)
        user_emb, item_emb = torch.split(x_final, [self.n_users, self.n_items], dim=0)
        return user_emb, item_emb

    def _native_concat_forward(self, adj_matrix, gs_layers):
        """Inference on a ROCm operand: every layer's fused kernel reads its input from, and
        writes its output into, its column block of the final [N, (K+1) d] table, so
        torch.cat(outs, dim=1) (ngcf.py:186) costs no extra pass over 2 GB at G100M. Same
        values as the layer-by-layer form (the kernels do not depend on row strides).
        None when a layer cannot take the fused path."""
        a = ops.as_operand(adj_matrix)
        d = self.embedding_dim
        if not all(layer._fused_ok(self.user_embedding.weight, a) and layer.W1.in_features == d
                   and (gs is None or gs.fusable())
                   for layer, gs in zip(self.layers, gs_layers)):
            return None
        n = self.n_users + self.n_items
        w = self.user_embedding.weight
        # placed so that the gathered blocks x0 .. x_{K-1} avoid the slow line offset
        # (ops.functional.gather_table); still a contiguous [N, (K+1) d] tensor
        out = ops.functional.gather_table(n, d * (self.n_layers + 1), d * self.n_layers,
                                          dtype=w.dtype, device=w.device)
        out[:self.n_users, :d].copy_(self.user_embedding.weight.detach())
        out[self.n_users:, :d].copy_(self.item_embedding.weight.detach())
        for k, (layer, gs) in enumerate(zip(self.layers, gs_layers)):
            blocks, perm = (gs.blocks(), gs.perm) if gs is not None else (None, None)
            ops.ngcf_layer(a, out[:, k * d:(k + 1) * d], layer.W1.weight, layer.W1.bias,
                           layer.W2.weight, layer.W2.bias, layer.activation.negative_slope,
                           gas_blocks=blocks, gas_perm=perm, fused=layer.single_kernel,
                           out=out[:, (k + 1) * d:(k + 2) * d])
        return out

    def predict(self, users, items, adj_matrix=None) -> torch.Tensor:
        if adj_matrix is None:
            raise ValueError("adj_matrix must be given for NGCF")
        user_emb, item_emb = self._serving_embeddings(adj_matrix)
        return self._score_pairs(user_emb, item_emb, users, items)

    def get_all_embeddings(self, adj_matrix=None) -> Tuple[torch.Tensor, torch.Tensor]:
        if adj_matrix is None:
            raise ValueError("adj_matrix must be given for NGCF")
        return self.forward(adj_matrix)


class NGCFGroupShuffle(NGCF):
    """BASELINE config 3: NGCF with a Group-and-Shuffle transform after every layer,
    x_{l+1} = GS_l(NGCFLayer_l(x_l)); fused into one kernel per layer on a ROCm operand.
    The composition is defined by this build (the reference has no such model class); its
    oracle is composed from the reference's NGCFLayer and GroupShuffleLayer."""

    def __init__(self, n_users: int, n_items: int, embedding_dim: int = 64,
                 layer_sizes: Optional[List[int]] = None, dropout: float = 0.1,
                 init_scale: float = 0.01, block_size: int = 8, gs_init_scale: float = 0.01):
        super().__init__(n_users, n_items, embedding_dim, layer_sizes, dropout, init_scale)
        from ..orthogonal_bundle.group_shuffle_layer import GroupShuffleLayer
        self.gs_layers = nn.ModuleList(GroupShuffleLayer(d, block_size, gs_init_scale)
                                       for d in self.layer_sizes)

    def forward(self, adj_matrix) -> Tuple[torch.Tensor, torch.Tensor]:
        x_final = self._native_concat_forward(adj_matrix, list(self.gs_layers))
        if x_final is None:
            x = self._initial_table()
            outs = [x]
            for layer, gs in zip(self.layers, self.gs_layers):
                x = layer(x, adj_matrix, gas=gs)
                outs.append(x)
            x_final = torch.cat(outs, dim=1)
        user_emb, item_emb = torch.split(x_final, [self.n_users, self.n_items], dim=0)
        return user_emb, item_emb
