"""OrthogonalBundleGNN over the MI355X kernels (reference: orthogonal_bundle/model.py).

Per layer l (adjacency path, model.py:159-201):
    x_conv = A x;  t = x_conv @ W_conn_l;  x_t = GS_l(t) = (t @ W_gs_l)[:, perm_l]
    x = (1 - alpha) x_t + alpha x_init        (dropout p = 0 by default)
final = sum_l softmax(layer_weights)_l x_l    (model.py:204-207)

W_conn_l @ W_gs_l[:, perm_l] composes to ONE dense d x d matrix M_l (2816/4096 nonzeros at
d = 64, bs = 8), a true small GEMM: on a ROCm operand in inference every layer is one
kernel — SpMM + MFMA (A x) @ M_l + residual + the softmax-weighted layer sum fused into its
epilogue (gnnrec_spmm_dense_f32). Training keeps the native SpMM (differentiable) and the
small transforms in torch. Parameter names/creation order follow the reference.
"""
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..base import BaseRecommender
from ... import ops
from ...ops.graph import CsrGraph
from .bundle_layer import BundleConnectionLayer
from .group_shuffle_layer import GroupShuffleLayer, param_key
from .parallel_transport import parallel_transport_along_edges


class OrthogonalBundleGNN(BaseRecommender):
    def __init__(self, n_users: int, n_items: int, embedding_dim: int = 64, n_layers: int = 3,
                 block_size: int = 8, residual_alpha: float = 0.1, dropout: float = 0.0,
                 init_scale: float = 0.01, use_parallel_transport: bool = True,
                 use_edge_index: bool = False):
        super().__init__(n_users, n_items, embedding_dim)
        if embedding_dim % block_size != 0:
            raise ValueError(f"embedding_dim ({embedding_dim}) must be divisible by "
                             f"block_size ({block_size})")
        self.n_layers = n_layers
        self.block_size = block_size
        self.residual_alpha = residual_alpha
        self.dropout = dropout
        self.use_parallel_transport = use_parallel_transport
        self.use_edge_index = use_edge_index
        self.user_embedding = nn.Embedding(n_users, embedding_dim)
        self.item_embedding = nn.Embedding(n_items, embedding_dim)
        nn.init.normal_(self.user_embedding.weight, std=0.01)
        nn.init.normal_(self.item_embedding.weight, std=0.01)
        if use_parallel_transport:
            self.connection_layers = nn.ModuleList(
                BundleConnectionLayer(embedding_dim, block_size) for _ in range(n_layers))
        self.local_transform_layers = nn.ModuleList(
            GroupShuffleLayer(embedding_dim, block_size, init_scale) for _ in range(n_layers))
        self.dropout_layer = nn.Dropout(dropout) if dropout > 0 else None
        self.layer_weights = nn.Parameter(torch.ones(n_layers + 1))

    # ---- helpers ----------------------------------------------------------------------------
    def composed_transform(self, layer_idx: int) -> torch.Tensor:
        """M_l = W_conn_l @ W_gs_l[:, perm_l]  (or W_gs_l[:, perm_l] without transport);
        cached between calls while no parameter changes (inference)."""
        gs = self.local_transform_layers[layer_idx]
        params = list(gs.skew_params) + (list(self.connection_layers[layer_idx].skew_params)
                                         if self.use_parallel_transport else [])
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return self._compose(layer_idx)
        key = param_key(params)
        cache = self.__dict__.setdefault("_composed_cache", {})
        if cache.get(layer_idx, (None,))[0] != key:
            cache[layer_idx] = (key, self._compose(layer_idx).detach())
        return cache[layer_idx][1]

    def _compose(self, layer_idx: int) -> torch.Tensor:
        gs = self.local_transform_layers[layer_idx]
        W_gs = gs._build_orthogonal_matrix()[:, gs.perm]
        if self.use_parallel_transport:
            return self.connection_layers[layer_idx]() @ W_gs
        return W_gs

    def _fused_ok(self, a, x0: torch.Tensor, edge_index) -> bool:
        if not isinstance(a, CsrGraph) or self.use_edge_index:
            return False
        if self.dropout_layer is not None and self.training:
            return False
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return False
        return self.embedding_dim in (32, 64, 128)

    def _transport(self, layer_idx, x, adj_matrix, edge_index):
        if self.use_parallel_transport:
            W_conn = self.connection_layers[layer_idx]()
            if self.use_edge_index:
                return parallel_transport_along_edges(x, edge_index, W_conn)
            return ops.sparse_mm(adj_matrix, x) @ W_conn
        if self.use_edge_index:
            return self._graph_conv_edge_index(x, edge_index)
        return ops.sparse_mm(adj_matrix, x)

    # ---- forward ------------------------------------------------------------------------------
    def forward(self, adj_matrix=None, edge_index=None) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.use_edge_index:
            if edge_index is None:
                raise ValueError("edge_index must be provided when use_edge_index=True")
        elif adj_matrix is None:
            raise ValueError("adj_matrix must be provided when use_edge_index=False")
        x_init = self._initial_table()
        a = ops.as_operand(adj_matrix) if adj_matrix is not None else None
        w = F.softmax(self.layer_weights, dim=0)
        if self._fused_ok(a, x_init, edge_index):
            ws = w.tolist()
            acc = torch.empty_like(x_init)
            x = x_init
            alpha = self.residual_alpha
            for l in range(self.n_layers):
                x = ops.dense_layer(a, x, self.composed_transform(l), 1 - alpha, x_init, alpha,
                                    acc=acc, acc_mode=1 if l == 0 else 2, w_out=ws[l + 1],
                                    w_res=ws[0], store_y=l + 1 < self.n_layers)
            x_final = acc
        else:
            x = x_init
            layers = [x]
            for l in range(self.n_layers):
                x_t = self.local_transform_layers[l](self._transport(l, x, a, edge_index))
                x = (1 - self.residual_alpha) * x_t + self.residual_alpha * x_init
                if self.dropout_layer is not None:
                    x = self.dropout_layer(x)
                layers.append(x)
            x_final = sum(wl * e for wl, e in zip(w, layers))
        return x_final[:self.n_users], x_final[self.n_users:]

    def _graph_conv_edge_index(self, x, edge_index):
        """index_add_(dst, x[src]) (model.py:215-220): on a ROCm device the edge list becomes a
        cached CSR of edge multiplicities and this is one native SpMM (same sum, fp32
        reassociation only)."""
        if x.is_cuda and x.dim() == 2 and x.stride(1) == 1:
            from .parallel_transport import edge_index_operand
            return ops.spmm(edge_index_operand(edge_index, x.size(0)), x)
        src, dst = edge_index
        out = torch.zeros_like(x)
        out.index_add_(0, dst, x[src])
        return out

    def predict(self, users, items, adj_matrix=None, edge_index=None) -> torch.Tensor:
        user_emb, item_emb = self._serving_embeddings(adj_matrix, edge_index)
        return self._score_pairs(user_emb, item_emb, users, items)

    def get_all_embeddings(self, adj_matrix=None, edge_index=None):
        return self.forward(adj_matrix, edge_index)

    # ---- monitors (model.py:246-302) ------------------------------------------------------------
    def get_orthogonality_errors(self) -> torch.Tensor:
        return torch.stack([l.get_orthogonality_error() for l in self.local_transform_layers])

    def get_orthogonality_metrics(self) -> Dict[str, torch.Tensor]:
        m: Dict[str, torch.Tensor] = {}
        fro, mx = zip(*(l.get_orthogonality_metrics() for l in self.local_transform_layers))
        m["local_fro_mean"] = torch.stack(fro).mean()
        m["local_fro_max"] = torch.stack(fro).max()
        m["local_max_dev"] = torch.stack(mx).max()
        if self.use_parallel_transport:
            cfro, cmx = zip(*(l.get_orthogonality_metrics() for l in self.connection_layers))
            m["conn_fro_mean"] = torch.stack(cfro).mean()
            m["conn_fro_max"] = torch.stack(cfro).max()
            m["conn_max_dev"] = torch.stack(cmx).max()
        return m

    def get_layer_embeddings(self, adj_matrix=None, edge_index=None) -> List[torch.Tensor]:
        """Per-layer x WITHOUT the residual/dropout, as the reference does (model.py:325-352)."""
        x = self._initial_table()
        out = [x.clone()]
        a = ops.as_operand(adj_matrix) if adj_matrix is not None else None
        fused = (isinstance(a, CsrGraph) and not (self.use_edge_index and edge_index is not None)
                 and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()))
                 and self.embedding_dim in (32, 64, 128))
        for l in range(self.n_layers):
            if fused:
                x = ops.dense_layer(a, x, self.composed_transform(l), 1.0, None, 0.0)
            else:
                if self.use_edge_index and edge_index is not None:
                    W = self.connection_layers[l]() if self.use_parallel_transport else None
                    t = (parallel_transport_along_edges(x, edge_index, W) if W is not None
                         else self._graph_conv_edge_index(x, edge_index))
                elif a is not None:
                    t = ops.sparse_mm(a, x)
                    if self.use_parallel_transport:
                        t = t @ self.connection_layers[l]()
                else:
                    raise ValueError("Must provide either adj_matrix or edge_index")
                x = self.local_transform_layers[l](t)
            out.append(x.clone())
        return out

    def reset_parameters(self):
        nn.init.normal_(self.user_embedding.weight, mean=0.0, std=0.01)
        nn.init.normal_(self.item_embedding.weight, mean=0.0, std=0.01)
        for layer in self.local_transform_layers:
            layer.reset_parameters()
