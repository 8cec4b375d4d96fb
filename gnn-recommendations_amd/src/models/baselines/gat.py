"""GAT for collaborative filtering (reference: src/models/baselines/gat.py), sparse on MI355X.

The reference materialises, per head and layer, a dense [N, N] score matrix masked by the
adjacency pattern (gat.py:99-141): O(N^2) memory, infeasible beyond N ~ 2e4. On a ROCm
operand each layer here is one dense projection for all heads (a plain library GEMM whose
weight also carries a_self^T W_h and a_neigh^T W_h, so h and both attention halves come out
of it together) plus ONE native sparse kernel that does the edge softmax and the aggregation for all
heads over the CSR pattern, with the head mean (last layer), F.elu and the layer mean
fused into its epilogue (gnnrec_gat_aggregate_f32). Parameters keep the reference's names
and creation order. Semantics difference, documented: an isolated node yields a NaN row
for that node only (softmax over an empty set); the reference's dense matmul spreads that
NaN to every node.
"""
import os
import warnings
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..base import BaseRecommender
from ... import ops
from ...ops._lib import EPI_ACC_ADD, EPI_ACC_DIV, EPI_ACC_INIT, EPI_NO_Y
from ...ops.graph import CsrGraph

# The reference's dense path (gat.py:99-141) holds an [N, N] fp32 mask plus, per head, [N, N]
# scores, their masked copy and the attention matrix; with autograd on, every head's [N, N]
# intermediates stay alive for the backward. A native operand that the sparse kernel cannot
# take (autograd on with parameters that require grad, attention dropout in training mode, a
# width without a kernel instance) runs that path only when its estimated footprint fits the
# device's free memory (a 288 GB MI355X holds it up to N ~ 8e4 for inference), and raises
# otherwise — never an allocation that is known not to fit. GNNREC_GAT_DENSE_MAX_NODES=<n>
# (or setting GAT_DENSE_MAX_NODES here) replaces the memory test with a fixed node cap.
GAT_DENSE_MAX_NODES = None

# Native layers form the attention scores in the kernel from the rows it gathers
# (gnnrec_gat_aggregate_att_f32) instead of reading projected score tables per neighbour
# (DESIGN §3.4, round 5); False keeps the score-table kernels (A/B and tests).
GAT_SCORES_FROM_ROWS = os.environ.get("GNNREC_GAT_SCORES_FROM_ROWS", "1") != "0"

# Training (autograd on, or attention dropout in training mode) on a native operand runs the
# native aggregation with its backward (gnnrec_gat_train_*) when the operand's pattern is
# symmetric; otherwise the reference's dense path, within check_dense_fallback's bound.
GAT_NATIVE_TRAIN = os.environ.get("GNNREC_GAT_NATIVE_TRAIN", "1") != "0"
DENSE_FALLBACK_MEM_FRACTION = 0.9


def dense_fallback_bytes(n_nodes: int, heads: int, grad: bool) -> int:
    """Peak bytes of the reference's dense masked softmax for one layer: the [N, N] mask plus
    three [N, N] per-head intermediates (scores, masked scores, attention), all heads' kept
    alive when autograd records them."""
    nn2 = 4 * int(n_nodes) * int(n_nodes)
    return nn2 * (1 + 3 * (max(1, int(heads)) if grad else 1))


def _available_bytes(device) -> int:
    if device is not None and torch.device(device).type == "cuda":
        free, _ = torch.cuda.mem_get_info(device)
        # blocks torch's caching allocator holds but does not use are free for this path too
        cached = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
        return int(free + max(0, cached))
    try:
        import psutil
        return int(psutil.virtual_memory().available)
    except Exception:  # noqa: BLE001
        return 1 << 62


def _node_cap():
    env = os.environ.get("GNNREC_GAT_DENSE_MAX_NODES")
    if env:
        return int(env)
    return GAT_DENSE_MAX_NODES


def check_dense_fallback(n_nodes: int, why: str, heads: int = 1, grad: bool = False,
                         device=None) -> None:
    """Refuse (RuntimeError) the dense masked-softmax path for a native operand when its
    estimated footprint (dense_fallback_bytes) exceeds DENSE_FALLBACK_MEM_FRACTION of the
    device's available memory, or when N exceeds a configured node cap
    (GNNREC_GAT_DENSE_MAX_NODES / GAT_DENSE_MAX_NODES); warn otherwise. `why` says what
    ruled the native kernel out."""
    need = dense_fallback_bytes(n_nodes, heads, grad)
    cap = _node_cap()
    if cap is not None:
        refuse = n_nodes > cap
        limit = f"the node cap GNNREC_GAT_DENSE_MAX_NODES = {cap}"
    else:
        avail = _available_bytes(device)
        refuse = need > DENSE_FALLBACK_MEM_FRACTION * avail
        limit = (f"{DENSE_FALLBACK_MEM_FRACTION:.0%} of the {avail / 1e9:.1f} GB available "
                 f"(GNNREC_GAT_DENSE_MAX_NODES sets a node cap instead)")
    if refuse:
        raise RuntimeError(
            f"GATLayer: the native sparse kernel does not apply ({why}) and the reference's "
            f"dense [N, N] softmax path would need ~{need / 1e9:.1f} GB for N = {n_nodes} "
            f"({heads} heads, autograd {'on' if grad else 'off'}), above {limit}. Run the "
            f"forward under torch.no_grad() / eval(), or on a smaller graph.")
    warnings.warn(f"GATLayer: dense O(N^2) reference path on a native operand "
                  f"(N = {n_nodes}, ~{need / 1e9:.2f} GB; {why})", RuntimeWarning, stacklevel=3)


class GATLayer(nn.Module):
    def __init__(self, in_dim: int, out_dim: int, n_heads: int = 1, dropout: float = 0.0,
                 alpha: float = 0.2, concat_heads: bool = True):
        super().__init__()
        self.in_dim, self.out_dim, self.n_heads = in_dim, out_dim, n_heads
        self.concat_heads, self.dropout, self.alpha = concat_heads, dropout, alpha
        self.W = nn.ModuleList(nn.Linear(in_dim, out_dim, bias=False) for _ in range(n_heads))
        self.a_self = nn.ParameterList(nn.Parameter(torch.zeros(size=(out_dim, 1)))
                                       for _ in range(n_heads))
        self.a_neigh = nn.ParameterList(nn.Parameter(torch.zeros(size=(out_dim, 1)))
                                        for _ in range(n_heads))
        self.leakyrelu = nn.LeakyReLU(alpha)
        self.dropout_layer = nn.Dropout(dropout)

    def native_block(self, a) -> Optional[str]:
        """Why the native kernel cannot run this layer on operand `a` (None: it can)."""
        if not isinstance(a, CsrGraph):
            return "not a native operand"
        width = self.n_heads * self.out_dim
        if width not in (16, 32, 64, 128, 256) or self.out_dim % 4:
            return f"heads*out_dim = {width} has no kernel instance"
        if self.training and self.dropout != 0.0:
            return "attention dropout in training mode"
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return "autograd is enabled and the native kernel has no backward"
        return None

    def native_ok(self, a, x) -> bool:
        return self.native_block(a) is None

    def fused_weight(self) -> torch.Tensor:
        """[H*o + 2H, in]: the stacked head projections W_h, then a_self_h^T W_h and
        a_neigh_h^T W_h, so ONE GEMM x @ W^T yields h and both attention halves (the
        reference computes mm(W_h x, a), gat.py:113-118: the same value reassociated).
        Cached until a parameter changes (inference only)."""
        from ..orthogonal_bundle.group_shuffle_layer import param_key
        params = list(self.W.parameters()) + list(self.a_self) + list(self.a_neigh)
        grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        key = None if grad else param_key(params)
        if key is not None and getattr(self, "_fused_key", None) == key:
            return self._fused_w
        Wcat = torch.cat([w.weight for w in self.W], dim=0)               # [H*o, in]
        ws = torch.stack([a[:, 0] @ w.weight for a, w in zip(self.a_self, self.W)])
        wn = torch.stack([a[:, 0] @ w.weight for a, w in zip(self.a_neigh, self.W)])
        out = torch.cat([Wcat, ws, wn], dim=0)
        if key is not None:
            self._fused_w, self._fused_key = out.detach(), key
        return out

    @staticmethod
    def _project(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        """x @ w^T; on a ROCm device the streaming MFMA row GEMM (gnnrec_rows_gemm_f32) for the
        shapes it has an instance for, otherwise — explicitly — a plain library GEMM
        (hipBLASLt through torch.matmul on the same device; rows_gemm itself never falls
        back)."""
        if x.is_cuda and ops.functional.rows_gemm_supported(x.shape[1], w.shape[0]):
            if not ops.functional._rows_view_ok(x):
                x = x.contiguous()
            return ops.functional.rows_gemm(x, w.t())
        return x @ w.t()

    def projections(self, x: torch.Tensor):
        """h = [W_0 x | ... | W_H x] and the per-head attention halves s_self, s_neigh, all
        from one GEMM (h is a strided view of its output)."""
        ho = self.n_heads * self.out_dim
        out = self._project(x, self.fused_weight())                        # [N, H*o + 2H]
        return out[:, :ho], out[:, ho:ho + self.n_heads], out[:, ho + self.n_heads:]

    def shares_input(self) -> bool:
        """Head-averaged layer: aggregate x itself per head and apply W_h afterwards,
        mean_h sum_j a_hj W_h x_j = (1/H) sum_h W_h (sum_j a_hj x_j), so a neighbour costs an
        in_dim-wide gather instead of the H*out_dim-wide h (4x fewer bytes for the last GAT
        layer). Same value reassociated (fp32 tolerance, like the rest of GAT)."""
        return (not self.concat_heads and self.in_dim % 4 == 0
                and self.n_heads * self.in_dim in (16, 32, 64, 128, 256)
                # the head mean W_h after the aggregation runs on the native row GEMM only
                and ops.functional.rows_gemm_supported(self.n_heads * self.in_dim,
                                                       self.out_dim))

    def head_mean_weight(self) -> torch.Tensor:
        """[H*in, out] = vstack(W_h^T) / H: z (per-head aggregates of x) @ this = the head mean."""
        return torch.cat([w.weight.t() for w in self.W], dim=0) / self.n_heads

    # ---- scores from the rows (gnnrec_gat_aggregate_att_f32): the projection writes h only --
    def att_dim(self) -> int:
        """Width of the row a head's scores are dotted with: in_dim (shared rows) or out_dim."""
        return self.in_dim if self.shares_input() else self.out_dim

    def att_ok(self) -> bool:
        """The ATT kernels take this layer (and GAT_SCORES_FROM_ROWS is on)."""
        return GAT_SCORES_FROM_ROWS and ops.functional.gat_att_supported(self.att_dim())

    def att_vectors(self) -> torch.Tensor:
        """[2, H, w]: the self / neighbour attention vectors the kernel dots rows with —
        a_self_h, a_neigh_h (w = out_dim, against h_h = W_h x), or for shared rows the row
        vectors a_h^T W_h (w = in_dim, against x itself). Cached until a parameter changes."""
        from ..orthogonal_bundle.group_shuffle_layer import param_key
        params = list(self.W.parameters()) + list(self.a_self) + list(self.a_neigh)
        key = param_key(params)
        if getattr(self, "_att_key", None) == key:
            return self._att
        with torch.no_grad():
            if self.shares_input():
                vs = [a[:, 0] @ w.weight for a, w in zip(self.a_self, self.W)]
                vn = [a[:, 0] @ w.weight for a, w in zip(self.a_neigh, self.W)]
            else:
                vs = [a[:, 0] for a in self.a_self]
                vn = [a[:, 0] for a in self.a_neigh]
            att = torch.stack([torch.stack(vs), torch.stack(vn)]).float().contiguous()
        self._att, self._att_key = att, key
        return att

    def head_weight(self) -> torch.Tensor:
        """[H*o, in]: the stacked head projections (h = x @ this^T)."""
        from ..orthogonal_bundle.group_shuffle_layer import param_key
        params = list(self.W.parameters())
        key = param_key(params)
        if getattr(self, "_hw_key", None) == key:
            return self._hw
        with torch.no_grad():
            w = torch.cat([w.weight for w in self.W], dim=0).float().contiguous()
        self._hw, self._hw_key = w, key
        return w

    def native_rows(self, x: torch.Tensor) -> torch.Tensor:
        """The table the ATT aggregation gathers for the rows of x: x itself (shared rows), or
        h = [W_0 x | ... | W_H x] written by the row GEMM into a gather-placed table
        (functional.hop_table: aligned rows, no line at the slow offset)."""
        if self.shares_input():
            return x
        w = self.head_weight()
        ho = w.shape[0]
        if x.is_cuda and ops.functional.rows_gemm_supported(x.shape[1], ho):
            if not ops.functional._rows_view_ok(x):
                x = x.contiguous()
            out = ops.functional.hop_table(x.shape[0], ho, device=x.device)
            ops.functional.rows_gemm(x, w.t(), out=out)
            return out
        return x @ w.t()

    def native_forward_att(self, a, feat, hself, *, apply_elu: bool = False, epi: int = 0,
                           self_rows=None, acc=None, acc_div: float = 1.0) -> torch.Tensor:
        """The native layer from native_rows: `feat` the gathered table (maybe exchanged),
        `hself` the destination rows' own rows of it."""
        att = self.att_vectors().to(feat.device)
        if not self.shares_input():
            return ops.functional.gat_aggregate_att(
                a, feat, hself, att, self.n_heads, self.out_dim, self.alpha,
                mean_heads=not self.concat_heads, apply_elu=apply_elu, epi=epi,
                self_rows=self_rows, acc=acc, acc_div=acc_div)
        z = ops.functional.gat_aggregate_att(a, feat, hself, att, self.n_heads, self.in_dim,
                                             self.alpha, shared_rows=True)
        return ops.functional.rows_gemm(z, self.head_mean_weight(), apply_elu=apply_elu, epi=epi,
                                        self_rows=self_rows, acc=acc, acc_div=acc_div)

    # ---- training on the native operand (gnnrec_gat_train_*: aggregation + backward) -------
    def train_ok(self, a) -> bool:
        """The differentiable native aggregation takes this layer on operand `a`."""
        return GAT_NATIVE_TRAIN and ops.functional.gat_train_supported(a, self.n_heads,
                                                                        self.out_dim)

    def native_train_forward(self, x: torch.Tensor, a) -> torch.Tensor:
        """gat.py:92-151 with autograd: h_q = W_q x, s_self = h_q a_self_q, s_neigh = h_q
        a_neigh_q in torch (the reference's ops), the masked softmax + dropout + weighted sum
        per head on the native kernels (their backward included); then concat or head mean.
        The dropout mask's seed is drawn from torch's generator (torch.manual_seed makes runs
        repeatable)."""
        H, o = self.n_heads, self.out_dim
        # (row-chunked weight gradients, ops.functional.linear_rows)
        h = torch.cat([ops.functional.linear_rows(x, w) for w in self.W], dim=1)   # [N, H*o]
        hs = h.view(-1, H, o)
        a_s = torch.stack([a[:, 0] for a in self.a_self])                  # [H, o]
        a_n = torch.stack([a[:, 0] for a in self.a_neigh])
        s_self = (hs * a_s).sum(-1)                                        # [N, H]
        s_neigh = (hs * a_n).sum(-1)
        p = self.dropout if self.training else 0.0
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if p > 0 else 0
        out = ops.functional.gat_aggregate_train(a, h, s_self, s_neigh, H, o, self.alpha, p, seed)
        return out if self.concat_heads else out.view(-1, H, o).mean(dim=1)

    def native_inputs(self, x: torch.Tensor):
        """(table gathered per neighbour, s_self, s_neigh) for the rows of x."""
        if self.shares_input():
            H = self.n_heads
            s = self._project(x, self.fused_weight()[H * self.out_dim:])    # [N, 2H]
            return x, s[:, :H], s[:, H:]
        return self.projections(x)

    def native_forward(self, a, feat, s_self, s_neigh, *, apply_elu: bool = False, epi: int = 0,
                       self_rows=None, acc=None, acc_div: float = 1.0) -> torch.Tensor:
        """The native layer given native_inputs (feat may be a gathered/exchanged table)."""
        if not self.shares_input():
            return ops.gat_aggregate(a, feat, s_self, s_neigh, self.n_heads, self.out_dim,
                                     self.alpha, mean_heads=not self.concat_heads,
                                     apply_elu=apply_elu, epi=epi, self_rows=self_rows, acc=acc,
                                     acc_div=acc_div)
        z = ops.gat_aggregate(a, feat, s_self, s_neigh, self.n_heads, self.in_dim, self.alpha,
                              mean_heads=False, apply_elu=False, shared_rows=True)
        # W_h, ELU and the layer-mean accumulator in one pass (the aggregation epilogue's order)
        return ops.functional.rows_gemm(z, self.head_mean_weight(), apply_elu=apply_elu, epi=epi,
                                        self_rows=self_rows, acc=acc, acc_div=acc_div)

    def forward(self, x: torch.Tensor, adj_matrix, *, apply_elu: bool = False, epi: int = 0,
                self_rows=None, acc=None, acc_div: float = 1.0) -> torch.Tensor:
        a = ops.as_operand(adj_matrix)
        why = self.native_block(a)
        if why is None:
            if self.att_ok():
                feat = self.native_rows(x)
                return self.native_forward_att(a, feat, feat, apply_elu=apply_elu, epi=epi,
                                               self_rows=self_rows, acc=acc, acc_div=acc_div)
            return self.native_forward(a, *self.native_inputs(x), apply_elu=apply_elu, epi=epi,
                                       self_rows=self_rows, acc=acc, acc_div=acc_div)
        if self.train_ok(a):
            out = self.native_train_forward(x, a)
            return F.elu(out) if apply_elu else out
        if isinstance(a, CsrGraph):
            grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
            check_dense_fallback(a.shape[0], why, heads=self.n_heads, grad=grad,
                                 device=a.row_ptr.device)
        out = self._dense_forward(x, a)
        return F.elu(out) if apply_elu else out

    def _dense_forward(self, x, adj_matrix):
        """The reference's dense masked-softmax path (gat.py:92-151)."""
        if isinstance(adj_matrix, CsrGraph):
            adj_matrix = adj_matrix.to_torch_sparse_coo()
        if adj_matrix.is_sparse:
            idx = adj_matrix.coalesce().indices()
            mask = torch.sparse_coo_tensor(idx, torch.ones(idx.size(1), device=x.device),
                                           adj_matrix.size()).to_dense()
        else:
            mask = adj_matrix
        heads = []
        for i in range(self.n_heads):
            h = self.W[i](x)
            scores = self.leakyrelu(torch.mm(h, self.a_self[i]) + torch.mm(h, self.a_neigh[i]).t())
            scores = scores.masked_fill(mask == 0, float("-inf"))
            att = self.dropout_layer(F.softmax(scores, dim=1))
            heads.append(torch.mm(att, h))
        return torch.cat(heads, dim=1) if self.concat_heads else torch.stack(heads).mean(dim=0)


class GAT(BaseRecommender):
    def __init__(self, n_users: int, n_items: int, embedding_dim: int = 64, n_layers: int = 3,
                 n_heads: int = 4, dropout: float = 0.1, alpha: float = 0.2,
                 init_scale: float = 0.01):
        super().__init__(n_users, n_items, embedding_dim)
        self.n_layers, self.n_heads = n_layers, n_heads
        self.dropout, self.alpha, self.init_scale = dropout, alpha, init_scale
        self.user_embedding = nn.Embedding(n_users, embedding_dim)
        self.item_embedding = nn.Embedding(n_items, embedding_dim)
        self.layers = nn.ModuleList()
        # gat.py:203-239: concat layers (embedding_dim // n_heads per head), last one averages
        for _ in range(max(1, n_layers - 1)):
            self.layers.append(GATLayer(embedding_dim, embedding_dim // n_heads, n_heads, dropout,
                                        alpha, concat_heads=True))
        if n_layers > 1:
            self.layers.append(GATLayer(embedding_dim, embedding_dim, n_heads, dropout, alpha,
                                        concat_heads=False))
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.normal_(self.user_embedding.weight, mean=0.0, std=self.init_scale)
        nn.init.normal_(self.item_embedding.weight, mean=0.0, std=self.init_scale)
        for layer in self.layers:
            for w in layer.W:
                nn.init.xavier_uniform_(w.weight)
            for p in layer.a_self:
                nn.init.xavier_uniform_(p.data)
            for p in layer.a_neigh:
                nn.init.xavier_uniform_(p.data)

    def forward(self, adj_matrix) -> Tuple[torch.Tensor, torch.Tensor]:
        x = self._initial_table()
        a = ops.as_operand(adj_matrix)
        L = len(self.layers)
        if all(layer.native_ok(a, x) for layer in self.layers):
            acc = torch.empty_like(x)
            for k, layer in enumerate(self.layers, start=1):
                epi = EPI_ACC_INIT if k == 1 else EPI_ACC_ADD
                if k == L:
                    epi |= EPI_ACC_DIV | EPI_NO_Y   # only the layer mean is read after it
                x = layer(x, a, apply_elu=True, epi=epi, self_rows=x, acc=acc,
                          acc_div=float(L + 1))
            x_final = acc
        else:
            outs = [x]
            for layer in self.layers:
                x = F.elu(layer(x, a))
                outs.append(x)
            x_final = torch.stack(outs, dim=0).mean(dim=0)
        user_emb, item_emb = torch.split(x_final, [self.n_users, self.n_items], dim=0)
        return user_emb, item_emb

    def predict(self, users, items, adj_matrix=None) -> torch.Tensor:
        if adj_matrix is None:
            raise ValueError("adj_matrix must be given for GAT")
        user_emb, item_emb = self._serving_embeddings(adj_matrix)
        return self._score_pairs(user_emb, item_emb, users, items)

    def get_all_embeddings(self, adj_matrix=None):
        if adj_matrix is None:
            raise ValueError("adj_matrix must be given for GAT")
        return self.forward(adj_matrix)
