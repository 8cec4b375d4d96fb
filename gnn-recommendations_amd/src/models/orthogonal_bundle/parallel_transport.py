"""Edge-list parallel transport (reference: orthogonal_bundle/parallel_transport.py:5-98).

Reference: x_src = x[src]; x_src @ W^T (or per-edge bmm); index_add_ into dst — it
materialises an [E, d] table (51 GB at 1e8 edges, d = 64). For a shared W the sum commutes
with the transform:  sum_{e: dst=j} x[src_e] W^T = (B x)_j W^T  with B the dst x src edge-count
matrix, so on a ROCm device the edge list is turned (once, cached) into a CsrGraph B and
the whole operation is ONE native SpMM + MFMA-transform kernel (gnnrec_spmm_dense_f32),
with no [E, d] intermediate. The sum order differs from index_add_'s (fp32 tolerance).
"""
import torch
import torch.nn as nn

from ... import ops
from ...ops.graph import CsrGraph

_EDGE_CACHE: dict = {}


def edge_index_operand(edge_index: torch.Tensor, num_nodes: int,
                       mask: torch.Tensor = None, tag=None) -> CsrGraph:
    """CsrGraph of B[dst, src] = multiplicity of (src -> dst), on edge_index's device (only
    the edges where `mask` holds, when given; `tag` names the subset in the cache key)."""
    key = (id(edge_index), edge_index.data_ptr(), edge_index._version, edge_index.shape[1],
           num_nodes, edge_index.device, tag)
    hit = _EDGE_CACHE.get(key)
    g = hit[0] if hit is not None else None
    if g is None:
        src, dst = edge_index[0].long(), edge_index[1].long()
        if mask is not None:
            src, dst = src[mask], dst[mask]
        vals = torch.ones(src.numel(), dtype=torch.float32, device=edge_index.device)
        coo = torch.sparse_coo_tensor(torch.stack([dst, src]), vals, (num_nodes, num_nodes))
        g = CsrGraph.from_torch_sparse(coo, symmetric=False)
        if len(_EDGE_CACHE) > 16:
            _EDGE_CACHE.clear()
        # holding edge_index keeps its id() and storage from being recycled while cached
        _EDGE_CACHE[key] = (g, edge_index)
    return g


def parallel_transport_typed(x: torch.Tensor, edge_index: torch.Tensor, edge_type: torch.Tensor,
                             W_types: torch.Tensor) -> torch.Tensor:
    """out[j] = sum over edges e = (i -> j) of W_types[edge_type[e]] @ x[i] — what
    parallel_transport_along_edges computes with the [E, d, d] tensor that
    EdgeSpecificBundleConnection.forward assembles (bundle_layer.py:106-149 feeding
    parallel_transport.py:37-43), without materialising it (16 KB per edge at d = 64): per
    type t the sum commutes with W_t, so out = sum_t (B_t x) W_t^T with B_t the type-t edge
    counts — one native SpMM + MFMA-transform launch per type, accumulated in place."""
    T = W_types.shape[0]
    if (x.is_cuda and x.dim() == 2 and x.shape[1] in (32, 64, 128)
            and not (torch.is_grad_enabled() and (x.requires_grad or W_types.requires_grad))):
        out = torch.zeros_like(x)
        for t in range(T):
            B = edge_index_operand(edge_index, x.size(0), edge_type == t,
                                   ("type", t, edge_type.data_ptr(), edge_type.numel()))
            if B.nnz == 0:
                continue
            ops.dense_layer(B, x, W_types[t].t(), 1.0, None, 0.0, acc=out, acc_mode=2,
                            w_out=1.0, store_y=False)
        return out
    return parallel_transport_along_edges(x, edge_index, W_types[edge_type.long()])


def parallel_transport_along_edges(x, edge_index, W_connection):
    src, dst = edge_index
    if (x.is_cuda and W_connection.dim() == 2 and x.dim() == 2 and x.shape[1] in (32, 64, 128)
            and not (torch.is_grad_enabled() and (x.requires_grad or W_connection.requires_grad))):
        B = edge_index_operand(edge_index, x.size(0))
        return ops.dense_layer(B, x, W_connection.t(), 1.0, None, 0.0)
    x_src = x[src]
    if W_connection.dim() == 2:
        x_t = torch.mm(x_src, W_connection.t())
    elif W_connection.dim() == 3:
        x_t = torch.bmm(W_connection, x_src.unsqueeze(-1)).squeeze(-1)
    else:
        raise ValueError(f"Invalid W_connection shape: {W_connection.shape}")
    out = torch.zeros_like(x)
    out.index_add_(0, dst, x_t)
    return out


class ParallelTransportLayer(nn.Module):
    """Transport + optional edge weights + GCN-style deg^-1/2 scaling (:55-98)."""

    def __init__(self, embedding_dim, normalize=True):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.normalize = normalize

    def forward(self, x, edge_index, W_connection, edge_weight=None):
        out = parallel_transport_along_edges(x, edge_index, W_connection)
        if edge_weight is not None:
            out = out * edge_weight.unsqueeze(-1)
        if self.normalize:
            deg = torch.zeros(x.size(0), device=x.device, dtype=torch.long)
            deg.index_add_(0, edge_index[1], torch.ones(edge_index.size(1), device=x.device,
                                                        dtype=torch.long))
            dis = deg.float().pow(-0.5)
            dis[dis == float("inf")] = 0
            out = out * dis.unsqueeze(-1)
        return out
