"""Bipartite operand construction with the reference's API (src/data/graph_builder.py).

`build_bipartite_graph`, `normalize_adjacency_matrix`, `convert_to_torch_sparse` and the
npz/pt save/load keep the reference's signatures and return types (scipy COO / torch COO) and
produce the same matrices, but are computed by the native builder (csrc/host.cpp): counting
sort + per-row merge instead of scipy's coo->csr->sparse-product chain (2.2 s vs 31 s at
2e8 nnz). `build_csr_graph` returns the device-resident operand the kernels consume.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import scipy.sparse as sp
import torch

from ..ops.graph import CsrGraph, inv_sqrt_degrees
from ..ops import _lib


def _pairs(interactions, user_col, item_col):
    if hasattr(interactions, "__getitem__") and not isinstance(interactions, (tuple, list)):
        u = np.asarray(interactions[user_col], dtype=np.int64)
        i = np.asarray(interactions[item_col], dtype=np.int64)
    else:
        u, i = (np.asarray(a, dtype=np.int64) for a in interactions)
    return u, i


def build_bipartite_graph(interactions, n_users: int, n_items: int, user_col: str = "userId",
                          item_col: str = "itemId", self_loop: bool = False) -> sp.coo_matrix:
    """A = [[0, R], [R^T, 0]] (+ I) as scipy COO (graph_builder.py:16-80); rows sorted,
    columns ascending, duplicate interactions summed (the same matrix as the reference's)."""
    u, i = _pairs(interactions, user_col, item_col)
    g = CsrGraph.from_interactions(u, i, n_users, n_items, normalization="none",
                                   self_loop=self_loop)
    rp = g.row_ptr.numpy()
    rows = np.repeat(np.arange(rp.size - 1), np.diff(rp))
    N = n_users + n_items
    print(f"bipartite graph: {N} nodes, {u.size} interactions, {g.nnz} non-zeros")
    return sp.coo_matrix((g.val.numpy(), (rows, g.col.numpy().astype(np.int64))), shape=(N, N),
                         dtype=np.float32)


def normalize_adjacency_matrix(adj, normalization: str = "symmetric") -> sp.coo_matrix:
    """D^-1/2 A D^-1/2 ('symmetric'), D^-1 A ('row') or A ('none') (graph_builder.py:83-144);
    values bit-identical to scipy's products (fl(fl(dis[r]*a)*dis[c]))."""
    if normalization == "none":
        return adj
    if normalization not in ("symmetric", "row"):
        raise ValueError(f"unknown normalization: {normalization}")
    csr = sp.csr_matrix(adj, dtype=np.float32)
    csr.sum_duplicates()
    csr.sort_indices()
    deg = np.asarray(csr.sum(axis=1), dtype=np.float32).ravel()
    dis = inv_sqrt_degrees(deg, normalization)
    rp = csr.indptr.astype(np.int64)
    col = csr.indices.astype(np.int32)
    cnt = csr.data.astype(np.float32)
    val = np.empty(max(1, cnt.size), np.float32)[:cnt.size]
    _lib.check(_lib.lib().gnnrec_normalize_values(
        rp.ctypes.data, col.ctypes.data, cnt.ctypes.data, rp.size - 1, dis.ctypes.data,
        0 if normalization == "symmetric" else 1, val.ctypes.data, 0), "normalize_values")
    out = sp.csr_matrix((val, col, rp), shape=csr.shape).tocoo()
    print(f"normalization applied: {normalization}")
    return out


def convert_to_torch_sparse(adj) -> torch.Tensor:
    """scipy -> torch COO exactly as graph_builder.py:147-174 (int64 indices, uncoalesced)."""
    adj = adj.tocoo()
    idx = torch.from_numpy(np.vstack([adj.row, adj.col]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(adj.data.astype(np.float32)),
                                   torch.Size(adj.shape))


def save_adjacency_matrix(adj, filepath: str, format: str = "npz"):
    if format == "npz":
        sp.save_npz(filepath, adj)
    elif format == "pt":
        torch.save(convert_to_torch_sparse(adj), filepath)
    else:
        raise ValueError(f"unknown format: {format}")


def load_adjacency_matrix(filepath: str, format: str = "npz") -> sp.coo_matrix:
    if format == "npz":
        return sp.load_npz(filepath)
    if format == "pt":
        t = torch.load(filepath, weights_only=True).coalesce()
        idx, val = t.indices().numpy(), t.values().numpy()
        return sp.coo_matrix((val, (idx[0], idx[1])), shape=tuple(t.shape))
    raise ValueError(f"unknown format: {format}")


def build_csr_graph(interactions, n_users: int, n_items: int, normalization: str = "symmetric",
                    self_loop: bool = False, device: Optional[str] = None,
                    user_col: str = "userId", item_col: str = "itemId") -> CsrGraph:
    """The resident operand for the kernels, straight from the interaction list."""
    u, i = _pairs(interactions, user_col, item_col)
    g = CsrGraph.from_interactions(u, i, n_users, n_items, normalization=normalization,
                                   self_loop=self_loop)
    return g.to(device) if device is not None else g
