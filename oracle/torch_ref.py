"""The reference's CPU propagation path, op for op in plain PyTorch — TEST/BASELINE ONLY.

Used by bench.py's cpu_baseline leg (the timed CPU comparator, kind "port") and by tests.
It restates, without importing the reference:
  * build_bipartite_graph + normalize_adjacency_matrix (graph_builder.py:16-144) with scipy,
    as the reference runs them (timed as the CPU graph-build baseline);
  * convert_to_torch_sparse (graph_builder.py:163-172): int64 [2, nnz] indices, fp32 values,
    torch.sparse_coo_tensor(...) left uncoalesced exactly as the reference leaves it;
  * LightGCN.forward (lightgcn.py:76-95): K x torch.sparse.mm, stack().mean(0).
"""
from __future__ import annotations

import numpy as np
import torch


def coo_operand(row_ptr: np.ndarray, col: np.ndarray, val: np.ndarray, n_cols: int,
                rows: slice | None = None) -> torch.Tensor:
    """Reference-layout COO tensor of the CSR rows `rows` (default: all rows)."""
    rp = np.asarray(row_ptr, np.int64)
    lo, hi = (0, rp.size - 1) if rows is None else (rows.start, rows.stop)
    k0, k1 = int(rp[lo]), int(rp[hi])
    r = np.repeat(np.arange(hi - lo, dtype=np.int64), np.diff(rp[lo:hi + 1]))
    idx = torch.from_numpy(np.vstack([r, np.asarray(col[k0:k1], np.int64)]))
    v = torch.from_numpy(np.ascontiguousarray(val[k0:k1], np.float32))
    return torch.sparse_coo_tensor(idx, v, (hi - lo, n_cols))


def lightgcn_forward(adj: torch.Tensor, x0: torch.Tensor, n_layers: int) -> torch.Tensor:
    layers = [x0]
    x = x0
    for _ in range(n_layers):
        x = torch.sparse.mm(adj, x)
        layers.append(x)
    return torch.stack(layers, dim=0).mean(dim=0)


def scipy_operand(users: np.ndarray, items: np.ndarray, n_users: int, n_items: int):
    """The reference's operand construction on the CPU (graph_builder.py:16-144 + 147-174):
    COO of both directions (fp32 ones), tocsr, fp32 row sums clamped at 1, D^-1/2 A D^-1/2 by
    sparse diagonal products, tocoo, and the uncoalesced int64 torch COO tensor."""
    import scipy.sparse as sp
    u = np.asarray(users, np.int64)
    i = np.asarray(items, np.int64) + n_users
    n = n_users + n_items
    a = sp.coo_matrix((np.ones(2 * u.size, np.float32),
                       (np.concatenate([u, i]), np.concatenate([i, u]))),
                      shape=(n, n), dtype=np.float32).tocsr()
    deg = np.maximum(np.array(a.sum(axis=1)).flatten(), 1.0)
    dis = np.power(deg, -0.5)
    dis[np.isinf(dis)] = 0.0
    d = sp.diags(dis)
    norm = (d @ a @ d).tocoo()
    idx = torch.from_numpy(np.vstack([norm.row, norm.col]).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(norm.data.astype(np.float32)), (n, n))
