"""The reference's CPU propagation path, op for op in plain PyTorch — TEST/BASELINE ONLY.

Used by bench.py's cpu_baseline leg (the timed CPU comparator, kind "port") and by tests.
It restates, without importing the reference:
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
