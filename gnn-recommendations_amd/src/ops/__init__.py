"""MI355X propagation ops: the graph operand, the native kernels and their dispatch.

`sparse_mm(adj, x)` is what the models call where the reference calls
``torch.sparse.mm(adj_matrix, x)``:

* a :class:`CsrGraph` on a ROCm device            -> libgnnrec SpMM (HIP, bit-exact)
* a torch sparse tensor on a ROCm device          -> converted once to a CsrGraph (cached)
                                                      -> libgnnrec SpMM
* a torch sparse tensor on the CPU                -> ``torch.sparse.mm`` (the reference's own
                                                      CPU path; BASELINE config 1)
* a dense tensor                                  -> ``torch.mm`` (as the reference)

A CsrGraph left on the CPU is an error: the native path never silently degrades.
"""
from __future__ import annotations

import torch

from .graph import CsrGraph, ShardInfo, inv_sqrt_degrees
from . import functional, library  # library: registers torch.ops.gnnrec.*
from .functional import (dense_layer, gas, gat_aggregate, lightgcn_propagate, ngcf_layer,
                         score_topk, spmm, spmm_gas)

__all__ = ["CsrGraph", "ShardInfo", "inv_sqrt_degrees", "functional", "spmm", "spmm_gas",
           "gas", "ngcf_layer", "dense_layer", "gat_aggregate", "score_topk", "lightgcn_propagate", "as_operand",
           "sparse_mm", "uses_native"]

_CACHE: dict = {}


def _cache_key(adj: torch.Tensor):
    if adj.layout == torch.sparse_coo:
        parts = (adj._indices(), adj._values())
    else:
        parts = (adj.crow_indices(), adj.col_indices(), adj.values())
    return (id(adj), tuple(adj.shape), adj._nnz(),
            tuple((t.data_ptr(), t._version) for t in parts))


def as_operand(adj):
    """Map the reference's adjacency argument onto the native operand where it applies."""
    if isinstance(adj, CsrGraph):
        if adj.device.type != "cuda":
            raise ValueError("CsrGraph operands must live on a ROCm device; call .to('cuda')")
        return adj
    if isinstance(adj, torch.Tensor) and adj.is_sparse or (
            isinstance(adj, torch.Tensor) and adj.layout == torch.sparse_csr):
        if adj.device.type == "cuda":
            key = _cache_key(adj)
            g = _CACHE.get(key)
            if g is None:
                _CACHE.clear()
                g = CsrGraph.from_torch_sparse(adj)
                # the entry holds the source tensor: while cached, neither its id() nor its
                # storage can be recycled by another operand that would then map to this graph
                _CACHE[key] = (g, adj)
            else:
                g = g[0]
            return g
    return adj


def uses_native(adj) -> bool:
    return isinstance(as_operand(adj), CsrGraph)


def sparse_mm(adj, x: torch.Tensor) -> torch.Tensor:
    a = as_operand(adj)
    if isinstance(a, CsrGraph):
        return spmm(a, x)
    if a.is_sparse:
        return torch.sparse.mm(a, x)
    return torch.mm(a, x)
