"""`torch.library` registration of the propagation ops.

    torch.ops.gnnrec.spmm(row_ptr, col, val, x, n_cols) -> y                 (= A x)
    torch.ops.gnnrec.lightgcn_propagate(row_ptr, col, val, x0, n_cols, n_layers, need=None)
        -> mean(x0, A x0, ..., A^K x0)                                       (lightgcn.py:76-95)
    and their gradients torch.ops.gnnrec.spmm_t / lightgcn_propagate_t (A^T g, mean_k (A^T)^k g)

The operand crosses the dispatcher as its three CSR tensors (int64 row_ptr [n_rows + 1]
with absolute offsets, int32 col, fp32 val — the CsrGraph layout), so `torch.compile`,
`torch.export` and FakeTensor tracing see ordinary tensor ops with known output shapes (the
fake kernels below). The CUDA (= ROCm) kernels run libgnnrec through `functional`; there is
no CPU kernel (a CPU operand is the reference's own torch.sparse.mm path, see ops.sparse_mm).

Autograd: d/dx of A x is A^T g, of the LightGCN mean is mean_k (A^T)^k g — the same native
launches over the transposed operand (A itself for the symmetric normalisation), exactly as
functional's forward/backward pair.

The ops find the CsrGraph that owns the three tensors (its column-ordered plan, heavy-row
lists and transpose are cached there): `functional.spmm` / `lightgcn_propagate` register
every graph they pass in (a weak map keyed by the tensors' storage, shape and version), and
raw tensors from elsewhere get a CsrGraph made once and kept with its source tensors.
"""
from __future__ import annotations

import weakref
from typing import Optional

import torch

from .graph import CsrGraph

_LIVE: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()
_OWNED: dict = {}          # raw-tensor operands: key -> (CsrGraph, source tensors)
_OWNED_MAX = 4
_OWNED_MAX_BYTES = 8 << 30  # operand bytes (CSR; cached plans come on top) kept alive here


def _key(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n_cols: int):
    return tuple((t.data_ptr(), t.numel(), t._version, t.device.index) for t in (row_ptr, col, val)) \
        + (int(n_cols),)


def register(g: CsrGraph) -> CsrGraph:
    """Make `g` the graph the ops use for its three tensors (while the caller keeps it).
    Skipped while torch.compile traces (the op then finds the graph an eager call registered,
    or makes one from the tensors)."""
    if not torch.compiler.is_compiling():
        _LIVE[_key(g.row_ptr, g.col, g.val, g.shape[1])] = g
    return g


def graph_of(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, n_cols: int) -> CsrGraph:
    k = _key(row_ptr, col, val, n_cols)
    g = _LIVE.get(k)
    if g is not None:
        return g
    hit = _OWNED.get(k)
    if hit is not None:
        return hit[0]
    # Not registered eagerly (e.g. an operand first seen under torch.compile, or one dropped
    # before backward): a fresh CsrGraph re-derives its plans and transpose on first use —
    # seconds of host work and GBs of device memory on a G100M-sized operand. Say so.
    import warnings
    nbytes = sum(t.numel() * t.element_size() for t in (row_ptr, col, val))
    warnings.warn(f"gnnrec: operand ({row_ptr.numel() - 1} rows, {col.numel()} nnz) was not "
                  "registered through functional.spmm / lightgcn_propagate; building a new "
                  "CsrGraph (its tiled plan and transpose are rebuilt on first use)",
                  RuntimeWarning, stacklevel=2)
    while _OWNED and (len(_OWNED) >= _OWNED_MAX or
                      sum(v[2] for v in _OWNED.values()) + nbytes > _OWNED_MAX_BYTES):
        _OWNED.pop(next(iter(_OWNED)))          # oldest first
    g = CsrGraph(row_ptr, col, val, (row_ptr.numel() - 1, int(n_cols)))
    _OWNED[k] = (g, (row_ptr, col, val), nbytes)
    return g


def _hold(ctx, row_ptr, col, val, n_cols) -> None:
    """Keep the forward's CsrGraph (its cached transpose and plans) alive until backward: a
    model called with a temporary graph (`m(g.to(dev))`) drops it before backward, which
    would then rebuild it from the raw tensors (graph_of's warning)."""
    ctx.graph = None
    if not torch.compiler.is_compiling():
        try:
            ctx.graph = _LIVE.get(_key(row_ptr, col, val, n_cols))
        except RuntimeError:   # fake / functional tensors (AOT tracing): nothing to hold
            ctx.graph = None


def _revive(ctx) -> None:
    if getattr(ctx, "graph", None) is not None:
        register(ctx.graph)


# ---- gnnrec::spmm -------------------------------------------------------------------------
@torch.library.custom_op("gnnrec::spmm", mutates_args=(), device_types="cuda")
def spmm_op(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, x: torch.Tensor,
            n_cols: int) -> torch.Tensor:
    from .functional import spmm_forward
    return spmm_forward(graph_of(row_ptr, col, val, n_cols), x)


@spmm_op.register_fake
def _spmm_fake(row_ptr, col, val, x, n_cols):
    return x.new_empty((row_ptr.shape[0] - 1, x.shape[1]))


def _spmm_setup(ctx, inputs, output):
    row_ptr, col, val, _x, n_cols = inputs
    ctx.save_for_backward(row_ptr, col, val)
    ctx.n_cols = n_cols
    _hold(ctx, row_ptr, col, val, n_cols)


def _spmm_backward(ctx, g):
    row_ptr, col, val = ctx.saved_tensors
    _revive(ctx)
    return None, None, None, torch.ops.gnnrec.spmm_t(row_ptr, col, val, g, ctx.n_cols), None


@torch.library.custom_op("gnnrec::spmm_t", mutates_args=(), device_types="cuda")
def spmm_t_op(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, g: torch.Tensor,
              n_cols: int) -> torch.Tensor:
    """A^T g: the gradient of gnnrec::spmm (the transpose is built once per operand and
    cached; the symmetric normalised operand is its own transpose)."""
    from .functional import spmm_forward
    a = graph_of(row_ptr, col, val, n_cols)
    if a.shard_info is not None:
        raise NotImplementedError("backward through a row shard: use ops.distributed")
    return spmm_forward(a.t(), g.contiguous())


@spmm_t_op.register_fake
def _spmm_t_fake(row_ptr, col, val, g, n_cols):
    return g.new_empty((n_cols, g.shape[1]))


spmm_op.register_autograd(_spmm_backward, setup_context=_spmm_setup)


# ---- gnnrec::lightgcn_propagate -----------------------------------------------------------
@torch.library.custom_op("gnnrec::lightgcn_propagate", mutates_args=(), device_types="cuda")
def lightgcn_op(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, x0: torch.Tensor,
                n_cols: int, n_layers: int, need: Optional[torch.Tensor] = None) -> torch.Tensor:
    from .functional import lightgcn_forward, lightgcn_forward_rows
    a = graph_of(row_ptr, col, val, n_cols)
    if need is not None:
        return lightgcn_forward_rows(a, x0, n_layers, need)
    out, _ = lightgcn_forward(a, x0, n_layers)
    return out


@lightgcn_op.register_fake
def _lightgcn_fake(row_ptr, col, val, x0, n_cols, n_layers, need=None):
    return x0.new_empty(x0.shape)


def _lightgcn_setup(ctx, inputs, output):
    row_ptr, col, val, _x0, n_cols, n_layers, _need = inputs
    ctx.save_for_backward(row_ptr, col, val)
    ctx.n_cols, ctx.n_layers = n_cols, n_layers
    _hold(ctx, row_ptr, col, val, n_cols)


def _lightgcn_backward(ctx, g):
    row_ptr, col, val = ctx.saved_tensors
    _revive(ctx)
    gx = torch.ops.gnnrec.lightgcn_propagate_t(row_ptr, col, val, g, ctx.n_cols, ctx.n_layers)
    return None, None, None, gx, None, None, None


@torch.library.custom_op("gnnrec::lightgcn_propagate_t", mutates_args=(), device_types="cuda")
def lightgcn_t_op(row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, g: torch.Tensor,
                  n_cols: int, n_layers: int) -> torch.Tensor:
    """mean_k (A^T)^k g: the gradient of gnnrec::lightgcn_propagate (functional.lightgcn_backward,
    its first hops skipping the all-zero rows of the sparse incoming gradient)."""
    from .functional import lightgcn_backward
    return lightgcn_backward(graph_of(row_ptr, col, val, n_cols), g, n_layers)


@lightgcn_t_op.register_fake
def _lightgcn_t_fake(row_ptr, col, val, g, n_cols, n_layers):
    return g.new_empty(g.shape)


lightgcn_op.register_autograd(_lightgcn_backward, setup_context=_lightgcn_setup)
