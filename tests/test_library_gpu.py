"""The registered ops on the GPU: torch.library.opcheck (schema, fake kernel, autograd
registration, AOT dispatch), gradients equal to the explicit transpose-SpMM / the reference's
autograd, and the models reaching the native kernels through torch.ops.gnnrec.*."""
import numpy as np
import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

import oracle
from src import ops
from src.models import LightGCN, NGCF
from src.ops import CsrGraph, functional as F

pytestmark = pytest.mark.gpu


def _graph(cuda, seed=0, nu=400, ni=300, n=5000):
    rng = np.random.default_rng(seed)
    g = CsrGraph.from_interactions(rng.integers(0, nu, n), rng.integers(0, ni, n), nu, ni)
    return g.to(cuda), g, nu, ni


def test_opcheck_spmm(cuda):
    g, _, _, _ = _graph(cuda)
    x = torch.randn(g.shape[0], 64, device=cuda, requires_grad=True)
    torch.library.opcheck(torch.ops.gnnrec.spmm.default, (g.row_ptr, g.col, g.val, x, g.shape[1]))


def test_opcheck_lightgcn(cuda):
    g, _, _, _ = _graph(cuda, 1)
    x = torch.randn(g.shape[0], 32, device=cuda, requires_grad=True)
    torch.library.opcheck(torch.ops.gnnrec.lightgcn_propagate.default,
                          (g.row_ptr, g.col, g.val, x, g.shape[1], 3))


def test_op_values_and_gradients(cuda):
    g, gh, _, _ = _graph(cuda, 2)
    x = (torch.randn(g.shape[0], 64, generator=torch.Generator().manual_seed(0)) * 0.1)
    xd = x.to(cuda).requires_grad_(True)
    y = torch.ops.gnnrec.spmm(g.row_ptr, g.col, g.val, xd, g.shape[1])
    ref = oracle.spmm(gh.row_ptr.numpy(), gh.col.numpy(), gh.val.numpy(), x.numpy())
    np.testing.assert_array_equal(y.detach().cpu().numpy().view(np.uint32), ref.view(np.uint32))
    w = torch.randn_like(y)
    (y * w).sum().backward()
    # the symmetric normalised operand: dX = A^T W = A W
    gref = F.spmm_forward(g.t(), w)
    assert torch.equal(xd.grad, gref)
    # the LightGCN op against torch autograd over torch.sparse.mm (the reference's path)
    xd.grad = None
    out = torch.ops.gnnrec.lightgcn_propagate(g.row_ptr, g.col, g.val, xd, g.shape[1], 3)
    (out * w).sum().backward()
    a = g.to_torch_sparse_coo()
    xr = x.to(cuda).requires_grad_(True)
    layers, h = [xr], xr
    for _ in range(3):
        h = torch.sparse.mm(a, h)
        layers.append(h)
    (torch.stack(layers).mean(0) * w).sum().backward()
    torch.testing.assert_close(xd.grad, xr.grad, rtol=0, atol=1e-6)


class _Seen(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = set()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        self.ops.add(str(func))
        return func(*args, **(kwargs or {}))


def test_models_dispatch_through_registered_ops(cuda):
    g, _, nu, ni = _graph(cuda, 3)
    torch.manual_seed(0)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1).to(cuda)
    seen = _Seen()
    with seen:
        u, i = m(g)
        (u.sum() + i.sum()).backward()
    assert "gnnrec.lightgcn_propagate.default" in seen.ops
    assert m.user_embedding.weight.grad is not None
    n = NGCF(nu, ni, 64, [64, 64, 64], 0.1, 0.1).to(cuda).train()
    seen = _Seen()
    with seen:
        u, i = n(g)
        u.sum().backward()
    assert "gnnrec.spmm.default" in seen.ops


def test_compile_traces_the_op(cuda):
    g, _, _, _ = _graph(cuda, 4)
    x = torch.randn(g.shape[0], 64, device=cuda)

    def f(x):
        return ops.spmm(g, x * 2.0) + 1.0

    eager = f(x)
    compiled = torch.compile(f, backend="aot_eager", fullgraph=True)(x)
    assert torch.equal(eager, compiled)


def test_temporary_graph_survives_until_backward(cuda):
    """m(g.to(dev)) drops the device graph before backward: the op's autograd context keeps
    it (and its cached transpose / plans), so backward finds it instead of rebuilding one
    from the raw tensors (graph_of's RuntimeWarning)."""
    import warnings
    _, g_host, nu, ni = _graph(cuda, 4)
    torch.manual_seed(0)
    m = LightGCN(nu, ni, embedding_dim=64, n_layers=3, init_scale=0.1).to(cuda)
    n = NGCF(nu, ni, 64, [64, 64, 64], 0.1, 0.1).to(cuda).train()
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        u, i = m(g_host.to(cuda))
        (u.sum() + i.sum()).backward()
        u, i = n(g_host.to(cuda))
        u.sum().backward()
    assert m.user_embedding.weight.grad is not None
