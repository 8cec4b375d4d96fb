"""torch.library registration of the propagation ops (src/ops/library.py): the ops exist with
their schemas, their fake kernels give the right shapes, and FakeTensor tracing (what
torch.compile / torch.export do) records them as single graph nodes. The GPU half —
torch.library.opcheck on the real kernels, autograd through them and the models dispatching
through them — is tests/test_library_gpu.py."""
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.proxy_tensor import make_fx

from src import ops  # noqa: F401  (registers torch.ops.gnnrec.*)


def _operand(n=10, nnz=25, d=16):
    rp = torch.linspace(0, nnz, n + 1).to(torch.int64)
    col = torch.randint(0, n, (nnz,), dtype=torch.int32)
    val = torch.rand(nnz)
    x = torch.randn(n, d)
    return rp, col, val, x


def test_ops_are_registered_with_schemas():
    s = str(torch.ops.gnnrec.spmm.default._schema)
    assert s.startswith("gnnrec::spmm(Tensor row_ptr, Tensor col, Tensor val, Tensor x, SymInt n_cols)") \
        or s.startswith("gnnrec::spmm(Tensor row_ptr, Tensor col, Tensor val, Tensor x, int n_cols)")
    s = str(torch.ops.gnnrec.lightgcn_propagate.default._schema)
    assert "n_layers" in s and "Tensor? need=None" in s


def test_fake_kernels_give_output_shapes():
    with FakeTensorMode() as mode:
        rp, col, val, x = (mode.from_tensor(t) for t in _operand())
        assert torch.ops.gnnrec.spmm(rp, col, val, x, 10).shape == (10, 16)
        assert torch.ops.gnnrec.lightgcn_propagate(rp, col, val, x, 10, 3).shape == (10, 16)


def test_fake_tracing_keeps_the_ops_as_nodes():
    def f(rp, col, val, x):
        y = torch.ops.gnnrec.spmm(rp, col, val, x, 10)
        return torch.ops.gnnrec.lightgcn_propagate(rp, col, val, y * 2, 10, 3).sum()

    gm = make_fx(f, tracing_mode="fake")(*_operand())
    targets = [str(n.target) for n in gm.graph.nodes if n.op == "call_function"]
    assert "gnnrec.spmm.default" in targets
    assert "gnnrec.lightgcn_propagate.default" in targets


def test_no_cpu_kernel():
    """A CPU operand never reaches these ops silently: there is no CPU kernel (the model
    layer routes CPU torch-sparse operands to torch.sparse.mm, as the reference)."""
    import pytest
    with pytest.raises(NotImplementedError):
        torch.ops.gnnrec.spmm(*_operand(), 10)
