"""§8f3 on-device operand construction: gnnrec_build_bipartite_csr_device +
gnnrec_normalize_values_device must reproduce the host builder (itself pinned bit-exact to the
reference's scipy operand by tests/test_native_host.py) bit for bit."""
import numpy as np
import pytest
import torch

from conftest import load_golden

from src.ops import CsrGraph

pytestmark = pytest.mark.gpu


def _same(a: CsrGraph, b: CsrGraph):
    assert a.shape == b.shape and a.nnz == b.nnz
    np.testing.assert_array_equal(a.row_ptr.cpu().numpy(), b.row_ptr.cpu().numpy())
    np.testing.assert_array_equal(a.col.cpu().numpy(), b.col.cpu().numpy())
    np.testing.assert_array_equal(a.val.cpu().numpy().view(np.uint32),
                                  b.val.cpu().numpy().view(np.uint32))


@pytest.mark.parametrize("name", ["g_small", "g_dup", "g_selfloop", "g_iso"])
@pytest.mark.parametrize("binary", [False, True])
def test_device_builder_matches_host_on_golden_graphs(cuda, name, binary):
    g = load_golden(f"graph_{name}")
    args = (g["users"], g["items"], int(g["n_users"]), int(g["n_items"]))
    kw = dict(self_loop=bool(g["self_loop"]), binary=binary)
    dev = CsrGraph.from_interactions_device(*args, device=cuda, **kw)
    host = CsrGraph.from_interactions(*args, **kw)
    _same(dev, host)
    if not binary:  # and with the reference's own values
        ref = CsrGraph.from_scipy(
            __import__("scipy.sparse", fromlist=["coo_matrix"]).coo_matrix(
                (g["val"], (g["row"], g["col"])), shape=dev.shape))
        np.testing.assert_array_equal(dev.val.cpu().numpy().view(np.uint32),
                                      ref.val.numpy().view(np.uint32))


@pytest.mark.parametrize("norm", ["symmetric", "row", "none"])
def test_device_builder_random_with_duplicates(cuda, norm):
    rng = np.random.default_rng(5)
    nu, ni = 5000, 3000
    u = rng.integers(0, nu, 200_000)
    i = np.minimum(rng.zipf(1.3, 200_000) - 1, ni - 1)     # heavy duplicates on hot items
    dev = CsrGraph.from_interactions_device(u, i, nu, ni, normalization=norm, device=cuda)
    host = CsrGraph.from_interactions(u, i, nu, ni, normalization=norm)
    _same(dev, host)


def test_device_builder_edge_cases(cuda):
    e = CsrGraph.from_interactions_device(np.zeros(0, np.int64), np.zeros(0, np.int64), 3, 2,
                                          device=cuda)
    assert e.nnz == 0 and e.row_ptr.cpu().tolist() == [0] * 6
    s = CsrGraph.from_interactions_device(np.zeros(0, np.int64), np.zeros(0, np.int64), 3, 2,
                                          self_loop=True, device=cuda)
    _same(s, CsrGraph.from_interactions(np.zeros(0), np.zeros(0), 3, 2, self_loop=True))
    with pytest.raises(ValueError, match="out of range"):
        CsrGraph.from_interactions_device([0, 1, 7], [0, 1, 1], 3, 2, device=cuda)


def test_device_built_operand_drives_the_hop(cuda):
    from src.ops import functional as F
    import oracle
    g = load_golden("graph_g_small")
    dev = CsrGraph.from_interactions_device(g["users"], g["items"], int(g["n_users"]),
                                            int(g["n_items"]), device=cuda)
    x = torch.randn(dev.shape[0], 64) * 0.1
    out, _ = F.lightgcn_forward(dev, x.to(cuda), 3)
    ref = oracle.lightgcn(dev.row_ptr.cpu().numpy(), dev.col.cpu().numpy(),
                          dev.val.cpu().numpy(), x.numpy(), 3)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
