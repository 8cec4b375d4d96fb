"""The drop-in model classes on a ROCm device: the native kernels behind the reference's
model API give the reference's outputs (bit-exact for LightGCN, 1e-5 otherwise)."""
import numpy as np
import pytest
import torch

from conftest import golden_csr, load_golden
from test_models import load_ob

from src.models import GAT, NGCF, LightGCN, NGCFGroupShuffle
from src.ops import CsrGraph, uses_native

pytestmark = pytest.mark.gpu


def golden_graph(cuda, name="g_small"):
    rp, col, val, nu, ni = golden_csr(name)
    return CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                    (rp.size - 1, rp.size - 1), nu, ni, True).to(cuda)


def bits(t):
    return t.detach().cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("operand", ["csr", "torch_coo"])
def test_lightgcn_model_bit_exact(cuda, operand):
    f = load_golden("lightgcn_K3_d64")
    torch.manual_seed(100 + 3 * 7 + 64)
    m = LightGCN(300, 500, embedding_dim=64, n_layers=3, init_scale=0.1).to(cuda).eval()
    g = golden_graph(cuda)
    adj = g if operand == "csr" else g.to_torch_sparse_coo()  # reference-style operand on GPU
    assert uses_native(adj)
    with torch.no_grad():
        u, i = m.get_all_embeddings(adj)
        layers = m.get_layer_embeddings(adj)
    np.testing.assert_array_equal(bits(u), f["user_out"].view(np.uint32))
    np.testing.assert_array_equal(bits(i), f["item_out"].view(np.uint32))
    for k in range(4):
        np.testing.assert_array_equal(bits(layers[k]), f["layers"][k].view(np.uint32))
    s = m.predict(torch.arange(5, device=cuda), torch.arange(5, device=cuda), adj)
    ref = (torch.from_numpy(f["user_out"][:5]) * torch.from_numpy(f["item_out"][:5])).sum(1)
    np.testing.assert_allclose(s.detach().cpu().numpy(), ref.numpy(), rtol=0, atol=1e-7)


def test_lightgcn_model_training_grads(cuda):
    f = load_golden("lightgcn_grad_K3_d64")
    torch.manual_seed(7)
    m = LightGCN(300, 500, embedding_dim=64, n_layers=3, init_scale=0.1).to(cuda)
    u, i = m(golden_graph(cuda))
    g_u = torch.from_numpy(f["g_u"]).to(cuda)
    g_i = torch.from_numpy(f["g_i"]).to(cuda)
    ((u * g_u).sum() + (i * g_i).sum()).backward()
    np.testing.assert_allclose(m.user_embedding.weight.grad.cpu().numpy(), f["grad_user"],
                               rtol=0, atol=1e-6)
    np.testing.assert_allclose(m.item_embedding.weight.grad.cpu().numpy(), f["grad_item"],
                               rtol=0, atol=1e-6)


def ngcf_from_golden(f, cuda):
    torch.manual_seed(11)
    m = NGCF(300, 500, embedding_dim=64, layer_sizes=[64, 64, 64], dropout=0.1, init_scale=0.01)
    with torch.no_grad():
        for li, L in enumerate(m.layers):
            L.W1.bias.copy_(torch.from_numpy(f[f"b1_{li}"]))
            L.W2.bias.copy_(torch.from_numpy(f[f"b2_{li}"]))
    return m.to(cuda).eval()


def test_ngcf_model_fused(cuda):
    f = load_golden("ngcf_d64")
    m = ngcf_from_golden(f, cuda)
    with torch.no_grad():
        u, i = m(golden_graph(cuda))
    np.testing.assert_allclose(u.cpu().numpy(), f["user_out"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(i.cpu().numpy(), f["item_out"], rtol=0, atol=1e-5)


def test_ngcf_model_training_path(cuda):
    """With autograd on: native SpMM (differentiable) + torch Linear, same outputs."""
    f = load_golden("ngcf_d64")
    m = ngcf_from_golden(f, cuda)
    u, i = m(golden_graph(cuda))
    np.testing.assert_allclose(u.detach().cpu().numpy(), f["user_out"], rtol=0, atol=1e-5)
    (u.sum() + i.sum()).backward()
    assert m.layers[0].W1.weight.grad is not None
    assert torch.isfinite(m.user_embedding.weight.grad).all()


def test_ngcf_group_shuffle_fused_vs_composed(cuda):
    torch.manual_seed(3)
    m = NGCFGroupShuffle(300, 500, embedding_dim=64, layer_sizes=[64, 64, 64], dropout=0.1,
                         gs_init_scale=0.3).eval()
    rp, col, val, nu, ni = golden_csr("g_small")
    cpu_adj = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                       (rp.size - 1, rp.size - 1), nu, ni, True).to_torch_sparse_coo()
    with torch.no_grad():
        ref_u, ref_i = m(cpu_adj)             # composed torch path on the CPU
        m = m.to(cuda)
        u, i = m(golden_graph(cuda))          # one fused kernel per layer
    np.testing.assert_allclose(u.cpu().numpy(), ref_u.numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(i.cpu().numpy(), ref_i.numpy(), rtol=0, atol=1e-5)


def test_orthogonal_bundle_model_fused(cuda):
    f = load_golden("ob_d64")
    m = load_ob(f).to(cuda).eval()
    g = golden_graph(cuda)
    with torch.no_grad():
        u, i = m(adj_matrix=g)
        layers = m.get_layer_embeddings(adj_matrix=g)
    np.testing.assert_allclose(u.cpu().numpy(), f["user_out"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(i.cpu().numpy(), f["item_out"], rtol=0, atol=1e-5)
    for k in range(4):
        np.testing.assert_allclose(layers[k].cpu().numpy(), f["layers"][k], rtol=0, atol=1e-5)


@pytest.mark.parametrize("pt", [0, 1])
def test_orthogonal_bundle_edge_index_path(cuda, pt):
    """use_edge_index=True with and without parallel transport (model.py:160-181, 215-220)
    against the reference's own output (tests/golden/ob_edge_index_pt*_d64.npz): the edge list
    becomes a cached CSR of edge multiplicities, one native SpMM (+ MFMA transform) per layer."""
    from test_models import load_ob_edge
    from src.models.orthogonal_bundle.parallel_transport import _EDGE_CACHE
    m, f, ei = load_ob_edge(pt)
    m = m.to(cuda)
    _EDGE_CACHE.clear()
    ei = ei.to(cuda)
    with torch.no_grad():
        u, i = m(edge_index=ei)
        layers = m.get_layer_embeddings(edge_index=ei)
    assert len(_EDGE_CACHE) == 1                       # the native edge operand was used
    np.testing.assert_allclose(u.cpu().numpy(), f["user_out"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(i.cpu().numpy(), f["item_out"], rtol=2e-5, atol=2e-5)
    for k in range(4):
        np.testing.assert_allclose(layers[k].cpu().numpy(), f["layers"][k], rtol=2e-5, atol=2e-5)


def test_gat_model_sparse(cuda):
    f = load_golden("gat_d64_h4")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    torch.manual_seed(42)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.1, alpha=0.2,
            init_scale=0.1).to(cuda).eval()
    g = CsrGraph.from_interactions(f["users"], f["items"], nu, ni).to(cuda)
    with torch.no_grad():
        u, i = m(g)
    np.testing.assert_allclose(u.cpu().numpy(), f["user_out"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(i.cpu().numpy(), f["item_out"], rtol=0, atol=2e-5)


def test_gat_refuses_dense_fallback_on_large_graph(cuda, monkeypatch):
    """With the native training path off (GAT_NATIVE_TRAIN; it also does not apply to a
    non-symmetric pattern or an unsupported width), a native operand with autograd on falls
    back to the reference's [N, N] path (gat.py:124-137 of the reference): when that would not
    fit the device's free memory the layer raises instead of allocating it (N = 2e5: ~2 TB
    with autograd), and on a small graph it warns and runs it. Under no_grad it runs
    natively."""
    from src.models.baselines import gat as gat_mod
    monkeypatch.setattr(gat_mod, "GAT_NATIVE_TRAIN", False)
    nu = ni = 100_000
    rng = np.random.default_rng(0)
    # every node has a neighbour (an isolated node is a NaN row by design)
    u = np.concatenate([np.arange(nu), rng.integers(0, nu, ni), rng.integers(0, nu, 4 * nu)])
    i = np.concatenate([rng.integers(0, ni, nu), np.arange(ni), rng.integers(0, ni, 4 * nu)])
    g = CsrGraph.from_interactions(u, i, nu, ni).to(cuda)
    torch.manual_seed(0)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.0).to(cuda).eval()
    with pytest.raises(RuntimeError, match="softmax path would need"):
        m(g)                                       # grad enabled, parameters require grad
    before = torch.cuda.max_memory_allocated(cuda)
    with torch.no_grad():
        uo, io = m(g)
    assert uo.shape == (nu, 64) and torch.isfinite(uo).all() and torch.isfinite(io).all()
    assert torch.cuda.max_memory_allocated(cuda) - before < (nu + ni) ** 2  # no [N, N] buffer
    small = CsrGraph.from_interactions([0, 1, 2, 0], [0, 1, 2, 1], 3, 3).to(cuda)
    ms = GAT(3, 3, embedding_dim=16, n_layers=2, n_heads=4, dropout=0.0).to(cuda)
    with pytest.warns(RuntimeWarning, match="dense O\\(N\\^2\\)"):
        us, _ = ms(small)
    us.sum().backward()                            # the dense path is differentiable
    assert ms.layers[0].W[0].weight.grad is not None


def test_gat_isolated_node_row_is_nan_only_locally(cuda):
    torch.manual_seed(0)
    m = GAT(4, 3, embedding_dim=16, n_layers=2, n_heads=4, dropout=0.0).to(cuda).eval()
    g = CsrGraph.from_interactions([0, 1, 2, 0], [0, 1, 2, 1], 4, 3).to(cuda)  # user 3 isolated
    with torch.no_grad():
        u, i = m(g)
    assert torch.isnan(u[3]).all()
    assert torch.isfinite(u[:3]).all() and torch.isfinite(i).all()


@pytest.mark.parametrize("threshold", [0, 5, 40])
def test_gat_heavy_row_split_matches_unsplit(cuda, threshold):
    """Power-law rows: the segment/merge path equals the one-pass path (fp32 tolerance)."""
    from src.ops import functional as F
    rng = np.random.default_rng(3)
    nu, ni = 50, 400
    u = np.concatenate([rng.integers(0, nu, 3000), np.zeros(390, np.int64), np.arange(nu)])
    i = np.concatenate([rng.integers(0, ni, 3000), np.arange(390), rng.integers(0, ni, nu)])
    g = CsrGraph.from_interactions(u, i, nu, ni).to(cuda)
    N = g.shape[0]
    for heads, o, mean in [(4, 16, False), (4, 64, True), (2, 8, False)]:
        h = torch.randn(N, heads * o, device=cuda)
        ss, sn = torch.randn(N, heads, device=cuda), torch.randn(N, heads, device=cuda)
        ref = F.gat_aggregate(g, h, ss, sn, heads, o, 0.2, mean, True, heavy_threshold=0)
        got = F.gat_aggregate(g, h, ss, sn, heads, o, 0.2, mean, True,
                              heavy_threshold=threshold or 10 ** 9)
        if threshold:
            assert g.heavy_plan(threshold, F.gat_knobs(g.n_rows)[1]) is not None
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    # and with a segment length smaller than the rows
    old = F.GAT_SEGMENT
    try:
        F.GAT_SEGMENT = 7
        got = F.gat_aggregate(g, h, ss, sn, heads, o, 0.2, False, False, heavy_threshold=20)
        ref = F.gat_aggregate(g, h, ss, sn, heads, o, 0.2, False, False, heavy_threshold=0)
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    finally:
        F.GAT_SEGMENT = old


@pytest.mark.parametrize("heavy", [0, 64])
def test_gat_shared_rows_equals_replicated_table(cuda, heavy):
    """head_stride 0 (every head aggregates the same x row) == the head-major table holding
    x once per head, bit for bit, on the normal and the heavy-row split path."""
    from src.ops import functional as F
    rng = np.random.default_rng(9)
    u = rng.integers(0, 300, 6000)
    i = np.minimum(rng.zipf(1.3, 6000) - 1, 199)
    g = CsrGraph.from_interactions(u, i, 300, 200).to(cuda)
    n, H, o = g.shape[0], 4, 64
    x = torch.randn(n, o, device=cuda) * 0.1
    ss, sn = torch.randn(n, H, device=cuda), torch.randn(n, H, device=cuda)
    z = F.gat_aggregate(g, x, ss, sn, H, o, 0.2, shared_rows=True, heavy_threshold=heavy)
    zr = F.gat_aggregate(g, x.repeat(1, H), ss, sn, H, o, 0.2, heavy_threshold=heavy)
    assert torch.isnan(z).any()                      # never-drawn items: empty rows -> NaN
    np.testing.assert_array_equal(z.cpu().numpy().view(np.uint32), zr.cpu().numpy().view(np.uint32))


def test_edge_specific_transport_native(cuda):
    """§8f4 on the GPU against the reference's EdgeSpecificBundleConnection + bmm transport
    (tests/golden/edge_specific_d64.npz): one CSR + SpMM/MFMA transform per edge type, no
    [E, d, d] tensor."""
    from test_models import load_edge_specific
    esbc, f = load_edge_specific()
    esbc = esbc.to(cuda)
    with torch.no_grad():
        out = esbc.transport(torch.from_numpy(f["x"]).to(cuda),
                             torch.from_numpy(f["edge_index"]).to(cuda),
                             torch.from_numpy(f["edge_type"]).to(cuda))
    assert out.is_cuda
    np.testing.assert_allclose(out.cpu().numpy(), f["y"], rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("shared", [False, True])
def test_gat_scores_read_in_place_with_row_strides(cuda, shared):
    """s_self / s_neigh as column views of a wider table (the projection's output) give the
    same bits as compacted copies, on the normal and the heavy-row path."""
    from src.ops import functional as F
    rng = np.random.default_rng(4)
    u = rng.integers(0, 300, 6000)
    i = np.minimum(rng.zipf(1.3, 6000) - 1, 199)
    g = CsrGraph.from_interactions(u, i, 300, 200).to(cuda)
    n, H, o = g.shape[0], 4, (64 if shared else 16)
    feat = torch.randn(n, o if shared else H * o, device=cuda)
    wide = torch.randn(n, 72, device=cuda)
    ss, sn = wide[:, 64:68], wide[:, 68:72]
    for heavy in (0, 64):
        got = F.gat_aggregate(g, feat, ss, sn, H, o, 0.2, shared_rows=shared, heavy_threshold=heavy)
        ref = F.gat_aggregate(g, feat, ss.contiguous(), sn.contiguous(), H, o, 0.2,
                              shared_rows=shared, heavy_threshold=heavy)
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32),
                                      ref.cpu().numpy().view(np.uint32))
