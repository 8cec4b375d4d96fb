"""Model classes on the CPU: drop-in construction (same parameters for the same seed as the
reference, pinned by the goldens) and the reference CPU path (torch sparse operand) giving
the reference's outputs. No GPU needed."""
import numpy as np
import pytest
import torch

from conftest import golden_csr, load_golden

from src.models import GAT, NGCF, LightGCN, OrthogonalBundleGNN
from src.models.orthogonal_bundle import BundleConnectionLayer, GroupShuffleLayer
from src.ops import CsrGraph


def torch_adj(name="g_small"):
    rp, col, val, nu, ni = golden_csr(name)
    g = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                 (rp.size - 1, rp.size - 1), nu, ni, True)
    return g.to_torch_sparse_coo(), nu, ni


@pytest.mark.parametrize("K,d", [(1, 32), (2, 64), (3, 64), (3, 128)])
def test_lightgcn_seeded_init_matches_reference(K, d):
    f = load_golden(f"lightgcn_K{K}_d{d}")
    torch.manual_seed(100 + K * 7 + d)
    m = LightGCN(300, 500, embedding_dim=d, n_layers=K, init_scale=0.1)
    np.testing.assert_array_equal(m.user_embedding.weight.detach().numpy(), f["user_w"])
    np.testing.assert_array_equal(m.item_embedding.weight.detach().numpy(), f["item_w"])


def test_lightgcn_cpu_reference_path():
    f = load_golden("lightgcn_K3_d64")
    torch.manual_seed(100 + 3 * 7 + 64)
    m = LightGCN(300, 500, embedding_dim=64, n_layers=3, init_scale=0.1).eval()
    adj, _, _ = torch_adj()
    with torch.no_grad():
        u, i = m(adj)
        layers = m.get_layer_embeddings(adj)
    np.testing.assert_array_equal(u.numpy(), f["user_out"])
    np.testing.assert_array_equal(i.numpy(), f["item_out"])
    for k in range(4):
        np.testing.assert_array_equal(layers[k].numpy(), f["layers"][k])
    with pytest.raises(ValueError):
        m.predict(torch.tensor([0]), torch.tensor([0]))


def test_ngcf_seeded_init_and_cpu_path():
    f = load_golden("ngcf_d64")
    torch.manual_seed(11)
    m = NGCF(300, 500, embedding_dim=64, layer_sizes=[64, 64, 64], dropout=0.1, init_scale=0.01)
    np.testing.assert_array_equal(m.user_embedding.weight.detach().numpy(), f["user_w"])
    for li, L in enumerate(m.layers):
        np.testing.assert_array_equal(L.W1.weight.detach().numpy(), f[f"W1_{li}"])
        np.testing.assert_array_equal(L.W2.weight.detach().numpy(), f[f"W2_{li}"])
        with torch.no_grad():
            L.W1.bias.copy_(torch.from_numpy(f[f"b1_{li}"]))
            L.W2.bias.copy_(torch.from_numpy(f[f"b2_{li}"]))
    m.eval()
    adj, _, _ = torch_adj()
    with torch.no_grad():
        u, i = m(adj)
    np.testing.assert_allclose(u.numpy(), f["user_out"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(i.numpy(), f["item_out"], rtol=0, atol=1e-6)


def load_ob(f):
    torch.manual_seed(31)
    m = OrthogonalBundleGNN(300, 500, embedding_dim=64, n_layers=3, block_size=8,
                            residual_alpha=0.1, dropout=0.0, init_scale=0.01,
                            use_parallel_transport=True)
    with torch.no_grad():
        m.layer_weights.copy_(torch.tensor([0.3, -0.2, 0.5, 0.1]))
        for L in list(m.local_transform_layers) + list(m.connection_layers):
            for p in L.skew_params:
                p.mul_(20.0)
    return m


def test_ob_seeded_init_and_cpu_path():
    f = load_golden("ob_d64")
    m = load_ob(f)
    np.testing.assert_array_equal(m.user_embedding.weight.detach().numpy(), f["user_w"])
    for li in range(3):
        gs, bc = m.local_transform_layers[li], m.connection_layers[li]
        np.testing.assert_array_equal(np.stack([p.detach().numpy() for p in gs.skew_params]),
                                      f[f"gs_skew_{li}"])
        np.testing.assert_array_equal(gs.perm.numpy(), f[f"gs_perm_{li}"])
        np.testing.assert_array_equal(np.stack([p.detach().numpy() for p in bc.skew_params]),
                                      f[f"bc_skew_{li}"])
        np.testing.assert_array_equal(bc.shuffle_perm.numpy(), f[f"bc_perm_{li}"])
    m.eval()
    adj, _, _ = torch_adj()
    with torch.no_grad():
        u, i = m(adj_matrix=adj)
        layers = m.get_layer_embeddings(adj_matrix=adj)
    np.testing.assert_allclose(u.numpy(), f["user_out"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(i.numpy(), f["item_out"], rtol=0, atol=1e-6)
    for k in range(4):
        np.testing.assert_allclose(layers[k].numpy(), f["layers"][k], rtol=0, atol=1e-6)


def test_gas_and_bundle_layers_match_reference():
    f = load_golden("gas_d64_bs8")
    torch.manual_seed(21)
    gs = GroupShuffleLayer(64, 8, init_scale=0.01)
    with torch.no_grad():
        for p in gs.skew_params:
            p.mul_(30.0)
        y = gs(torch.from_numpy(f["x"]))
    np.testing.assert_array_equal(gs.perm.numpy(), f["perm"])
    np.testing.assert_allclose(y.numpy(), f["y"], rtol=0, atol=1e-6)
    # torch.matrix_exp picks its CPU kernel by ISA: the golden's host and this one may differ
    # by a few ulps on the [-1, 1] block entries (measured 3e-7 on a re-created container)
    np.testing.assert_allclose(gs.blocks().detach().numpy(), f["blocks"], rtol=0, atol=1e-6)
    fro, mx = gs.get_orthogonality_metrics()
    assert fro.item() < 1e-4 and mx.item() < 1e-5
    b = load_golden("bundle_d64_bs8")
    torch.manual_seed(22)
    bc = BundleConnectionLayer(64, 8)
    with torch.no_grad():
        # W = blockdiag(matrix_exp(skew))[perm]: few-ulp CPU-ISA spread, as for GAS above
        np.testing.assert_allclose(bc().numpy(), b["W"], rtol=0, atol=1e-6)


def test_gat_seeded_init_and_cpu_path():
    f = load_golden("gat_d64_h4")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    torch.manual_seed(42)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.1, alpha=0.2,
            init_scale=0.1).eval()
    np.testing.assert_array_equal(m.user_embedding.weight.detach().numpy(), f["user_w"])
    for li, L in enumerate(m.layers):
        np.testing.assert_array_equal(np.stack([w.weight.detach().numpy() for w in L.W]),
                                      f[f"W_{li}"])
        assert int(L.concat_heads) == int(f[f"concat_{li}"])
    G = CsrGraph.from_interactions(f["users"], f["items"], nu, ni)
    with torch.no_grad():
        u, i = m(G.to_torch_sparse_coo())
    np.testing.assert_allclose(u.numpy(), f["user_out"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(i.numpy(), f["item_out"], rtol=0, atol=1e-6)


def test_cpu_csrgraph_operand_is_rejected():
    """No silent CPU fallback: a CsrGraph must live on a ROCm device."""
    g = CsrGraph.from_interactions([0, 1], [1, 0], 2, 2)
    m = LightGCN(2, 2, embedding_dim=8, n_layers=1)
    with pytest.raises(ValueError, match="ROCm"):
        m(g)


def _typed_edges(seed=0, n=200, e=3000):
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, e), generator=g)
    et = torch.randint(0, 2, (e,), generator=g)
    x = torch.randn(n, 64, generator=g) * 0.1
    return ei, et, x


def test_edge_specific_transport_cpu_matches_reference_formula():
    """§8f4: EdgeSpecificBundleConnection.transport == parallel_transport_along_edges with the
    [E, d, d] tensor its forward() builds (the reference's composition)."""
    from src.models.orthogonal_bundle import EdgeSpecificBundleConnection
    from src.models.orthogonal_bundle.parallel_transport import parallel_transport_along_edges
    torch.manual_seed(4)
    esbc = EdgeSpecificBundleConnection(64, 8)
    ei, et, x = _typed_edges()
    with torch.no_grad():
        ref = parallel_transport_along_edges(x, ei, esbc(ei, et))
        out = esbc.transport(x, ei, et)
    torch.testing.assert_close(out, ref, rtol=0, atol=1e-6)


def test_predict_serving_cache_tracks_parameters():
    """predict() in eval/no-grad reuses the propagated tables until a parameter changes."""
    rp, col, val, nu, ni = golden_csr("g_small")
    g = CsrGraph(torch.from_numpy(rp), torch.from_numpy(col), torch.from_numpy(val),
                 (rp.size - 1, rp.size - 1), nu, ni, True)
    adj = g.to_torch_sparse_coo()
    torch.manual_seed(0)
    m = LightGCN(nu, ni, 32, 2, 0.1).eval()
    users, items = torch.tensor([0, 5, 7]), torch.tensor([1, 2, 3])
    with torch.no_grad():
        a = m.predict(users, items, adj)
        assert m._serving_cache is not None
        b = m.predict(users, items, adj)
        assert torch.equal(a, b)
        m.user_embedding.weight.add_(0.5)          # in-place update: cache must refresh
        c = m.predict(users, items, adj)
        ue, ie = m.get_all_embeddings(adj)
    assert torch.equal(c, (ue[users] * ie[items]).sum(1)) and not torch.equal(a, c)


def load_ob_edge(pt: int):
    """OrthogonalBundleGNN(use_edge_index=True) seeded as in make_golden.make_edge_paths;
    returns (model, golden, edge_index). The seeded construction must reproduce the
    reference's parameters exactly (same RNG order)."""
    f = load_golden(f"ob_edge_index_pt{pt}_d64")
    torch.manual_seed(int(f["seed"]))
    m = OrthogonalBundleGNN(300, 500, embedding_dim=64, n_layers=3, block_size=8,
                            residual_alpha=0.1, dropout=0.0, init_scale=0.01,
                            use_parallel_transport=bool(pt), use_edge_index=True)
    with torch.no_grad():
        m.layer_weights.copy_(torch.tensor([0.3, -0.2, 0.5, 0.1]))
        conn = list(m.connection_layers) if pt else []
        for L in list(m.local_transform_layers) + conn:
            for p in L.skew_params:
                p.mul_(20.0)
    np.testing.assert_array_equal(m.user_embedding.weight.detach().numpy(), f["user_w"])
    np.testing.assert_array_equal(m.item_embedding.weight.detach().numpy(), f["item_w"])
    for li in range(3):
        gs = m.local_transform_layers[li]
        np.testing.assert_array_equal(np.stack([p.detach().numpy() for p in gs.skew_params]),
                                      f[f"gs_skew_{li}"])
        np.testing.assert_array_equal(gs.perm.numpy(), f[f"gs_perm_{li}"])
        if pt:
            bc = m.connection_layers[li]
            np.testing.assert_array_equal(np.stack([p.detach().numpy() for p in bc.skew_params]),
                                          f[f"bc_skew_{li}"])
            np.testing.assert_array_equal(bc.shuffle_perm.numpy(), f[f"bc_perm_{li}"])
    return m.eval(), f, torch.from_numpy(f["edge_index"])


def load_edge_specific():
    """EdgeSpecificBundleConnection seeded as make_golden.make_edge_paths (params checked)."""
    from src.models.orthogonal_bundle import EdgeSpecificBundleConnection
    f = load_golden("edge_specific_d64")
    torch.manual_seed(71)
    esbc = EdgeSpecificBundleConnection(64, 8, n_edge_types=2)
    with torch.no_grad():
        for L in esbc.connection_layers:
            for p in L.skew_params:
                p.mul_(20.0)
    for t, L in enumerate(esbc.connection_layers):
        np.testing.assert_array_equal(np.stack([p.detach().numpy() for p in L.skew_params]),
                                      f["skew"][t])
        np.testing.assert_array_equal(L.shuffle_perm.numpy(), f["perm"][t])
    return esbc, f


@pytest.mark.parametrize("pt", [0, 1])
def test_ob_edge_index_cpu_matches_reference(pt):
    """use_edge_index=True (model.py:160-181, 215-220): golden from the reference itself."""
    m, f, ei = load_ob_edge(pt)
    with torch.no_grad():
        u, i = m(edge_index=ei)
        layers = m.get_layer_embeddings(edge_index=ei)
    # the transport matrices come from torch.matrix_exp, whose CPU kernel (and so its last
    # ulps) depends on the host ISA; after 3 layers that spreads to ~5e-6 on O(1) values.
    # north_star's tolerance for embeddings is 1e-4.
    np.testing.assert_allclose(u.numpy(), f["user_out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(i.numpy(), f["item_out"], rtol=1e-5, atol=1e-5)
    for k in range(4):
        np.testing.assert_allclose(layers[k].numpy(), f["layers"][k], rtol=1e-5, atol=1e-5)


def test_edge_specific_cpu_matches_reference():
    """EdgeSpecificBundleConnection (bundle_layer.py:106-149) + the bmm transport
    (parallel_transport.py:37-43): both forward() + the torch transport and transport()
    against the reference's output."""
    from src.models.orthogonal_bundle.parallel_transport import parallel_transport_along_edges
    esbc, f = load_edge_specific()
    ei, et = torch.from_numpy(f["edge_index"]), torch.from_numpy(f["edge_type"])
    x = torch.from_numpy(f["x"])
    with torch.no_grad():
        # matrix_exp's CPU kernel is host-ISA dependent (few ulps)
        np.testing.assert_allclose(esbc.type_matrices().numpy(), f["W_types"], rtol=0, atol=1e-6)
        ref_path = parallel_transport_along_edges(x, ei, esbc(ei, et))
        out = esbc.transport(x, ei, et)
    np.testing.assert_allclose(ref_path.numpy(), f["y"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out.numpy(), f["y"], rtol=1e-5, atol=1e-5)


def test_rows_gemm_guards_on_host():
    """rows_gemm has no torch fallback: host tensors and mismatched shapes raise before any
    native call; GAT picks the native row GEMM only for shapes it has an instance for."""
    from src.ops import functional as F
    from src.models.baselines.gat import GATLayer
    with pytest.raises(ValueError):
        F.rows_gemm(torch.randn(8, 64), torch.randn(64, 8))          # x on the host
    with pytest.raises(ValueError):
        F.rows_gemm(torch.randn(8, 64), torch.randn(32, 8))          # B rows != k
    assert F.rows_gemm_supported(64, 72) and F.rows_gemm_supported(128, 64)
    assert not F.rows_gemm_supported(64, 84) and not F.rows_gemm_supported(32, 8)
    assert not F.rows_gemm_supported(128, 136) and not F.rows_gemm_supported(64, 6)
    # last (head-mean) layer of a 128-wide GAT: H * in = 512 has no instance -> not shared
    assert not GATLayer(128, 128, 4, concat_heads=False).shares_input()
    assert GATLayer(64, 64, 4, concat_heads=False).shares_input()


def test_gat_dense_fallback_guard(monkeypatch):
    """A native operand that the sparse kernel cannot take falls back to the reference's dense
    [N, N] softmax only when its estimated footprint fits the available memory (with a
    warning), and raises otherwise; a node cap (GNNREC_GAT_DENSE_MAX_NODES) replaces the
    memory test when set (the old fixed 20K cap refused graphs a 288 GB device
    runs). The reason is reported."""
    from src.models.baselines import gat as gat_mod
    from src.models.baselines.gat import (GATLayer, check_dense_fallback,
                                          dense_fallback_bytes)
    monkeypatch.delenv("GNNREC_GAT_DENSE_MAX_NODES", raising=False)
    assert dense_fallback_bytes(1000, 4, grad=True) == 4 * 10**6 * 13
    assert dense_fallback_bytes(1000, 4, grad=False) == 4 * 10**6 * 4
    with pytest.raises(RuntimeError, match="dense \\[N, N\\] softmax path would need"):
        check_dense_fallback(10**7, "autograd", heads=4, grad=True)       # 5.2 PB
    with pytest.warns(RuntimeWarning, match="dense O\\(N\\^2\\)"):
        check_dense_fallback(100, "autograd", heads=4, grad=True)
    monkeypatch.setenv("GNNREC_GAT_DENSE_MAX_NODES", "50")
    with pytest.raises(RuntimeError, match="node cap GNNREC_GAT_DENSE_MAX_NODES = 50"):
        check_dense_fallback(100, "autograd")
    with pytest.warns(RuntimeWarning):
        check_dense_fallback(50, "autograd")
    monkeypatch.delenv("GNNREC_GAT_DENSE_MAX_NODES")
    monkeypatch.setattr(gat_mod, "GAT_DENSE_MAX_NODES", 10)
    with pytest.raises(RuntimeError, match="node cap"):
        check_dense_fallback(11, "autograd")
    layer = GATLayer(64, 16, 4)
    g = CsrGraph(torch.tensor([0, 1, 2]), torch.tensor([1, 0], dtype=torch.int32),
                 torch.ones(2), (2, 2), 1, 1, True)
    assert "autograd" in layer.native_block(g)
    with torch.no_grad():
        assert layer.native_block(g) is None
        layer.train()
        layer.dropout = 0.1
        assert "dropout" in layer.native_block(g)
    assert layer.native_block(torch.zeros(2, 2)) == "not a native operand"


def test_gat_sampled_row_checker_matches_reference_dense_layer():
    """The config-5 sampled-row checker (oracle/gat_sample.py) is itself pinned to the
    reference layer semantics: at a row sample, layer_rows equals GATLayer's dense masked
    softmax path (the reference's gat.py:92-151, run here on the CPU) + F.elu, for a concat and
    a head-averaged layer; sub_csr cuts exactly the sampled rows."""
    import oracle.gat_sample as gs
    from src.models.baselines.gat import GATLayer
    rng = np.random.default_rng(2)
    nu, ni = 120, 90
    u = np.concatenate([np.arange(nu), rng.integers(0, nu, ni), rng.integers(0, nu, 1500)])
    i = np.concatenate([rng.integers(0, ni, nu), np.arange(ni), rng.integers(0, ni, 1500)])
    g = CsrGraph.from_interactions(u, i, nu, ni)
    deg = np.diff(g.row_ptr.numpy())
    rows = gs.sample_rows(deg, n_heavy=5, per_decile=7, seed=0)
    assert np.all(np.isin(np.argsort(-deg)[:5], rows))
    rp_sub, col_sub = gs.sub_csr(g.row_ptr, g.col, rows)
    for j, r in enumerate(rows):
        np.testing.assert_array_equal(col_sub[rp_sub[j]:rp_sub[j + 1]],
                                      g.col.numpy()[g.row_ptr[r]:g.row_ptr[r + 1]])
    torch.manual_seed(0)
    x = torch.randn(nu + ni, 32) * 0.3
    A = g.to_torch_sparse_coo()
    for concat, out_dim in ((True, 8), (False, 32)):
        layer = GATLayer(32, out_dim, 4, 0.0, 0.2, concat_heads=concat)
        for w in layer.W:
            torch.nn.init.xavier_uniform_(w.weight)
        for p in list(layer.a_self) + list(layer.a_neigh):
            torch.nn.init.xavier_uniform_(p.data)
        with torch.no_grad():
            ref = torch.nn.functional.elu(layer._dense_forward(x, A)).numpy()
        got = gs.layer_rows(layer, x, rp_sub, col_sub, rows)
        res = gs.close(got, ref[rows])
        assert res["within_tolerance"], res


def test_gat_dense_restatement_gradients_match_reference():
    """The CPU / dense path (GATLayer._dense_forward, the restatement of gat.py:92-151) trains
    like the reference: every parameter gradient of tests/golden/gat_grad_d64_h4.npz (made by
    importing the reference) within fp32 tolerance — this pins the fixture the native
    backward is checked against on the GPU."""
    f = load_golden("gat_grad_d64_h4")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    g = CsrGraph.from_interactions(f["users"], f["items"], nu, ni)
    A = g.to_torch_sparse_coo()
    torch.manual_seed(42)
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.0, alpha=0.2,
            init_scale=0.1).train()
    ue, ie = m(A)
    loss = (ue * torch.from_numpy(f["Ru"])).sum() + (ie * torch.from_numpy(f["Ri"])).sum()
    loss.backward()
    for name, prm in m.named_parameters():
        np.testing.assert_allclose(prm.grad.numpy(), f["grad." + name], rtol=1e-4, atol=1e-7,
                                   err_msg=name)
