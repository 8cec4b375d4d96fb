"""Models of the real-shape reference fixtures (tests/golden/make_golden.py: make_ml1m_models,
make_gat_heavy), rebuilt by the drop-in classes: seeded construction (the reference's RNG
order, pinned by the embedding-table hashes) plus the fixture's layer weights. Shared by the
CPU checks (tests/test_real_shapes.py) and the GPU parity tests (tests/test_real_shapes_gpu.py).
"""
import numpy as np
import torch

from conftest import load_golden, sha256
from src.models import GAT, NGCF, NGCFGroupShuffle, OrthogonalBundleGNN
from src.ops import CsrGraph


def ml1m_graph() -> CsrGraph:
    """Config 2's ML-1M-shaped graph (rows up to 5 857 neighbours), host CSR."""
    f = load_golden("lightgcn_ml1m_K3_d64")
    return CsrGraph.from_interactions(f["users"].astype(np.int64), f["items"].astype(np.int64),
                                      int(f["n_users"]), int(f["n_items"]))


def _emb_hashes(m):
    return [sha256(m.user_embedding.weight.detach().numpy()),
            sha256(m.item_embedding.weight.detach().numpy())]


def _load_ngcf_layers(m, f):
    with torch.no_grad():
        for li, L in enumerate(m.layers):
            L.W1.weight.copy_(torch.from_numpy(f[f"W1_{li}"]))
            L.W1.bias.copy_(torch.from_numpy(f[f"b1_{li}"]))
            L.W2.weight.copy_(torch.from_numpy(f[f"W2_{li}"]))
            L.W2.bias.copy_(torch.from_numpy(f[f"b2_{li}"]))


def ngcf_ml1m(gas: bool = False):
    """(model, fixture): the reference's NGCF K=3 d=64 (gas=False, ngcf_ml1m_d64) or NGCF +
    GAS composed from the reference's layers (gas=True, ngcf_gas_ml1m_d64) on the ML-1M graph."""
    f = load_golden("ngcf_gas_ml1m_d64" if gas else "ngcf_ml1m_d64")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    torch.manual_seed(int(f["seed"]))
    kw = dict(embedding_dim=64, layer_sizes=[64, 64, 64], dropout=0.1, init_scale=0.1)
    m = NGCFGroupShuffle(nu, ni, **kw) if gas else NGCF(nu, ni, **kw)
    assert _emb_hashes(m) == list(f["emb_sha256"]), "seeded init drifted from the reference"
    _load_ngcf_layers(m, f)
    if gas:
        with torch.no_grad():
            for li, gs in enumerate(m.gs_layers):
                for p, s in zip(gs.skew_params, f[f"gs_skew_{li}"]):
                    p.copy_(torch.from_numpy(s))
                gs.perm.copy_(torch.from_numpy(f[f"gs_perm_{li}"]))
    return m.eval(), f


def ob_ml1m():
    """(model, fixture): the reference's OrthogonalBundleGNN (adjacency path, parallel
    transport) on the ML-1M graph (ob_ml1m_d64)."""
    f = load_golden("ob_ml1m_d64")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    torch.manual_seed(int(f["seed"]))
    m = OrthogonalBundleGNN(nu, ni, embedding_dim=64, n_layers=3, block_size=8,
                            residual_alpha=0.1, dropout=0.0, init_scale=0.1,
                            use_parallel_transport=True)
    assert _emb_hashes(m) == list(f["emb_sha256"]), "seeded init drifted from the reference"
    with torch.no_grad():
        m.layer_weights.copy_(torch.from_numpy(f["layer_weights"]))
        for li in range(3):
            gs, bc = m.local_transform_layers[li], m.connection_layers[li]
            for p, s in zip(gs.skew_params, f[f"gs_skew_{li}"]):
                p.copy_(torch.from_numpy(s))
            for p, s in zip(bc.skew_params, f[f"bc_skew_{li}"]):
                p.copy_(torch.from_numpy(s))
            assert np.array_equal(gs.perm.numpy(), f[f"gs_perm_{li}"])
            assert np.array_equal(bc.shuffle_perm.numpy(), f[f"bc_perm_{li}"])
    return m.eval(), f


def gat_heavy():
    """(model, fixture, graph): the reference's dense GAT K=3 d=64, 4 heads on the power-law
    graph whose longest rows (up to 2 992 neighbours) exceed GAT_HEAVY_THRESHOLD
    (gat_heavy_d64_h4)."""
    f = load_golden("gat_heavy_d64_h4")
    nu, ni = int(f["n_users"]), int(f["n_items"])
    torch.manual_seed(int(f["seed"]))
    m = GAT(nu, ni, embedding_dim=64, n_layers=3, n_heads=4, dropout=0.1, alpha=0.2,
            init_scale=0.1)
    for li, L in enumerate(m.layers):
        assert np.array_equal(np.stack([w.weight.detach().numpy() for w in L.W]), f[f"W_{li}"])
        assert np.array_equal(np.stack([a.detach().numpy()[:, 0] for a in L.a_self]),
                              f[f"a_self_{li}"])
    g = CsrGraph.from_interactions(f["users"].astype(np.int64), f["items"].astype(np.int64),
                                   nu, ni)
    return m.eval(), f, g
