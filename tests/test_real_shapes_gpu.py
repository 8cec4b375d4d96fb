"""BASELINE configs 3 and 5 pinned to the reference ITSELF at real shapes, on the GPU:

* NGCF K=3 d=64, NGCF + GAS and OrthogonalBundleGNN on config 2's ML-1M-shaped graph (rows of
  up to 5 857 neighbours) — tests/golden/{ngcf,ngcf_gas,ob}_ml1m_d64.npz, made by the
  reference's NGCF / NGCFLayer + GroupShuffleLayer / OrthogonalBundleGNN. Every native form of
  a layer runs: the split form on the row-parallel CSR hop (heavy-row kernel included), the
  split form on the column-ordered hop forced onto this operand (the path config 3 takes at
  G100M), and the single-kernel form.
* GAT d=64, 4 heads, K=3 on a min-degree-1 power-law graph whose longest rows (2 500 - 2 992
  neighbours) exceed GAT_HEAVY_THRESHOLD, so config 5's segment + merge kernels run —
  tests/golden/gat_heavy_d64_h4.npz, the reference's dense [N, N] masked softmax; and each
  head of a layer against the oracle's float64 restatement (oracle.gat_head).

Tolerances are fp32 reassociation (MKL's summation order is not reproducible): 1e-5 relative
on NGCF's O(1) outputs, 1e-4 relative on OB's and GAT's O(0.01) ones."""
import numpy as np
import pytest
import torch

import oracle
from real_shapes import gat_heavy, ml1m_graph, ngcf_ml1m, ob_ml1m
from src.ops import functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g_ml1m(cuda):
    return ml1m_graph().to(cuda)


def force_tiled(monkeypatch):
    """Take the column-ordered hop on this operand (below TILED_MIN_ROWS, rows above
    TILED_MAX_DEGREE): the hop config 3 runs at G100M."""
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    monkeypatch.setattr(F, "TILED_MAX_DEGREE", 1 << 30)


@pytest.mark.parametrize("gas", [False, True])
@pytest.mark.parametrize("mode", ["split_csr", "split_tiled", "single_kernel"])
def test_ngcf_ml1m_matches_reference(cuda, g_ml1m, monkeypatch, gas, mode):
    if mode == "split_tiled":
        force_tiled(monkeypatch)
        assert F.tiled_plan_for(g_ml1m, torch.empty(g_ml1m.shape[0], 64, device=cuda)) is not None
    m, f = ngcf_ml1m(gas)
    m = m.to(cuda)
    for L in m.layers:
        L.single_kernel = mode == "single_kernel"
    with torch.no_grad():
        u, i = m(g_ml1m)
    out = torch.cat([u, i]).cpu().numpy()[f["rows"]]
    np.testing.assert_allclose(out, f["out_rows"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", ["split_csr", "split_tiled"])
def test_ob_ml1m_matches_reference(cuda, g_ml1m, monkeypatch, mode):
    if mode == "split_tiled":
        force_tiled(monkeypatch)
    m, f = ob_ml1m()
    m = m.to(cuda)
    with torch.no_grad():
        u, i = m(adj_matrix=g_ml1m)
        layers = m.get_layer_embeddings(adj_matrix=g_ml1m)
    rows = f["rows"]
    np.testing.assert_allclose(torch.cat([u, i]).cpu().numpy()[rows], f["out_rows"], rtol=1e-4,
                               atol=1e-7)
    for k in range(4):
        np.testing.assert_allclose(layers[k].cpu().numpy()[rows], f["layers_rows"][k],
                                   rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("threshold", [2048, 64, 0])
def test_gat_heavy_rows_match_reference(cuda, monkeypatch, threshold):
    """The whole model: rows > threshold through the segment + merge kernels (2048: the
    shipped bucket — 3 rows; 64: hundreds of rows, most segments merged; 0: no split)."""
    monkeypatch.setattr(F, "GAT_HEAVY_THRESHOLD", threshold)
    m, f, g = gat_heavy()
    g = g.to(cuda)
    if threshold:
        assert g.heavy_plan(threshold, F.gat_knobs(g.n_rows)[1]) is not None
    m = m.to(cuda)
    with torch.no_grad():
        u, i = m(g)
    np.testing.assert_allclose(u.cpu().numpy(), f["user_out"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(i.cpu().numpy(), f["item_out"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("threshold", [2048, 64])
@pytest.mark.parametrize("segment", [1024, 100])
def test_gat_heavy_heads_match_oracle(cuda, monkeypatch, threshold, segment):
    """One layer's aggregation head by head against oracle.gat_head (float64), on the
    projections of the model's first (concat) and last (head-averaged, shared-row) layers,
    with the heavy rows split at `threshold` into `segment`-edge segments."""
    monkeypatch.setattr(F, "GAT_SEGMENT", segment)
    m, _, g = gat_heavy()
    gd = g.to(cuda)
    m = m.to(cuda)
    rp, col = g.row_ptr.numpy(), g.col.numpy()
    x = m._initial_table().detach()
    with torch.no_grad():
        for layer in (m.layers[0], m.layers[-1]):
            H = layer.n_heads
            feat, ss, sn = layer.native_inputs(x)
            shared = layer.shares_input()
            o = layer.in_dim if shared else layer.out_dim
            z = F.gat_aggregate(gd, feat, ss, sn, H, o, layer.alpha, mean_heads=False,
                                shared_rows=shared, heavy_threshold=threshold)
            fh, ssh, snh = feat.cpu().numpy(), ss.cpu().numpy(), sn.cpu().numpy()
            zh = z.cpu().numpy()
            for h in range(H):
                hf = fh if shared else fh[:, h * o:(h + 1) * o]
                ref = oracle.gat_head(rp, col, hf, ssh[:, h], snh[:, h], layer.alpha)
                np.testing.assert_allclose(zh[:, h * o:(h + 1) * o], ref, rtol=1e-4, atol=1e-6,
                                           err_msg=f"head {h}")
