"""GAT aggregation with the attention scores formed from the rows (ABI 10,
gnnrec_gat_aggregate_att_f32 / gnnrec_gat_heavy_att_f32) against oracle.gat_head.

The reference computes per head h = W_h x, s_self = h a_self, s_neigh = h a_neigh
(gat.py:113-118) and a masked softmax over the row's neighbours (gat.py:120-141). The ATT
kernels read only the gathered rows and form both scores as fp32 dots in registers; the
oracle gets the same scores as float64 dots of the same rows with the same vectors, then its
float64 edge softmax. Covered: head-major tables (o_dim 4..64, 1..8 heads), the shared-row
table (head_stride 0, the head-averaged layer's form; the 4-head / 64-wide fast kernel and the
generic one), head mean, ELU and the layer-mean epilogue, the heavy-row split (segments +
merge, short segments), empty rows (NaN), and the model path end to end.
"""
import numpy as np
import pytest
import torch

import oracle
from src.ops import CsrGraph
from src.ops import _lib
from src.ops import functional as F

pytestmark = pytest.mark.gpu


def _graph(cuda, seed=5, nu=300, ni=200, n=6000, iso=False):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, nu, n)
    i = np.minimum(rng.zipf(1.3, n) - 1, ni - 1)
    if not iso:   # every node has a neighbour
        u = np.concatenate([u, np.arange(nu), rng.integers(0, nu, ni)])
        i = np.concatenate([i, rng.integers(0, ni, nu), np.arange(ni)])
    g = CsrGraph.from_interactions(u, i, nu, ni)
    return g, g.to(cuda)


def _oracle(g, feat, att, heads, o, shared, slope=0.2):
    """[n, heads*o] per-head oracle aggregation with float64 scores from att."""
    rp, col = g.row_ptr.numpy(), g.col.numpy()
    f = feat.cpu().numpy()
    a = att.cpu().double().numpy()
    outs = []
    for h in range(heads):
        sl = slice(0, o) if shared else slice(h * o, (h + 1) * o)
        hf = np.ascontiguousarray(f[:, sl])
        s = hf.astype(np.float64)
        outs.append(oracle.gat_head(rp, col, hf, (s @ a[0, h]).astype(np.float32),
                                    (s @ a[1, h]).astype(np.float32), slope))
    return np.concatenate(outs, axis=1)


@pytest.mark.parametrize("heads,o", [(4, 16), (1, 64), (2, 32), (8, 8), (4, 4), (2, 16)])
@pytest.mark.parametrize("heavy", [0, 64])
def test_att_head_major_vs_oracle(cuda, heads, o, heavy):
    g, gd = _graph(cuda)
    n = g.shape[0]
    torch.manual_seed(heads * 100 + o)
    feat = torch.randn(n, heads * o, device=cuda) * 0.3
    att = torch.randn(2, heads, o, device=cuda) * 0.5
    z = F.gat_aggregate_att(gd, feat, feat, att, heads, o, 0.2, heavy_threshold=heavy)
    if heavy:
        assert gd.heavy_plan(heavy, F.gat_knobs(gd.n_rows)[1]) is not None
    np.testing.assert_allclose(z.cpu().numpy(), _oracle(g, feat, att, heads, o, False),
                               rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("heads,o", [(4, 64), (4, 32), (2, 64), (4, 16)])
@pytest.mark.parametrize("heavy", [0, 64])
def test_att_shared_rows_vs_oracle(cuda, heads, o, heavy):
    """head_stride 0: every head aggregates the same o-wide row; (4, 64) takes the 16-lane
    shared-row kernel with the DPP reduce-scatter of the 32 neighbour scores, the others the
    generic kernel."""
    g, gd = _graph(cuda, seed=7)
    n = g.shape[0]
    torch.manual_seed(o)
    x = torch.randn(n, o, device=cuda) * 0.3
    att = torch.randn(2, heads, o, device=cuda) * 0.3
    z = F.gat_aggregate_att(gd, x, x, att, heads, o, 0.2, shared_rows=True, heavy_threshold=heavy)
    np.testing.assert_allclose(z.cpu().numpy(), _oracle(g, x, att, heads, o, True),
                               rtol=1e-4, atol=1e-6)


def test_att_short_segments_and_epilogue(cuda, monkeypatch):
    """Segments shorter than the rows (GAT_SEGMENT 7, threshold 20), head mean + ELU + the
    layer-mean epilogue (ACC_INIT then ACC_ADD | DIV) against the oracle composition."""
    monkeypatch.setattr(F, "GAT_SEGMENT", 7)
    g, gd = _graph(cuda, seed=11)
    n, heads, o = g.shape[0], 4, 16
    torch.manual_seed(3)
    feat = torch.randn(n, heads * o, device=cuda) * 0.3
    att = torch.randn(2, heads, o, device=cuda) * 0.5
    ref = _oracle(g, feat, att, heads, o, False).reshape(n, heads, o).mean(axis=1)
    ref = np.where(ref > 0, ref, np.expm1(ref))
    self_rows = torch.randn(n, o, device=cuda)
    acc = torch.empty(n, o, device=cuda)
    y = F.gat_aggregate_att(gd, feat, feat, att, heads, o, 0.2, mean_heads=True, apply_elu=True,
                            epi=_lib.EPI_ACC_INIT, self_rows=self_rows, acc=acc,
                            heavy_threshold=20)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(acc.cpu().numpy(), self_rows.cpu().numpy() + ref, rtol=1e-4,
                               atol=1e-6)
    F.gat_aggregate_att(gd, feat, feat, att, heads, o, 0.2, mean_heads=True, apply_elu=True,
                        epi=_lib.EPI_ACC_ADD | _lib.EPI_ACC_DIV | _lib.EPI_NO_Y, acc=acc,
                        acc_div=4.0, heavy_threshold=20)
    np.testing.assert_allclose(acc.cpu().numpy(), (self_rows.cpu().numpy() + 2 * ref) / 4,
                               rtol=1e-4, atol=1e-6)


def test_att_hself_is_the_destination_rows_own_table(cuda):
    """hself decouples the self score from the gathered table (a shard: the gathered table is
    the exchanged padded layout, the own rows are the rank's local rows)."""
    g, gd = _graph(cuda, seed=13)
    n, heads, o = g.shape[0], 4, 16
    feat = torch.randn(n, heads * o, device=cuda)
    att = torch.randn(2, heads, o, device=cuda) * 0.3
    other = torch.randn(n, heads * o, device=cuda)
    z = F.gat_aggregate_att(gd, feat, other, att, heads, o, 0.2)
    rp, col = g.row_ptr.numpy(), g.col.numpy()
    f, oth, a = feat.cpu().numpy(), other.cpu().numpy(), att.cpu().double().numpy()
    for h in range(heads):
        sl = slice(h * o, (h + 1) * o)
        ref = oracle.gat_head(rp, col, np.ascontiguousarray(f[:, sl]),
                              (oth[:, sl].astype(np.float64) @ a[0, h]).astype(np.float32),
                              (f[:, sl].astype(np.float64) @ a[1, h]).astype(np.float32), 0.2)
        np.testing.assert_allclose(z.cpu().numpy()[:, sl], ref, rtol=1e-4, atol=1e-6)


def test_att_empty_row_is_nan(cuda):
    g, gd = _graph(cuda, seed=2, iso=True)
    deg = np.diff(g.row_ptr.numpy())
    assert (deg == 0).any()
    n = g.shape[0]
    for shared, width in ((False, 64), (True, 64)):
        feat = torch.randn(n, width, device=cuda)
        att = torch.randn(2, 4, 16 if not shared else 64, device=cuda)
        z = F.gat_aggregate_att(gd, feat, feat, att, 4, 16 if not shared else 64, 0.2,
                                shared_rows=shared).cpu().numpy()
        assert np.isnan(z[deg == 0]).all() and np.isfinite(z[deg > 0]).all()


def test_att_rejects_wide_heads(cuda):
    g, gd = _graph(cuda)
    feat = torch.randn(g.shape[0], 128, device=cuda)
    with pytest.raises(ValueError, match="unsupported"):
        F.gat_aggregate_att(gd, feat, feat, torch.zeros(2, 1, 128, device=cuda), 1, 128)


def test_att_model_forward_equals_score_table_forward(cuda, monkeypatch):
    """The model's forward through the ATT kernels (the default) against the score-table
    kernels (GAT_SCORES_FROM_ROWS off): the same layers reassociated, fp32 tolerance; both
    with the heavy split active."""
    from src.models import GAT
    from src.models.baselines import gat as gat_mod
    monkeypatch.setattr(F, "GAT_HEAVY_THRESHOLD", 64)
    g, gd = _graph(cuda, seed=17, nu=400, ni=300, n=20000)
    torch.manual_seed(0)
    m = GAT(400, 300, 64, 3, 4, 0.1, 0.2, 0.1).to(cuda).eval()
    assert all(layer.att_ok() for layer in m.layers)
    with torch.no_grad():
        ua, ia = m(gd)
        monkeypatch.setattr(gat_mod, "GAT_SCORES_FROM_ROWS", False)
        assert not any(layer.att_ok() for layer in m.layers)
        ut, it = m(gd)
    torch.testing.assert_close(ua, ut, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(ia, it, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("shared", [False, True])
def test_att_segment_order_and_xcd_blocks_keep_the_bits(cuda, monkeypatch, shared):
    """Heavy segments run sorted by their first column (heavy_plan_by_column) and/or with each
    XCD on a contiguous eighth of the list: the same segments and the same merge order, so the
    same bits as the row-grouped order."""
    monkeypatch.setattr(F, "GAT_SEGMENT", 50)
    g, gd = _graph(cuda, seed=19, nu=500, ni=400, n=40000)
    n, heads, o = g.shape[0], 4, (64 if shared else 16)
    torch.manual_seed(1)
    feat = torch.randn(n, o if shared else heads * o, device=cuda) * 0.3
    att = torch.randn(2, heads, o, device=cuda) * 0.4
    outs = {}
    for order in ("row", "column"):
        for xcd in (False, True):
            monkeypatch.setattr(F, "GAT_SEGMENT_ORDER", order)
            monkeypatch.setattr(F, "GAT_XCD_ORDER", xcd)
            outs[order, xcd] = F.gat_aggregate_att(gd, feat, feat, att, heads, o, 0.2,
                                                   shared_rows=shared, heavy_threshold=100)
    plan = gd.heavy_plan_by_column(100, 50)
    first = gd.col[plan["seg_beg"]].cpu().numpy()
    assert plan["seg_row"].numel() > 64 and np.all(np.diff(first) >= 0)
    base = outs["row", False].cpu().numpy().view(np.uint32)
    for k, v in outs.items():
        np.testing.assert_array_equal(v.cpu().numpy().view(np.uint32), base, err_msg=str(k))
    np.testing.assert_allclose(outs["column", True].cpu().numpy(),
                               _oracle(g, feat, att, heads, o, shared), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("shared", [False, True])
def test_att_panel_cut_segments_vs_oracle(cuda, monkeypatch, shared):
    """Heavy rows cut at column-panel boundaries (heavy_plan_panels: every such row's
    segments start in one panel, then sorted by first column) give the oracle's aggregation;
    every heavy edge is in exactly one segment."""
    monkeypatch.setattr(F, "GAT_SEGMENT_ORDER", "panel")
    monkeypatch.setattr(F, "GAT_PANEL", 16)
    monkeypatch.setattr(F, "GAT_PANEL_MIN_EDGES", 2)
    monkeypatch.setattr(F, "GAT_SEGMENT", 9)
    g, gd = _graph(cuda, seed=23, nu=500, ni=400, n=40000)
    n, heads, o = g.shape[0], 4, (64 if shared else 16)
    torch.manual_seed(2)
    feat = torch.randn(n, o if shared else heads * o, device=cuda) * 0.3
    att = torch.randn(2, heads, o, device=cuda) * 0.4
    z = F.gat_aggregate_att(gd, feat, feat, att, heads, o, 0.2, shared_rows=shared,
                            heavy_threshold=100)
    plan = gd.heavy_plan_panels(100, 9, 16, 2)
    assert plan["n_cut_rows"] > 0
    beg, end = plan["seg_beg"].cpu().numpy(), plan["seg_end"].cpu().numpy()
    rp = g.row_ptr.numpy()
    heavy = plan["heavy_rows"].cpu().numpy()
    assert (end - beg).sum() == (rp[heavy + 1] - rp[heavy]).sum()
    covered = np.zeros(g.nnz, np.int64)
    for b, e in zip(beg, end):
        covered[b:e] += 1
    hv = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in heavy])
    assert np.all(covered[hv] == 1)
    np.testing.assert_allclose(z.cpu().numpy(), _oracle(g, feat, att, heads, o, shared),
                               rtol=1e-4, atol=1e-6)
