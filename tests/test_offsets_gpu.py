"""int64 nonzero offsets past 2^31 (G1B's operand holds ~2e9 nonzeros).

The ABI passes row_ptr as ABSOLUTE int64 offsets into col / val (include/gnnrec.h: row_ptr[0]
need not be 0). Shifting row_ptr up by OFF >= 2^31 and the col / val base pointers down by the
same OFF addresses exactly the same nonzeros, so every kernel that indexes col / val must give
the same bits as on the unshifted operand — which it only does if no offset is truncated to
32 bits on the way (row_ptr -> col/val indexing in spmm.hip, gat.hip). No 8 GB operand needed.
"""
import numpy as np
import pytest
import torch

import oracle
from src.ops import CsrGraph, _lib
from src.ops import functional as F

pytestmark = pytest.mark.gpu

OFF = (1 << 31) + 4096          # a multiple of 4: the same 16-B alignment as the real index


@pytest.fixture(scope="module")
def case(cuda):
    rng = np.random.default_rng(23)
    nu, ni = 900, 700
    # power-law items, a hub user with 600 items, every node at least one edge
    u = np.concatenate([rng.integers(0, nu, 30000), np.zeros(600, np.int64), np.arange(nu),
                        rng.integers(0, nu, ni)])
    i = np.concatenate([np.minimum(rng.zipf(1.4, 30000) - 1, ni - 1), np.arange(600),
                        rng.integers(0, ni, nu), np.arange(ni)])
    g = CsrGraph.from_interactions(u, i, nu, ni)
    deg = np.diff(g.row_ptr.numpy())
    assert deg.max() > 600 and deg.min() >= 1
    gd = g.to(cuda)
    rp_shift = (gd.row_ptr + OFF).contiguous()
    col_p = gd.col.data_ptr() - 4 * OFF
    val_p = gd.val.data_ptr() - 4 * OFF
    return g, gd, rp_shift, col_p, val_p


def _stream(cuda):
    return _lib.stream_of(cuda)


def bits(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("heavy", [0, 64])
@pytest.mark.parametrize("d", [64, 128])
def test_spmm_split_with_shifted_offsets(cuda, case, heavy, d):
    """gnnrec_spmm_csr_split_f32: row-parallel kernel (+ the workgroup-per-row heavy kernel
    at threshold 64) on row_ptr + 2^31, with the fused layer-mean epilogue."""
    g, gd, rp_shift, col_p, val_p = case
    L = _lib.lib()
    n = g.shape[0]
    x = torch.randn(n, d, device=cuda) * 0.1
    hr = gd.heavy_rows(heavy) if heavy else None
    nh = 0 if hr is None else hr.numel()
    outs = []
    for rp, cp, vp in ((gd.row_ptr.data_ptr(), gd.col.data_ptr(), gd.val.data_ptr()),
                       (rp_shift.data_ptr(), col_p, val_p)):
        y = torch.empty(n, d, device=cuda)
        acc = torch.empty(n, d, device=cuda)
        _lib.check(L.gnnrec_spmm_csr_split_f32(rp, cp, vp, n, x.data_ptr(), d, y.data_ptr(), d, d,
                                               _lib.EPI_ACC_INIT, x.data_ptr(), d, acc.data_ptr(),
                                               d, 1.0, _lib.ptr(hr), nh, heavy if nh else 0,
                                               _stream(cuda)), "spmm_csr_split")
        outs.append((y, acc))
    torch.cuda.synchronize()
    assert np.array_equal(bits(outs[0][0]), bits(outs[1][0]))
    assert np.array_equal(bits(outs[0][1]), bits(outs[1][1]))
    ref = oracle.spmm(g.row_ptr.numpy(), g.col.numpy(), g.val.numpy(), x.cpu().numpy())
    assert np.array_equal(bits(outs[1][0]), ref.view(np.uint32))


def test_masked_hop_and_mark_rows_with_shifted_offsets(cuda, case):
    """gnnrec_spmm_csr_masked_f32 (sparse input, row subset) and gnnrec_mark_active_rows."""
    g, gd, rp_shift, col_p, val_p = case
    L = _lib.lib()
    n, d = g.shape[0], 64
    x = torch.zeros(n, d, device=cuda)
    x[::37] = torch.randn(x[::37].shape, device=cuda)
    xm = F.row_nonzero(x)
    outs = []
    for rp, cp, vp in ((gd.row_ptr.data_ptr(), gd.col.data_ptr(), gd.val.data_ptr()),
                       (rp_shift.data_ptr(), col_p, val_p)):
        act = torch.empty(n, dtype=torch.uint8, device=cuda)
        _lib.check(L.gnnrec_mark_active_rows(rp, cp, n, xm.data_ptr(), n, act.data_ptr(),
                                             _stream(cuda)), "mark_active_rows")
        y = torch.empty(n, d, device=cuda)
        _lib.check(L.gnnrec_spmm_csr_masked_f32(rp, cp, vp, n, x.data_ptr(), d, xm.data_ptr(),
                                                act.data_ptr(), y.data_ptr(), d, d, 0, None, d,
                                                None, d, 1.0, None, 0, 0, _stream(cuda)),
                   "spmm_csr_masked")
        outs.append((act, y))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and int(outs[1][0].sum()) > 0
    assert np.array_equal(bits(outs[0][1]), bits(outs[1][1]))


def test_fused_lightgcn_with_shifted_offsets(cuda, case):
    """gnnrec_lightgcn_split_f32 (K hops + layer mean in one call) on row_ptr + 2^31."""
    g, gd, rp_shift, col_p, val_p = case
    L = _lib.lib()
    n, d, K = g.shape[0], 64, 3
    x0 = torch.randn(n, d, device=cuda) * 0.1
    hr = gd.heavy_rows(64)
    outs = []
    for rp, cp, vp in ((gd.row_ptr.data_ptr(), gd.col.data_ptr(), gd.val.data_ptr()),
                       (rp_shift.data_ptr(), col_p, val_p)):
        w0, w1, out = (torch.empty(n, d, device=cuda) for _ in range(3))
        _lib.check(L.gnnrec_lightgcn_split_f32(rp, cp, vp, n, x0.data_ptr(), d, K, w0.data_ptr(),
                                               w1.data_ptr(), None, out.data_ptr(), d,
                                               hr.data_ptr(), hr.numel(), 64, _stream(cuda)),
                   "lightgcn_split")
        outs.append(out)
    torch.cuda.synchronize()
    assert np.array_equal(bits(outs[0]), bits(outs[1]))
    ref = oracle.lightgcn(g.row_ptr.numpy(), g.col.numpy(), g.val.numpy(), x0.cpu().numpy(), K)
    assert np.array_equal(bits(outs[1]), ref.view(np.uint32))


@pytest.mark.parametrize("shared", [False, True])
def test_gat_light_and_heavy_with_shifted_offsets(cuda, case, shared):
    """gnnrec_gat_aggregate_f32 (light rows) + gnnrec_gat_heavy_f32 (segments of the rows
    above 200, their CSR ranges shifted too) on row_ptr + 2^31, against the unshifted call
    (same bits) and oracle.gat_head."""
    g, gd, rp_shift, col_p, _ = case
    L = _lib.lib()
    n, H = g.shape[0], 4
    o = 64 if shared else 16
    feat = torch.randn(n, o if shared else H * o, device=cuda) * 0.1
    ss, sn = torch.randn(n, H, device=cuda), torch.randn(n, H, device=cuda)
    thr = 200
    plan = gd.heavy_plan(thr, 64)
    assert plan is not None
    n_seg = plan["seg_row"].numel()
    outs = []
    for shift in (0, OFF):
        rp = gd.row_ptr.data_ptr() if not shift else rp_shift.data_ptr()
        cp = gd.col.data_ptr() - 4 * shift
        out = torch.empty(n, H * o, device=cuda)
        common = (feat.data_ptr(), feat.stride(0), 0 if shared else o, ss.data_ptr(),
                  sn.data_ptr(), H, H, H, o, 0.2, 0, 0, out.data_ptr(), H * o, 0, None, H * o,
                  None, H * o, 1.0)
        _lib.check(L.gnnrec_gat_aggregate_f32(rp, cp, n, *common, thr, _stream(cuda)),
                   "gat_aggregate")
        sb = (plan["seg_beg"] + shift).contiguous()
        se = (plan["seg_end"] + shift).contiguous()
        work = torch.empty(n_seg * (H * o + 2 * H) + 4, device=cuda)
        _lib.check(L.gnnrec_gat_heavy_f32(cp, plan["seg_row"].data_ptr(), sb.data_ptr(),
                                          se.data_ptr(), n_seg, plan["heavy_rows"].data_ptr(),
                                          plan["heavy_seg_ptr"].data_ptr(),
                                          plan["heavy_rows"].numel(), work.data_ptr(), *common,
                                          _stream(cuda)), "gat_heavy")
        torch.cuda.synchronize()
        outs.append(out)
    assert np.array_equal(bits(outs[0]), bits(outs[1]))
    fh, ssh, snh, z = feat.cpu().numpy(), ss.cpu().numpy(), sn.cpu().numpy(), outs[1].cpu().numpy()
    for h in range(H):
        hf = fh if shared else fh[:, h * o:(h + 1) * o]
        ref = oracle.gat_head(g.row_ptr.numpy(), g.col.numpy(), hf, ssh[:, h], snh[:, h], 0.2)
        np.testing.assert_allclose(z[:, h * o:(h + 1) * o], ref, rtol=1e-4, atol=1e-6)
