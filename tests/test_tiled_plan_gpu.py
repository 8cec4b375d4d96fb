"""The device planner (gnnrec_tiled_plan_device, csrc/tiled_plan.hip) against the host
planner (gnnrec_tiled_plan_build/emit): the same slot words, values, headers, chunk offsets
and step counts, bit for bit — on uniform and power-law graphs, with and without the
sub-panel order, many small panels (many steps, empty panels skipped), short blocks, rows
longer than a panel's share, and at full G100M size; and a hop through each plan gives the
same bits."""
import numpy as np
import pytest
import torch

import oracle
from src.ops import CsrGraph, functional as F

pytestmark = pytest.mark.gpu


def _uniform(nu, ni, n, seed):
    rng = np.random.default_rng(seed)
    return CsrGraph.from_interactions(rng.integers(0, nu, n), rng.integers(0, ni, n), nu, ni,
                                      binary=True)


def _powerlaw(nu, ni, n, seed):
    rng = np.random.default_rng(seed)
    u = np.concatenate([rng.integers(0, nu, n), np.zeros(3000, np.int64)])   # a 3000-item user
    i = np.concatenate([np.minimum(rng.zipf(1.3, n) - 1, ni - 1), np.arange(3000) % ni])
    return CsrGraph.from_interactions(u, i, nu, ni, binary=True)


def _same(a, b):
    for k in ("slot", "val", "hdr", "wave_ptr", "n_steps"):
        x, y = a[k].cpu(), b[k].cpu()
        assert x.shape == y.shape, k
        assert torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x,
                           y.view(torch.int32) if y.dtype == torch.float32 else y), k
    for k in ("n_blocks", "n_chunks", "n_slots"):
        assert a[k] == b[k], k


@pytest.mark.parametrize("kind,R,panel,sub", [
    ("uniform", 1117, 49152, 4096), ("uniform", 300, 4096, 512), ("uniform", 64, 1000, 0),
    ("uniform", 1279, 2048, 100), ("powerlaw", 700, 8192, 1024), ("powerlaw", 1, 4096, 256),
    ("powerlaw", 513, 300, 0)])
def test_device_plan_equals_host_plan(cuda, kind, R, panel, sub):
    g = (_uniform(20000, 15000, 600000, 3) if kind == "uniform"
         else _powerlaw(20000, 15000, 400000, 4))
    gd = g.to(cuda)
    dev = gd._tiled_plan_device(R, panel, sub)
    host = gd._tiled_plan_host(R, panel, sub)
    for p in (dev, host):
        p["n_slots"] = p["n_chunks"] * 64
    _same(dev, host)


def test_device_plan_edge_cases(cuda):
    # empty rows at both ends and a trailing short block
    rp = torch.tensor([0, 0, 3, 3, 7, 7, 7], dtype=torch.int64)
    col = torch.tensor([0, 5, 9, 1, 2, 3, 8], dtype=torch.int32)
    val = torch.arange(1, 8, dtype=torch.float32)
    g = CsrGraph(rp, col, val, (6, 10)).to(cuda)
    for R in (1, 2, 4, 6):
        for panel, sub in ((4, 0), (4, 2), (100, 3)):
            dev = g._tiled_plan_device(R, panel, sub)
            host = g._tiled_plan_host(R, panel, sub)
            for p in (dev, host):
                p["n_slots"] = p["n_chunks"] * 64
            _same(dev, host)
    bad = CsrGraph(rp, torch.tensor([0, 5, -1, 1, 2, 3, 8], dtype=torch.int32), val,
                   (6, 10)).to(cuda)
    with pytest.raises(ValueError):
        bad._tiled_plan_device(2, 4, 0)
    with pytest.raises(ValueError):
        bad._tiled_plan_host(2, 4, 0)


def test_hop_through_device_plan_bit_exact(cuda):
    g = _uniform(60000, 50000, 3_000_000, 5)
    gd = g.to(cuda)
    x = torch.randn(g.shape[0], 64, device=cuda) * 0.1
    ref = torch.empty_like(x)
    F.TILED_HOP, was = False, F.TILED_HOP
    try:
        F.spmm_into(gd, x, ref)
    finally:
        F.TILED_HOP = was
    for planner in ("device", "host"):
        gd._plans.pop(("tiled", 700, 8192, 1024), None)
        plan = gd.tiled_plan(rows_per_block=700, panel=8192, sub_panel=1024, planner=planner)
        y = torch.empty_like(x)
        F.spmm_tiled_into(gd, x, y, plan)
        assert torch.equal(y.view(torch.int32), ref.view(torch.int32)), planner


def test_device_plan_equals_host_plan_g100m(cuda):
    import time
    import bench
    g = bench.build_graph(1_000_000, 1_000_000, 100_000_000, 0, 16)
    gd = g.to(cuda)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev = gd._tiled_plan_device(1117, 49152, 4096)
    torch.cuda.synchronize()
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    host = gd._tiled_plan_host(1117, 49152, 4096)
    t_host = time.perf_counter() - t0
    print(f"\n[plan G100M] device {t_dev:.3f} s, host {t_host:.3f} s")
    for p in (dev, host):
        p["n_slots"] = p["n_chunks"] * 64
    _same(dev, host)


def test_device_plan_retries_a_small_step_cap(cuda, monkeypatch):
    """A step larger than the scratch's step cap fails the pass (error 2) and the planner
    re-runs it with the block bound: the same arrays."""
    from src.ops import graph as G
    monkeypatch.setattr(G, "TILED_PLAN_STEP_CAP", 16)
    g = _uniform(20000, 15000, 600000, 3).to(cuda)
    dev = g._tiled_plan_device(700, 8192, 1024)
    host = g._tiled_plan_host(700, 8192, 1024)
    for p in (dev, host):
        p["n_slots"] = p["n_chunks"] * 64
    _same(dev, host)


def test_quad_plan_layout_is_padding_plus_permutation(cuda):
    """CsrGraph._quad_plan (the layout of a GNNREC_TILED_QUAD kernel build): every wave's
    chunk range is padded to a multiple of 4 with empty chunks (scratch row, header 0), the
    slots of 4 chunks are interleaved per lane, the headers stay chunk-major, and the real
    chunks are exactly the chunk-major plan's, in order."""
    from src.ops import _lib
    rng = np.random.default_rng(4)
    g = CsrGraph.from_interactions(rng.integers(0, 3000, 60000), rng.integers(0, 2000, 60000),
                                   3000, 2000).to(cuda)
    R = 333
    plan = g._tiled_plan_host(R, 4096, 512)
    plan.update(rows_per_block=R)
    std = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in plan.items()}
    CsrGraph._quad_plan(plan)
    W, CH = _lib.TILED_WAVES, _lib.TILED_CHUNK
    wp_old, wp = std["wave_ptr"].cpu().numpy(), plan["wave_ptr"].cpu().numpy()
    assert np.all(np.diff(wp) % 4 == 0) and np.all(wp % 4 == 0)
    total = int(wp[-1])
    assert plan["n_chunks"] == total and plan["slot"].numel() == (total + 16) * CH
    slot = plan["slot"].view(-1, CH, 4).transpose(1, 2).reshape(-1, CH).cpu().numpy()
    val = plan["val"].view(-1, CH, 4).transpose(1, 2).reshape(-1, CH).cpu().numpy()
    hdr = plan["hdr"].view(-1, 4).cpu().numpy()
    s_old = std["slot"].view(-1, CH).cpu().numpy()
    v_old = std["val"].view(-1, CH).cpu().numpy()
    h_old = std["hdr"].view(-1, 4).cpu().numpy()
    for w in range(wp_old.size - 1):
        a, b = wp_old[w], wp_old[w + 1]
        na = wp[w]
        np.testing.assert_array_equal(slot[na:na + b - a], s_old[a:b])
        np.testing.assert_array_equal(val[na:na + b - a], v_old[a:b])
        np.testing.assert_array_equal(hdr[na:na + b - a], h_old[a:b])
        pad = slice(na + b - a, wp[w + 1])
        assert np.all(slot[pad] == R) and np.all(hdr[pad] == 0) and np.all(val[pad] == 0)
    assert np.all(slot[total:] == R) and np.all(hdr[total:] == 0)
    # a factored plan's class bytes move the same way
    g2 = CsrGraph.from_interactions(rng.integers(0, 3000, 60000), rng.integers(0, 2000, 60000),
                                    3000, 2000, binary=True).to(cuda)
    p2 = g2._tiled_plan_device(R, 4096, 512)
    p2.update(rows_per_block=R)
    assert g2._factor_plan(p2)
    c_old = p2["cls"].view(-1, CH).cpu().numpy().copy()
    w2 = p2["wave_ptr"].cpu().numpy().copy()
    CsrGraph._quad_plan(p2)
    cls = p2["cls"].view(-1, CH, 4).transpose(1, 2).reshape(-1, CH).cpu().numpy()
    wq = p2["wave_ptr"].cpu().numpy()
    for w in range(w2.size - 1):
        n = w2[w + 1] - w2[w]
        np.testing.assert_array_equal(cls[wq[w]:wq[w] + n], c_old[w2[w]:w2[w + 1]])
        assert np.all(cls[wq[w] + n:wq[w + 1]] == 0)


def test_chunk_major_plan_on_quad_build_is_flagged(cuda):
    """a raw-ABI caller passing the planner's chunk-major arrays to a quad-layout
    build gets the error word set (sync[GNNREC_TILED_SYNC_ERR_WORD]; the launch's rows are then
    undefined, gnnrec.h), and the Python wrapper refuses such a plan before launching."""
    from src.ops import _lib
    L = _lib.lib()
    if not L.gnnrec_tiled_plan_quad():
        pytest.skip("chunk-major build")
    rng = np.random.default_rng(6)
    g = CsrGraph.from_interactions(rng.integers(0, 3000, 60000), rng.integers(0, 2000, 60000),
                                   3000, 2000).to(cuda)
    R = 333
    plan = g._tiled_plan_host(R, 4096, 512)
    plan.update(rows_per_block=R)
    wp = plan["wave_ptr"].cpu().numpy()
    assert np.any(wp % 4 != 0)          # this plan has ranges a quad build would misread
    # a quad build prefetches up to 12 chunks past a wave's range: give the chunk-major
    # arrays the quad layout's tail so no load leaves them
    pad = _lib.TILED_QUAD_TAIL * _lib.TILED_CHUNK
    for k, n in (("slot", pad), ("val", pad), ("hdr", _lib.TILED_QUAD_TAIL * 4)):
        plan[k] = torch.cat([plan[k], torch.zeros(n, dtype=plan[k].dtype, device=cuda)])
    x = torch.randn(g.shape[0], 32, device=cuda)
    y = torch.full_like(x, 7.0)
    with pytest.raises(ValueError, match="layout"):
        F.spmm_tiled_into(g, x, y, plan)
    sync = torch.zeros(_lib.TILED_SYNC_WORDS, dtype=torch.int32, device=cuda)
    _lib.check(L.gnnrec_spmm_tiled_f32(
        _lib.ptr(plan["slot"]), _lib.ptr(plan["val"]), 0, 0, 0, 0, _lib.ptr(plan["hdr"]),
        _lib.ptr(plan["wave_ptr"]), _lib.ptr(plan["n_steps"]), plan["n_blocks"], R, _lib.ptr(x),
        x.shape[0], x.stride(0), _lib.ptr(y), y.stride(0), g.n_rows, 32, 0, 0, 32, 0, 32, 1.0,
        0, 32, _lib.ptr(sync), 0, _lib.stream_of(cuda)), "tiled")
    torch.cuda.synchronize()
    assert int(sync[_lib.TILED_SYNC_ERR_WORD]) != 0
    # the launch zeroes the word: the quad plan of the same operand runs clean and right
    qp = g.tiled_plan(rows_per_block=R, panel=4096, sub_panel=512)
    y2 = torch.empty_like(x)
    F.spmm_tiled_into(g, x, y2, qp)
    torch.cuda.synchronize()
    assert int(qp["sync"][_lib.TILED_SYNC_ERR_WORD]) == 0
    ref = oracle.spmm(g.row_ptr.cpu().numpy(), g.col.cpu().numpy(), g.val.cpu().numpy(),
                      x.cpu().numpy())
    assert np.array_equal(y2.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_csr_row_stats_native_equals_host(cuda):
    """gnnrec_csr_row_stats (the planner's longest row and block-edge bound, one kernel of this
    library instead of torch reductions) against the host numpy restatement, incl. empty rows,
    a ragged last block and block_rows <= 0."""
    rng = np.random.default_rng(3)
    g = CsrGraph.from_interactions(rng.integers(0, 5000, 80000), rng.zipf(1.7, 80000) % 3000,
                                   5000, 3000)
    gd = g.to(cuda)
    for R in (0, 1, 7, 1117, 10**6):
        assert gd.row_stats(R) == g.row_stats(R), R
    assert gd.max_degree() == int(np.diff(g.row_ptr.numpy()).max())
