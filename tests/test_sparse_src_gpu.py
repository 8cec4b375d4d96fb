"""Row-sparse input hop (gnnrec_spmm_sparse_src_f32): y = A^T x for an x that is zero outside
a few rows — the training backward's first hop (the BPR gradient of a batch, trainer.py:199-281
through lightgcn.py:88). Every reached output row must carry the dense hop's bits, the others
+0; the backward through it must equal the dense backward bit for bit."""
import numpy as np
import pytest
import torch

import oracle
from src.ops import CsrGraph, _lib, functional as F

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _graph(cuda, binary=True, seed=0, nu=30000, ni=20000, n=600000):
    rng = np.random.default_rng(seed)
    g = CsrGraph.from_interactions(rng.integers(0, nu, n), rng.integers(0, ni, n), nu, ni,
                                   binary=binary)
    return g.to(cuda), g


def _sparse_x(n, d, rows, cuda, seed=1):
    x = torch.zeros(n, d)
    x[rows] = torch.randn(len(rows), d, generator=torch.Generator().manual_seed(seed)) * 0.1
    return x.to(cuda)


def _dense_t(gd, x):
    """The dense hop over A^T through the row-parallel CSR kernel."""
    at = gd.t()
    y = torch.empty(at.n_rows, x.shape[1], device=x.device)
    F.TILED_HOP, was = False, F.TILED_HOP
    try:
        F.spmm_into(at, x, y)
    finally:
        F.TILED_HOP = was
    return y


@pytest.mark.parametrize("binary,d", [(True, 64), (False, 64), (True, 32), (True, 128)])
def test_sparse_src_equals_dense_hop(cuda, binary, d):
    gd, gh = _graph(cuda, binary=binary, seed=d)
    n = gd.shape[0]
    rows = np.sort(np.random.default_rng(d).choice(n, 300, replace=False))
    x = _sparse_x(n, d, rows, cuda)
    src = F.sparse_sources(gd, x)
    assert src is not None and src.rows.numel() == 300
    y = torch.full((n, d), float("nan"), device=cuda)
    F.spmm_sparse_src_into(src, x, y)
    ref = _dense_t(gd, x)
    assert torch.equal(y.view(torch.int32), ref.view(torch.int32))
    # and the oracle over the explicit transpose
    at = gd.t()
    rp, col, val = (t.cpu().numpy() for t in (at.row_ptr, at.col, at.val))
    np.testing.assert_array_equal(bits(y.cpu().numpy()), bits(oracle.spmm(rp, col, val,
                                                                          x.cpu().numpy())))


def test_sparse_src_edge_cases(cuda):
    gd, _ = _graph(cuda, seed=3, nu=3000, ni=2000, n=40000)
    n = gd.shape[0]
    # no non-zero row: all zeros
    x = torch.zeros(n, 64, device=cuda)
    src = F.sparse_sources(gd, x)
    y = torch.full_like(x, 7.0)
    F.spmm_sparse_src_into(src, x, y)
    assert torch.all(y == 0)
    # a NaN row is a source (NaN spreads to its neighbours as in the dense hop)
    x[5, 3] = float("nan")
    x[17] = 0.25
    src = F.sparse_sources(gd, x)
    assert src.rows.tolist() == [5, 17]
    F.spmm_sparse_src_into(src, x, y)
    ref = _dense_t(gd, x)
    assert torch.equal(y.view(torch.int32), ref.view(torch.int32))
    # a short pair bound fails loudly
    bad = F.SparseSrc(gd, src.rows, max(src.pairs - 1, 0))
    with pytest.raises(ValueError, match="max_pairs"):
        F.spmm_sparse_src_into(bad, x, y)
    # too many sources for the fraction: None (the caller keeps the masked hop)
    assert F.sparse_sources(gd, torch.ones(n, 64, device=cuda)) is None


@pytest.mark.parametrize("short", [1, 2, 10**9])
def test_sparse_src_short_bound_leaves_y_untouched(cuda, short):
    """Through the C ABI with a max_pairs below the sources' entries: the call fails with
    EINVAL and y is not written (the chain kernel sees the scatter's overflow flag and never
    reads the key slots the scatter skipped)."""
    gd, _ = _graph(cuda, seed=5, nu=3000, ni=2000, n=40000)
    n = gd.shape[0]
    rows = np.sort(np.random.default_rng(5).choice(n, 200, replace=False))
    x = _sparse_x(n, 64, rows, cuda)
    src = F.sparse_sources(gd, x)
    max_pairs = 0 if short == 10**9 else src.pairs // (2 * short) + 1   # 0: nothing to do
    y = torch.full((n, 64), 7.0, device=cuda)
    L = _lib.lib()
    nbytes = _lib.C.c_size_t(0)
    args = (_lib.ptr(gd.row_ptr), _lib.ptr(gd.col), _lib.ptr(gd.val), gd.n_rows, gd.shape[1],
            _lib.ptr(src.rows), src.rows.numel(), max_pairs, _lib.ptr(x), x.stride(0),
            _lib.ptr(y), y.stride(0), 64)
    stream = _lib.stream_of(gd.device)
    assert L.gnnrec_spmm_sparse_src_f32(*args, None, _lib.C.addressof(nbytes), stream) == 0
    work = torch.full((max(int(nbytes.value), 1),), 0xAB, dtype=torch.uint8, device=cuda)
    rc = L.gnnrec_spmm_sparse_src_f32(*args, _lib.ptr(work), _lib.C.addressof(nbytes), stream)
    torch.cuda.synchronize()
    if max_pairs:
        assert rc != 0 and b"max_pairs" in L.gnnrec_last_error()
    else:
        assert rc == 0
    assert torch.all(y == 7.0)


def test_backward_through_sparse_src_equals_dense_backward(cuda, monkeypatch):
    """lightgcn_backward's first hop on the row-sparse path (deferred schedule, tiled hops 2-3)
    gives the dense backward's bits."""
    gd, _ = _graph(cuda, seed=9, nu=40000, ni=30000, n=900000)
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    n = gd.shape[0]
    rows = np.sort(np.random.default_rng(4).choice(n, 1500, replace=False))
    g = _sparse_x(n, 64, rows, cuda, seed=2)
    calls = []
    orig = F.spmm_sparse_src_into
    monkeypatch.setattr(F, "spmm_sparse_src_into", lambda *a: (calls.append(1), orig(*a)))
    got = F.lightgcn_backward(gd, g, 3)
    assert calls, "the row-sparse hop was not used"
    ref = F.lightgcn_backward(gd, g, 3, masked_hops=0)          # dense hops only
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
