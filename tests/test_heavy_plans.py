"""Heavy-row segment plans of the GAT kernels (CsrGraph.heavy_plan, heavy_plan_by_column,
heavy_plan_panels) on the CPU: every heavy edge in exactly one segment, the merge's
row-grouped numbering (heavy_seg_ptr through seg_pos) lists each row's own segments, the
execution order is by first column, and panel-cut rows never cross a panel or exceed the
segment length."""
import numpy as np
import pytest

from src.ops import CsrGraph


def _zipf_graph(seed=23, nu=500, ni=400, n=40000):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, nu, n)
    i = np.minimum(rng.zipf(1.3, n) - 1, ni - 1)
    u = np.concatenate([u, np.arange(nu), rng.integers(0, nu, ni)])
    i = np.concatenate([i, rng.integers(0, ni, nu), np.arange(ni)])
    return CsrGraph.from_interactions(u, i, nu, ni)


@pytest.mark.parametrize("kind,args", [("column", (100, 9)), ("panel", (100, 9, 16, 2)),
                                       ("panel", (100, 1024, 64, 4)), ("panel", (50, 7, 8, 1))])
def test_heavy_plans_cover_every_heavy_edge_once(kind, args):
    g = _zipf_graph()
    plan = g.heavy_plan_by_column(*args) if kind == "column" else g.heavy_plan_panels(*args)
    rp, col = g.row_ptr.numpy(), g.col.numpy()
    heavy = plan["heavy_rows"].numpy()
    beg, end = plan["seg_beg"].numpy(), plan["seg_end"].numpy()
    srow, pos, ptr = plan["seg_row"].numpy(), plan["seg_pos"].numpy(), plan["heavy_seg_ptr"].numpy()
    assert np.all(end > beg)
    cov = np.zeros(g.nnz, np.int64)
    for b, e in zip(beg, end):
        cov[b:e] += 1
    hv = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in heavy])
    assert np.all(cov[hv] == 1) and cov.sum() == hv.size
    for h, r in enumerate(heavy):                      # the merge's numbering
        js = pos[ptr[h]:ptr[h + 1]]
        assert np.all(srow[js] == r) and np.all((beg[js] >= rp[r]) & (end[js] <= rp[r + 1]))
    assert np.all(np.diff(col[beg]) >= 0)              # execution order: first column
    if kind == "panel":
        _, seg_len, panel, min_pp = args
        deg = rp[heavy + 1] - rp[heavy]
        n_pan = -(-g.shape[1] // panel)
        cut = set(heavy[deg >= min_pp * n_pan].tolist())
        assert plan["n_cut_rows"] == len(cut) and len(cut) > 0
        for b, e, r in zip(beg, end, srow):
            if r in cut:
                assert col[b] // panel == col[e - 1] // panel and e - b <= seg_len


def test_tiled_plan_refuses_hub_rows(monkeypatch):
    """CsrGraph.tiled_plan refuses rows past TILED_PLAN_MAX_DEGREE instead of planning them
    serially (the SpMM never plans them: functional.TILED_MAX_DEGREE sends them to CSR)."""
    from src.ops import graph
    g = _zipf_graph()
    monkeypatch.setattr(graph, "TILED_PLAN_MAX_DEGREE", g.max_degree() - 1)
    with pytest.raises(ValueError, match="TILED_PLAN_MAX_DEGREE"):
        g.tiled_plan(rows_per_block=100, planner="host")
    monkeypatch.setattr(graph, "TILED_PLAN_MAX_DEGREE", g.max_degree())
    assert g.tiled_plan(rows_per_block=100, planner="host")["n_chunks"] > 0


def test_heavy_rows_longest_first_and_sliced_prefix():
    """The SpMM's heavy-row list (CsrGraph.heavy_rows) is longest first, and
    heavy_rows_longer(t, L) — the sliced rows gnnrec_spmm_csr_heavy_f32 takes as its first
    n_sliced entries — is exactly the prefix of rows longer than L."""
    g = _zipf_graph()
    deg = np.diff(g.row_ptr.numpy())
    for t in (8, 50, 100):
        rows = g.heavy_rows(t).numpy()
        assert set(rows) == set(np.nonzero(deg > t)[0])
        d = deg[rows]
        assert np.all(np.diff(d) <= 0)
        for L in (t, 2 * t, 10 * t, 10**9):
            n = g.heavy_rows_longer(t, L)
            assert n == int((deg > max(t, L)).sum()) if L >= t else True
            assert np.all(d[:n] > L) and np.all(d[n:] <= L)


def test_row_stats_host():
    """CsrGraph.row_stats on the host (the device path is gnnrec_csr_row_stats, pinned against
    it in test_tiled_plan_gpu.py): the longest row and the planner's block edge bound."""
    g = _zipf_graph()
    rp = g.row_ptr.numpy()
    assert g.row_stats()[0] == int(np.diff(rp).max()) == g.max_degree()
    for R in (1, 7, 333, 10**7):
        starts = np.arange(0, g.n_rows, R)
        want = int((rp[np.minimum(starts + R, g.n_rows)] - rp[starts]).max())
        assert g.row_stats(R) == (int(np.diff(rp).max()), want)


def test_heavy_knobs_by_operand():
    """functional.heavy_knobs: the round-6 sweeps' choices (small operands 256 / 2048 when the
    light rows run in the heavy launch, 128 / 1024 for masked hops, other widths or the
    two-launch flags; large ones 256 / 4096 at d <= 64 and 512 / 4096 above) and the module
    overrides."""
    from src.ops import _lib
    from src.ops import functional as F
    assert F.heavy_knobs(9746, 64) == (256, 2048)
    assert F.heavy_knobs(65536, 128) == (256, 2048)
    assert F.heavy_knobs(9746, 64, masked=True) == (128, 1024)
    assert F.heavy_knobs(9746, 16) == (128, 1024)
    saved_flags = F.CSR_FLAGS
    try:
        for fl in (_lib.CSR_TWO_LAUNCHES, _lib.CSR_FORK, _lib.CSR_LIGHT_THROUGHPUT):
            F.CSR_FLAGS = fl
            assert F.heavy_knobs(9746, 64) == (128, 1024)
    finally:
        F.CSR_FLAGS = saved_flags
    assert F.heavy_knobs(4_000_000, 64) == (256, 4096)
    assert F.heavy_knobs(4_000_000, 32) == (256, 4096)
    assert F.heavy_knobs(4_000_000, 128) == (512, 4096)
    saved = F.SPMM_HEAVY_THRESHOLD, F.SPMM_SLICE_LEN
    try:
        F.SPMM_HEAVY_THRESHOLD, F.SPMM_SLICE_LEN = 300, 0
        assert F.heavy_knobs(9746, 64) == (300, 0)
    finally:
        F.SPMM_HEAVY_THRESHOLD, F.SPMM_SLICE_LEN = saved


def test_light_form_flag_by_light_row_degree():
    """functional.light_form_flag: on operands above SMALL_OPERAND_ROWS rows the latency form
    of the row-parallel chain when the light rows average at most LIGHT_LATENCY_MAX_AVG
    neighbours (the heavy rows' edges excluded), else the caller's flags unchanged; small
    operands and an explicit form in CSR_FLAGS are left alone."""
    from src.ops import _lib
    from src.ops import functional as F
    rng = np.random.default_rng(5)
    nu, ni = 60_000, 20_000
    sparse = CsrGraph.from_interactions(rng.integers(0, nu, 200_000), rng.integers(0, ni, 200_000),
                                        nu, ni)
    assert sparse.n_rows > F.SMALL_OPERAND_ROWS
    assert sparse.light_avg_degree(0) == pytest.approx(sparse.nnz / sparse.n_rows)
    rp = sparse.row_ptr.numpy()
    deg = np.diff(rp)
    t = int(np.sort(deg)[-10]) - 1   # a handful of heavy rows
    light = deg[deg <= t]
    assert sparse.light_avg_degree(t) == pytest.approx(light.sum() / light.size)
    assert F.light_form_flag(sparse, t) == _lib.CSR_LIGHT_LATENCY
    dense = CsrGraph.from_interactions(rng.integers(0, nu, 1_200_000),
                                       rng.integers(0, 1_000, 1_200_000), nu, 1_000)
    assert dense.light_avg_degree(0) > F.LIGHT_LATENCY_MAX_AVG
    assert F.light_form_flag(dense, 0) == 0
    saved = F.CSR_FLAGS
    try:
        F.CSR_FLAGS = _lib.CSR_LIGHT_THROUGHPUT
        assert F.light_form_flag(sparse, t) == _lib.CSR_LIGHT_THROUGHPUT
        F.CSR_FLAGS = _lib.CSR_FORK
        assert F.light_form_flag(sparse, t) == _lib.CSR_FORK | _lib.CSR_LIGHT_LATENCY
    finally:
        F.CSR_FLAGS = saved
    small = CsrGraph.from_interactions(rng.integers(0, 500, 5_000), rng.integers(0, 500, 5_000),
                                       500, 500)
    assert F.light_form_flag(small, 0) == F.CSR_FLAGS


def test_gat_split_knobs_by_operand():
    """functional.gat_knobs / gat_train_knobs: the GAT heavy-row split on small operands
    (<= SMALL_OPERAND_ROWS rows: 64 / 32 forward, 128 / 64 training) and large ones (2048 /
    1024), and the module overrides."""
    from src.ops import functional as F
    assert F.gat_knobs(9746) == (64, 32) and F.gat_knobs(20_000_000) == (2048, 1024)
    assert F.gat_train_knobs(9746) == (128, 64) and F.gat_train_knobs(4_000_000) == (2048, 1024)
    saved = (F.GAT_HEAVY_THRESHOLD, F.GAT_SEGMENT, F.GAT_TRAIN_HEAVY_THRESHOLD,
             F.GAT_TRAIN_SEGMENT)
    try:
        F.GAT_HEAVY_THRESHOLD, F.GAT_SEGMENT = 0, 7
        assert F.gat_knobs(9746) == (0, 7) and F.gat_knobs(20_000_000) == (0, 7)
        F.GAT_TRAIN_HEAVY_THRESHOLD = 300
        assert F.gat_train_knobs(9746) == (300, 64)
    finally:
        (F.GAT_HEAVY_THRESHOLD, F.GAT_SEGMENT, F.GAT_TRAIN_HEAVY_THRESHOLD,
         F.GAT_TRAIN_SEGMENT) = saved
