"""Factored column-ordered plans (ABI 8, gnnrec_tiled_plan_factor): a slot carries its
column's 1-byte degree class instead of its fp32 value, and the hop forms the value as
fl(row_factor[r] * class_table[k]) — the product the operand's builder stored
(graph_builder.py:119-126: fl(dis_r * dis_c) for a binary interaction graph). The hop through a
factored plan must give the same bits as the oracle and as the explicit-value plan; an operand
whose values are not such products must keep its values."""
import numpy as np
import pytest
import torch

import oracle
from src.ops import CsrGraph, _lib, functional as F
from src.ops import graph as G

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _binary(nu, ni, n, seed, device):
    rng = np.random.default_rng(seed)
    g = CsrGraph.from_interactions(rng.integers(0, nu, n), rng.integers(0, ni, n), nu, ni,
                                   binary=True)
    return g.to(device), (g.row_ptr.numpy(), g.col.numpy(), g.val.numpy())


@pytest.mark.parametrize("R,panel,sub,d", [(1117, 49152, 4096, 64), (37, 512, 64, 32),
                                           (1232, 8192, 1024, 128), (1, 64, 0, 64)])
def test_factored_plan_bit_exact(cuda, R, panel, sub, d):
    g, (rp, col, val) = _binary(30000, 20000, 700000, R, cuda)
    plan = g.tiled_plan(rows_per_block=R, panel=panel, sub_panel=sub)
    assert "cls" in plan and "val" not in plan, "a binary operand's plan must factor"
    assert plan["n_classes"] <= _lib.TILED_MAX_CLASSES
    x = torch.randn(g.shape[0], d, generator=torch.Generator().manual_seed(d)) * 0.1
    ref = bits(oracle.spmm(rp, col, val, x.numpy()))
    y = torch.full((g.shape[0], d), float("nan"), device=cuda)
    F.spmm_tiled_into(g, x.to(cuda), y, plan)
    np.testing.assert_array_equal(bits(y.cpu().numpy()), ref)
    # the explicit-value plan of the same operand: the same bits
    g2 = CsrGraph(g.row_ptr, g.col, g.val, g.shape, g.n_users, g.n_items, g.symmetric)
    G.TILED_FACTOR, was = False, G.TILED_FACTOR
    try:
        plain = g2.tiled_plan(rows_per_block=R, panel=panel, sub_panel=sub)
    finally:
        G.TILED_FACTOR = was
    assert "val" in plain and "cls" not in plain
    y2 = torch.full_like(y, float("nan"))
    F.spmm_tiled_into(g2, x.to(cuda), y2, plain)
    assert torch.equal(y.view(torch.int32), y2.view(torch.int32))


def test_factored_lightgcn_deferred_mean_bit_exact(cuda, monkeypatch):
    """The model path (deferred layer mean: ACC_INIT | ADD | X epilogues) through factored
    plans equals the oracle's LightGCN bit for bit."""
    g, (rp, col, val) = _binary(40000, 30000, 900000, 7, cuda)
    x = torch.randn(g.shape[0], 64, generator=torch.Generator().manual_seed(5)) * 0.1
    ref = bits(oracle.lightgcn(rp, col, val, x.numpy(), 3))
    monkeypatch.setattr(F, "TILED_MIN_ROWS", 0)
    monkeypatch.setattr(F, "TILED_MIN_TABLE_BYTES", 0)
    plan = F.tiled_plan_for(g, x.to(cuda))
    assert plan is not None and "cls" in plan
    out, _ = F.lightgcn_forward(g, x.to(cuda), 3)
    np.testing.assert_array_equal(bits(out.cpu().numpy()), ref)


def test_non_product_values_keep_explicit_plan(cuda):
    """Duplicate pairs (multiplicity 2, not a binary graph) or values edited after the build:
    gnnrec_tiled_plan_factor finds mismatches and the plan keeps its values — same bits."""
    rng = np.random.default_rng(3)
    u, i = rng.integers(0, 3000, 60000), rng.integers(0, 2500, 60000)
    dup = CsrGraph.from_interactions(u, i, 3000, 2500).to(cuda)          # multiplicities
    assert "val" in dup.tiled_plan(rows_per_block=300, panel=4096)
    g, (rp, col, val) = _binary(3000, 2500, 60000, 4, cuda)
    val2 = val.copy()
    val2[12345] = np.nextafter(val2[12345], np.float32(1))               # one ulp off
    g2 = CsrGraph(g.row_ptr, g.col, torch.from_numpy(val2).to(cuda), g.shape, 3000, 2500)
    plan = g2.tiled_plan(rows_per_block=300, panel=4096)
    assert "val" in plan and "cls" not in plan
    x = torch.randn(g.shape[0], 32, device=cuda) * 0.1
    y = torch.empty_like(x)
    F.spmm_tiled_into(g2, x, y, plan)
    np.testing.assert_array_equal(bits(y.cpu().numpy()),
                                  bits(oracle.spmm(rp, col, val2, x.cpu().numpy())))


def test_factor_kernel_counts_mismatches(cuda):
    """gnnrec_tiled_plan_factor through the C ABI: zero mismatches for the operand's own
    factors, one per perturbed slot value."""
    g, _ = _binary(5000, 4000, 100000, 9, cuda)
    # the planner's chunk-major arrays (what the factor kernel reads; a quad-layout build
    # interleaves the plan only after factoring)
    plan = g._tiled_plan_device(200, 2048, 256)
    rowf, col_class, table = g.degree_factors()
    L = _lib.lib()

    def run(val):
        cls = torch.zeros(plan["slot"].numel(), dtype=torch.uint8, device=cuda)
        bad = torch.zeros(1, dtype=torch.int32, device=cuda)
        _lib.check(L.gnnrec_tiled_plan_factor(
            _lib.ptr(plan["slot"]), _lib.ptr(val), _lib.ptr(plan["hdr"]),
            _lib.ptr(plan["wave_ptr"]), plan["n_blocks"], 200, g.n_rows, g.shape[1],
            _lib.ptr(rowf), _lib.ptr(col_class), _lib.ptr(table), table.numel(), _lib.ptr(cls),
            _lib.ptr(bad), _lib.stream_of(cuda)), "factor")
        return int(bad), cls

    nbad, cls = run(plan["val"])
    assert nbad == 0
    real = (plan["slot"] & 2047) < 200
    assert not bool((cls[~real] != 0).any())          # padding and tail slots: class 0
    v = plan["val"].clone()
    idx = torch.nonzero(real).flatten()[:3]
    v[idx] = v[idx] * 2
    assert run(v)[0] == 3


def test_degree_factors_limits(cuda):
    """More than TILED_MAX_CLASSES distinct degrees, or a non-square operand: no factors."""
    n = 600
    rows = np.repeat(np.arange(n), np.arange(1, n + 1))          # degrees 1..600
    cols = np.concatenate([np.arange(k) for k in range(1, n + 1)])
    rp = np.concatenate([[0], np.cumsum(np.arange(1, n + 1))]).astype(np.int64)
    g = CsrGraph(torch.from_numpy(rp), torch.from_numpy(cols.astype(np.int32)),
                 torch.ones(rows.size), (n, n)).to(cuda)
    assert g.degree_factors() is None
    rect = CsrGraph(torch.tensor([0, 1, 2]), torch.tensor([0, 3], dtype=torch.int32),
                    torch.ones(2), (2, 5)).to(cuda)
    assert rect.degree_factors() is None
